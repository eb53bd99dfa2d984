"""The fused pre-smoothing pass (gs_jacobi_sweep2_restrict: two sweeps, the residual of their result
and the full weighting in one kernel) against the two-pass path it replaces at level 0 of a 2+2
V-cycle — gs_jacobi_sweep2_norm followed by gs_residual_restrict (CpuSolver.cpp:94-99) — bit for bit
on v'' and the coarse f (whole padded arrays), the norm of f - A v to 1e-12 (block order differs).
Shapes hit every tile edge: one and several x-waves, rows not a multiple of 64, ragged 4-row tiles,
odd plane counts (the last fine plane has no coarse plane over it), one and several z-chunks."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402

SHAPES = [(2, 2, 2), (3, 2, 5), (7, 6, 5), (33, 4, 3), (64, 64, 64), (65, 10, 19), (100, 9, 130), (127, 13, 40),
          (128, 8, 9), (257, 6, 10), (500, 7, 9), (511, 37, 23), (512, 5, 9), (512, 64, 66), (300, 3, 517)]


def k():
    assert torch.cuda.is_available()
    return gsv.kernels()


def st():
    return torch.cuda.current_stream().cuda_stream


def ok(rc):
    assert rc == 0, k().gs_strerror(rc).decode()


def rand_full(rng, nx, ny, nz, scale):
    a = np.zeros((nx + 2, ny + 2, nz + 2))
    a[1:nx + 1, 1:ny + 1, 1:nz + 1] = rng.uniform(-scale, scale, (nx, ny, nz))
    return a


def norm(p):
    return float(torch.sqrt(p.sum()).item())


@pytest.mark.parametrize("shape", SHAPES)
def test_pair_restrict_equals_pair_then_restrict(shape):
    S = gsv.Stencil().to_abi()
    rng = np.random.default_rng(abs(hash(shape)) % 2**32)
    nx, ny, nz = shape
    h = 1.0 / (ny + 1)
    v0, f0 = rand_full(rng, nx, ny, nz, 1.0), rand_full(rng, nx, ny, nz, 100.0)
    v, f = DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0)
    out1, out2 = DevField(nx, ny, nz, fill=0.0), DevField(nx, ny, nz, fill=0.0)
    cn = (nx // 2, ny // 2, nz // 2)
    c1, c2, c2b = DevField(*cn, fill=-7.0), DevField(*cn, fill=-7.0), DevField(*cn, fill=-7.0)
    L, CL = v.level(h), c1.level(2 * h)
    assert gsv.diag().gs_jacobi_sweep2_restrict_supported(C.byref(S), C.byref(L), C.byref(CL), 0) == 1
    n1 = k().gs_jacobi_sweep2_num_partials(C.byref(S), C.byref(L), 0)
    n2 = gsv.diag().gs_jacobi_sweep2_restrict_num_partials(C.byref(S), C.byref(L), C.byref(CL))
    assert n1 > 0 and n2 > 0
    p1 = torch.zeros(n1, dtype=torch.float64, device="cuda")
    p2 = torch.zeros(n2, dtype=torch.float64, device="cuda")
    ok(k().gs_jacobi_sweep2_norm(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, out1.ptr, f.ptr, None, 0, 0,
                                 p1.data_ptr(), st()))
    ok(k().gs_residual_restrict(C.byref(S), C.byref(L), 0, 1.0, out1.ptr, f.ptr, None, c1.ptr, None, C.byref(CL),
                                st()))
    ok(gsv.diag().gs_jacobi_sweep2_restrict(C.byref(S), C.byref(L), 0.8, v.ptr, out2.ptr, f.ptr, p2.data_ptr(), c2.ptr,
                                     c2b.ptr, C.byref(CL), st()))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out2.to_xyz(), out1.to_xyz())
    np.testing.assert_array_equal(c2.to_xyz(), c1.to_xyz())
    np.testing.assert_array_equal(c2b.to_xyz(), c1.to_xyz())
    a, b = norm(p1), norm(p2)
    assert abs(a - b) <= 1e-12 * a, (a, b)


def test_pair_restrict_supported_cases():
    S = gsv.Stencil().to_abi()
    v, c = DevField(64, 16, 16), DevField(32, 8, 8)
    L, CL = v.level(1.0 / 17), c.level(2.0 / 17)
    assert gsv.diag().gs_jacobi_sweep2_restrict_supported(C.byref(S), C.byref(L), C.byref(CL), 0) == 1
    for mode in (1, 2):  # LINEAR only
        assert gsv.diag().gs_jacobi_sweep2_restrict_supported(C.byref(S), C.byref(L), C.byref(CL), mode) == 0
    wide, cw = DevField(513, 4, 4), DevField(256, 2, 2)  # rows > 512 points
    assert gsv.diag().gs_jacobi_sweep2_restrict_supported(C.byref(S), C.byref(wide.level(0.2)), C.byref(cw.level(0.4)), 0) == 0
    other = DevField(32, 8, 9)  # coarse not fine / 2
    assert gsv.diag().gs_jacobi_sweep2_restrict_supported(C.byref(S), C.byref(L), C.byref(other.level(0.1)), 0) == 0
    gen = gsv.Stencil()
    gen.values = [6.5, -1, -1, -1, -1, -1, -1.5]  # not the unit-neighbour stencil
    assert gsv.diag().gs_jacobi_sweep2_restrict_supported(C.byref(gen.to_abi()), C.byref(L), C.byref(CL), 0) == 0


@pytest.mark.parametrize("shape", SHAPES + [(256, 256, 64), (255, 31, 17)])
def test_zero_pair_restrict_equals_zero_pair_then_restrict(shape):
    """gs_smooth2_restrict_zero (diagnostics library: a coarse level's first step from v = 0 in one pass, r04) against
    the zero-iterate pair (v_in NULL) followed by gs_residual_restrict, bit for bit on v'' and the coarse f."""
    S = gsv.Stencil().to_abi()
    rng = np.random.default_rng(abs(hash(shape)) % 2**32 + 5)
    nx, ny, nz = shape
    h = 1.0 / (ny + 1)
    f = DevField(nx, ny, nz).from_xyz(rand_full(rng, nx, ny, nz, 100.0))
    out1, out2 = DevField(nx, ny, nz, fill=0.0), DevField(nx, ny, nz, fill=0.0)
    cn = (nx // 2, ny // 2, nz // 2)
    c1, c2 = DevField(*cn, fill=-7.0), DevField(*cn, fill=-7.0)
    L, CL = f.level(h), c1.level(2 * h)
    assert gsv.diag().gs_smooth2_restrict_zero_supported(C.byref(S), C.byref(L), C.byref(CL), 0) == 1
    ok(k().gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, None, out1.ptr, f.ptr, None, 0, 0, st()))
    ok(k().gs_residual_restrict(C.byref(S), C.byref(L), 0, 1.0, out1.ptr, f.ptr, None, c1.ptr, None, C.byref(CL),
                                st()))
    ok(gsv.diag().gs_smooth2_restrict_zero(C.byref(S), C.byref(L), 0.8, out2.ptr, f.ptr, c2.ptr, C.byref(CL), st()))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out2.to_xyz(), out1.to_xyz())
    np.testing.assert_array_equal(c2.to_xyz(), c1.to_xyz())


def test_zero_pair_restrict_refusals():
    S = gsv.Stencil().to_abi()
    v, c = DevField(64, 16, 16), DevField(32, 8, 8)
    L, CL = v.level(1.0 / 17), c.level(2.0 / 17)
    assert gsv.diag().gs_smooth2_restrict_zero_supported(C.byref(S), C.byref(L), C.byref(CL), 0) == 1
    for mode in (1, 2):  # LINEAR only
        assert gsv.diag().gs_smooth2_restrict_zero_supported(C.byref(S), C.byref(L), C.byref(CL), mode) == 0
    wide, cw = DevField(513, 4, 4), DevField(256, 2, 2)  # rows > 512 points
    assert gsv.diag().gs_smooth2_restrict_zero_supported(C.byref(S), C.byref(wide.level(0.2)), C.byref(cw.level(0.4)), 0) == 0
    gen = gsv.Stencil()
    gen.values = [6.5, -1, -1, -1, -1, -1, -1.5]  # not the unit-neighbour stencil
    assert gsv.diag().gs_smooth2_restrict_zero_supported(C.byref(gen.to_abi()), C.byref(L), C.byref(CL), 0) == 0
    rc = gsv.diag().gs_smooth2_restrict_zero(C.byref(gen.to_abi()), C.byref(L), 0.8, v.ptr, v.ptr, c.ptr, C.byref(CL), st())
    assert rc == gsv._abi.GS_EINVAL
