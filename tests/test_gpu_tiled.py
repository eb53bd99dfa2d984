"""The small-level tiled kernels (LINEAR and NEWTON) (gs_smooth2_restrict_tiled, gs_prolong_smooth2_tiled: one launch of
LDS tiles that recompute their halos) against the unfused sequences they replace, bit for bit:
two gs_jacobi_sweep + gs_residual_restrict (CpuSolver.cpp:88-99: jacobi(pre = 2), compResidual,
restrict; v = 0 first for the zero-iterate form, CpuSolver.cpp:100-101) and gs_prolong_add + two
gs_jacobi_sweep (CpuSolver.cpp:127-134). Shapes cover whole and ragged 8^3 tiles, odd extents (the
coarse level is fine / 2 per axis), one-tile and degenerate levels, and a non-unit stencil."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402

from test_gpu_sweep2 import k, ok, rand_full, st  # noqa: E402

SHAPES = [(2, 2, 2), (3, 5, 2), (8, 8, 8), (9, 9, 9), (15, 15, 15), (16, 16, 16), (17, 9, 12), (31, 32, 33),
          (32, 32, 32), (64, 64, 64), (40, 8, 24), (7, 30, 11)]
STENCILS = {"unit": gsv.Stencil(), "aniso": gsv.Stencil([4, -1, -1, -0.5, -0.5, -0.5, -0.5])}


def sweeps(S, L, v, f, n, zero, mode=0, w=None):
    """n gs_jacobi_sweep calls; returns the field holding the result (v is overwritten)."""
    alt = DevField(L.nx, L.ny, L.nz)
    src = None if zero else v.ptr
    wp = w.ptr if w is not None else None
    for i in range(n):
        ok(k().gs_jacobi_sweep(C.byref(S), C.byref(L), mode, 0.8, 1.0, src if i == 0 else v.ptr, alt.ptr, f.ptr, wp,
                               st()))
        v, alt = alt, v
        src = v.ptr
    return v


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("stencil", sorted(STENCILS))
@pytest.mark.parametrize("zero", [True, False])
@pytest.mark.parametrize("shape", SHAPES)
def test_smooth2_restrict_tiled(shape, zero, stencil, mode):
    S = STENCILS[stencil].to_abi()
    rng = np.random.default_rng(abs(hash((shape, zero, stencil, mode))) % 2**32)
    nx, ny, nz = shape
    cd = [x // 2 for x in shape]
    h = 1.0 / (ny + 1)
    v0, f0, w0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0), rand_full(rng, *shape, 0.5)
    L = DevField(nx, ny, nz).level(h)
    assert k().gs_tiled_supported(C.byref(S), C.byref(L), mode) == 1
    w = DevField(nx, ny, nz).from_xyz(w0) if mode == 2 else None
    wp = w.ptr if w is not None else None
    # reference: two sweeps, then residual + restriction
    v, f = DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0)
    vr = sweeps(S, L, v, f, 2, zero, mode, w)
    cref = DevField(*cd)
    Lc = cref.level(2 * h)
    ok(k().gs_residual_restrict(C.byref(S), C.byref(L), mode, 1.0, vr.ptr, f.ptr, wp, cref.ptr, None, C.byref(Lc),
                                st()))
    # tiled
    v2, out, cgot = DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz), DevField(*cd)
    ok(k().gs_smooth2_restrict_tiled(C.byref(S), C.byref(L), mode, 0.8, 1.0, None if zero else v2.ptr, out.ptr, f.ptr,
                                     wp, cgot.ptr, C.byref(Lc), st()))
    want = vr.to_xyz()
    got = out.to_xyz()
    np.testing.assert_array_equal(got[1:-1, 1:-1, 1:-1], want[1:-1, 1:-1, 1:-1])
    np.testing.assert_array_equal(cgot.to_xyz(), cref.to_xyz())


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("stencil", sorted(STENCILS))
@pytest.mark.parametrize("shape", SHAPES)
def test_prolong_smooth2_tiled(shape, stencil, mode):
    S = STENCILS[stencil].to_abi()
    rng = np.random.default_rng(abs(hash((shape, stencil, 7, mode))) % 2**32)
    nx, ny, nz = shape
    cd = [x // 2 for x in shape]
    h = 1.0 / (ny + 1)
    v0, f0, c0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0), rand_full(rng, *cd)
    w0 = rand_full(rng, *shape, 0.5)
    L = DevField(nx, ny, nz).level(h)
    w = DevField(nx, ny, nz).from_xyz(w0) if mode == 2 else None
    v, f, c = DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0), DevField(*cd).from_xyz(c0)
    Lc = c.level(2 * h)
    ok(k().gs_prolong_add(c.ptr, None, C.byref(Lc), v.ptr, C.byref(L), st()))
    want = sweeps(S, L, v, f, 2, False, mode, w).to_xyz()
    v2, out = DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz)
    ok(k().gs_prolong_smooth2_tiled(C.byref(S), C.byref(L), mode, 0.8, 1.0, v2.ptr, c.ptr, C.byref(Lc), out.ptr, f.ptr,
                                    w.ptr if w is not None else None, st()))
    np.testing.assert_array_equal(out.to_xyz()[1:-1, 1:-1, 1:-1], want[1:-1, 1:-1, 1:-1])
    np.testing.assert_array_equal(v2.to_xyz(), v0)  # the input iterate is left as it was


def test_tiled_rejects():
    S = gsv.Stencil().to_abi()
    L = DevField(16, 16, 16).level(1 / 17.0)
    assert k().gs_tiled_supported(C.byref(S), C.byref(L), 1) == 0  # NONLINEAR (FAS) keeps the general path
    assert k().gs_tiled_supported(C.byref(S), C.byref(L), 2) == 1
    perm = gsv.Stencil([-1, -1, 6, -1, -1, -1, -1], [(0, -1, 0), (1, 0, 0), (0, 0, 0), (0, 0, -1), (-1, 0, 0),
                                                     (0, 1, 0), (0, 0, 1)]).to_abi()
    assert k().gs_tiled_supported(C.byref(perm), C.byref(L), 0) == 0
    slab = DevField(16, 16, 16).level(1 / 17.0, z0=16)
    assert k().gs_tiled_supported(C.byref(S), C.byref(slab), 0) == 0
    f, out, c = DevField(16, 16, 16), DevField(16, 16, 16), DevField(7, 8, 8)  # coarse != fine / 2
    assert k().gs_smooth2_restrict_tiled(C.byref(S), C.byref(L), 0, 0.8, 1.0, None, out.ptr, f.ptr, None, c.ptr,
                                         C.byref(c.level(1 / 9.0)), st()) == gsv._abi.GS_EINVAL
    c2 = DevField(8, 8, 8)  # NEWTON without newtonV
    assert k().gs_smooth2_restrict_tiled(C.byref(S), C.byref(L), 2, 0.8, 1.0, None, out.ptr, f.ptr, None, c2.ptr,
                                         C.byref(c2.level(1 / 9.0)), st()) == gsv._abi.GS_EINVAL
