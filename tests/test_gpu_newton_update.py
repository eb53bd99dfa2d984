"""findError's newtonV += v fused into the compF that follows it (gs_newton_F_update, NewtonSolver.cpp:105-107
then :48-81). The one-pass kernel must equal gs_axpy(w, e, 1) + gs_newton_F bit for bit: w_out over the whole
padded array, f on the interior, every per-block partial and the finished norm. Inside whole Newton solves
the driver's fused path (default) must leave every level's v / newtonV and the residual history identical
to the two-pass path (GS_NO_NEWTON_FUSED_UPDATE), which test_gpu_solver.py pins to the reference."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def k():
    assert torch.cuda.is_available(), "GPU tests need a GPU (no CPU fallback exists)"
    return gsv.kernels()


def stream():
    return torch.cuda.current_stream().cuda_stream


def ok(rc):
    assert rc == 0, k().gs_strerror(rc).decode()


def interior_random(rng, dims, scale):
    a = np.zeros(tuple(d + 2 for d in dims))
    a[1:-1, 1:-1, 1:-1] = rng.uniform(-scale, scale, dims)
    return a


@pytest.mark.parametrize("dims,values", [
    ((512, 128, 64), (6, -1, -1, -1, -1, -1, -1)),
    ((300, 150, 71), (6, -1, -1, -1, -1, -1, -1)),  # ragged x-blocks and rows, odd plane count
    ((260, 130, 130), (6.5, -1.25, -0.75, -1, -1, -1.5, -0.5)),  # non-unit stencil
    ((512, 64, 130), (6, -1, -1, -1, -1, -1, -1)),
])  # (the register-blocked pass needs >= 1024 blocks of 4-plane chunks)
def test_fused_update_equals_axpy_then_compF(dims, values):
    S = gsv.Stencil(list(values), list(gsv.CANONICAL_OFFSETS)).to_abi()
    rng = np.random.default_rng(sum(dims))
    w0, e0 = interior_random(rng, dims, 0.7), interior_random(rng, dims, 0.3)
    F0 = rng.uniform(-2, 2, tuple(d + 2 for d in dims))  # NONLINEAR rhs: the whole padded array
    h = 1.0 / (dims[1] + 1)
    gamma = 1.0
    w, e, F = DevField(*dims).from_xyz(w0), DevField(*dims).from_xyz(e0), DevField(*dims).from_xyz(F0)
    L = w.level(h)
    assert k().gs_newton_F_update_supported(C.byref(S), C.byref(L)) == 1
    n = k().gs_residual_num_partials(C.byref(S), C.byref(L))
    # reference sequence: newtonV += v over the span, then compF
    w_ref = DevField(*dims).from_xyz(w0)
    f_ref = DevField(*dims, fill=np.nan)
    p_ref = torch.zeros(n, dtype=torch.float64, device="cuda")
    ok(k().gs_axpy(w_ref.ptr, e.ptr, 1.0, w_ref.span, stream()))
    ok(k().gs_newton_F(C.byref(S), C.byref(L), gamma, w_ref.ptr, F.ptr, f_ref.ptr, p_ref.data_ptr(), stream()))
    # fused: w_out starts as zeros (the driver's vAlt), f as NaN outside what the pass writes
    w_out = DevField(*dims)
    f_got = DevField(*dims, fill=np.nan)
    p_got = torch.full((n,), np.nan, dtype=torch.float64, device="cuda")
    ok(k().gs_newton_F_update(C.byref(S), C.byref(L), gamma, w.ptr, e.ptr, F.ptr, w_out.ptr, f_got.ptr,
                              p_got.data_ptr(), stream()))
    np.testing.assert_array_equal(w_out.to_xyz(), w_ref.to_xyz())
    np.testing.assert_array_equal(f_got.to_xyz()[1:-1, 1:-1, 1:-1], f_ref.to_xyz()[1:-1, 1:-1, 1:-1])
    np.testing.assert_array_equal(p_got.cpu().numpy(), p_ref.cpu().numpy())
    # the operands are read only
    np.testing.assert_array_equal(w.to_xyz(), w0)
    np.testing.assert_array_equal(e.to_xyz(), e0)


@pytest.mark.parametrize("dims,values", [
    ((512, 128, 64), (6, -1, -1, -1, -1, -1, -1)),   # even extents: the last chunk runs one step past the level
    ((300, 150, 71), (6, -1, -1, -1, -1, -1, -1)),   # ragged x-blocks and rows, odd plane count
    ((301, 151, 129), (6, -1, -1, -1, -1, -1, -1)),  # odd everywhere: coarse n/2 leaves the last fine line unread
    ((260, 130, 130), (6.5, -1.25, -0.75, -1, -1, -1.5, -0.5)),  # non-unit stencil
])
def test_fused_update_restrict_equals_update_then_restrict(dims, values):
    """gs_newton_F_update_restrict = gs_newton_F_update followed by gs_restrict of the new newtonV onto the next
    level (NewtonSolver.cpp:88-92), bit for bit: w_out, f, the partials and every coarse point."""
    S = gsv.Stencil(list(values), list(gsv.CANONICAL_OFFSETS)).to_abi()
    rng = np.random.default_rng(sum(dims) + 1)
    w0, e0 = interior_random(rng, dims, 0.7), interior_random(rng, dims, 0.3)
    F0 = rng.uniform(-2, 2, tuple(d + 2 for d in dims))
    h = 1.0 / (dims[1] + 1)
    cd = tuple(d // 2 for d in dims)
    w, e, F = DevField(*dims).from_xyz(w0), DevField(*dims).from_xyz(e0), DevField(*dims).from_xyz(F0)
    L = w.level(h)
    Lc = DevField(*cd).level(1.0 / (cd[1] + 1))
    assert k().gs_newton_F_update_restrict_supported(C.byref(S), C.byref(L), C.byref(Lc)) == 1
    n = k().gs_residual_num_partials(C.byref(S), C.byref(L))
    w_ref, f_ref = DevField(*dims), DevField(*dims, fill=np.nan)
    c_ref = DevField(*cd)
    p_ref = torch.zeros(n, dtype=torch.float64, device="cuda")
    ok(k().gs_newton_F_update(C.byref(S), C.byref(L), 1.0, w.ptr, e.ptr, F.ptr, w_ref.ptr, f_ref.ptr,
                              p_ref.data_ptr(), stream()))
    ok(k().gs_restrict(w_ref.ptr, C.byref(L), c_ref.ptr, C.byref(c_ref.level(Lc.h)), stream()))
    w_got, f_got = DevField(*dims), DevField(*dims, fill=np.nan)
    c_got = DevField(*cd)  # (the pass writes the coarse interior only, as gs_restrict does)
    p_got = torch.full((n,), np.nan, dtype=torch.float64, device="cuda")
    ok(k().gs_newton_F_update_restrict(C.byref(S), C.byref(L), 1.0, w.ptr, e.ptr, F.ptr, w_got.ptr, f_got.ptr,
                                       p_got.data_ptr(), c_got.ptr, C.byref(c_got.level(Lc.h)), stream()))
    np.testing.assert_array_equal(w_got.to_xyz(), w_ref.to_xyz())
    np.testing.assert_array_equal(f_got.to_xyz()[1:-1, 1:-1, 1:-1], f_ref.to_xyz()[1:-1, 1:-1, 1:-1])
    np.testing.assert_array_equal(p_got.cpu().numpy(), p_ref.cpu().numpy())
    np.testing.assert_array_equal(c_got.to_xyz(), c_ref.to_xyz())


def test_fused_update_refuses_what_it_cannot_run():
    S = gsv.Stencil([6, -1, -1, -1, -1, -1, -1], list(gsv.CANONICAL_OFFSETS)).to_abi()
    w = DevField(8, 8, 8)
    L = w.level(1.0 / 9)
    assert k().gs_newton_F_update_supported(C.byref(S), C.byref(L)) == 0  # tiny level: the 1-point pass
    x, y, z = DevField(8, 8, 8), DevField(8, 8, 8), DevField(8, 8, 8)
    assert k().gs_newton_F_update(C.byref(S), C.byref(L), 1.0, w.ptr, x.ptr, x.ptr, y.ptr, z.ptr, None,
                                  stream()) == gsv._abi.GS_EINVAL
    big, b2, b3 = DevField(512, 128, 64), DevField(512, 128, 64), DevField(512, 128, 64)
    Lb = big.level(1.0 / 129)
    assert k().gs_newton_F_update_supported(C.byref(S), C.byref(Lb)) == 1
    # w_out aliasing an operand is refused
    assert k().gs_newton_F_update(C.byref(S), C.byref(Lb), 1.0, big.ptr, b2.ptr, b3.ptr, big.ptr, b3.ptr, None,
                                  stream()) == gsv._abi.GS_EINVAL


class env:
    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.old = {k_: os.environ.get(k_) for k_ in self.kw}
        os.environ.update({k_: str(v) for k_, v in self.kw.items()})

    def __exit__(self, *a):
        for k_, v in self.old.items():
            if v is None:
                del os.environ[k_]
            else:
                os.environ[k_] = v


def solve(params):
    with gsv.HipGridData(params) as g:
        hist = gsv.NewtonSolver.solve(g)
        fields = {(l, n): g.field(l, n) for l in range(g.numLevels()) for n in ("v", "newtonV", "f")}
    return hist, fields


@pytest.mark.parametrize("dims,pre,post,iters", [((255, 127, 127), 2, 2, 3), ((256, 128, 128), 2, 2, 3),
                                                 ((300, 150, 71), 3, 1, 2),
                                                 ((64, 64, 64), 2, 2, 2)])  # 64^3: no fused pass
def test_newton_solve_fused_update_bit_identical(dims, pre, post, iters):
    p = gsv.GridParams(maxiter=iters, tol=0.0, gridDim=dims, mode=gsv.GS_NEWTON, preSmoothing=pre,
                       postSmoothing=post)
    with env(GS_NO_NEWTON_FUSED_UPDATE=1):
        h_ref, f_ref = solve(p)
    h_got, f_got = solve(p)
    np.testing.assert_array_equal(h_got, h_ref)  # (power-of-two sizes diverge: inf / NaN compare equal here)
    for key, a in f_ref.items():
        np.testing.assert_array_equal(f_got[key], a, err_msg=str(key))


@pytest.mark.parametrize("n,doff,soff", [(1 << 20, 0, 0), (1000003, 0, 0), (4097, 1, 1), (4096, 1, 1), (1, 1, 1),
                                          (777, 0, 1), (0, 0, 0)])
def test_copy(n, doff, soff):
    """gs_copy (NewtonSolver.cpp:12 newtonF = f): every element and nothing else, for odd lengths, for operands
    8 B past a 16-B boundary (a field's origin: one head element, then dwordx4) and for operands without a
    common 16-B alignment (the hipMemcpyAsync path)."""
    src = torch.randn(n + 2, dtype=torch.float64, device="cuda")
    dst = torch.full((n + 2,), np.nan, dtype=torch.float64, device="cuda")
    ok(k().gs_copy(dst.data_ptr() + 8 * doff, src.data_ptr() + 8 * soff, n, stream()))
    torch.cuda.synchronize()
    assert torch.equal(dst[doff: doff + n], src[soff: soff + n])
    assert torch.isnan(dst[doff + n:]).all() and torch.isnan(dst[:doff]).all()


@pytest.mark.parametrize("dims", [(1100, 20, 18), (700, 12, 10)])
def test_newton_long_rows_vs_oracle(dims):
    """NEWTON on rows of more than 512 points: column-block pairs (k_tb2 up to 1024 points before r04), against the
    CPU oracle (pinned to src/cpu); 1e-10 on newtonV (ocml vs glibc exp), 1e-9 on the history."""
    import oracle as O
    from conftest import rel
    og = O.Grid(dims, mode=2, maxiter=2, omega=0.8, gamma=1.0, pre=2, post=2)
    oh = og.solve()
    ref = og.field(0, "newtonV").copy()
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=gsv.GS_NEWTON, preSmoothing=2, postSmoothing=2)
    with gsv.HipGridData(p) as g:
        hist = gsv.NewtonSolver.solve(g)
        got = g.field(0, "newtonV")
    assert len(hist) == len(oh)
    scale = max(np.abs(ref).max(), 1e-300)
    assert np.abs(got - ref).max() <= 1e-10 * scale
    for a, b in zip(hist, oh):
        assert rel(a, b) < 1e-9, (a, b)
