"""GS_NEWTON_B (include/gpusolve_hip.h): the inner Newton solves read the precomputed linearisation factor
B = gamma (1 + newtonV) exp(newtonV) (gs_newton_bfac, once per level and Newton iteration) instead of evaluating
exp(newtonV) in every sweep, residual and restriction. The Jacobi denominator preFac + B is the reference's
bit for bit; the operator term B * v re-associates the reference's (gamma (1 + w) v) exp(w), so the mode-3
kernels agree with the mode-2 ones to a few ulps (and their Jacobi quotient r / (preFac + B) is formed through the
denominator's one-step refined reciprocal, within 1 ulp of the IEEE quotient: test_nb_quotient_ulps), and whole Newton solves with GS_NO_NEWTON_B (mode 2 inside)
to far below the 1e-10 field / 1e-9 history tolerances the oracle comparisons use (test_gpu_solver.py,
test_gpu_zslab.py pin the default path to the reference itself)."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402

NEWTON, NEWTON_B, NEWTON_G = gsv.GS_NEWTON, gsv.GS_NEWTON_B, gsv.GS_NEWTON_G
NB_QUOT_ULPS = 1  # the quotient's bound (gs_device.hpp nb_quot: measured max 1 ulp over these draws, r05p)


def k():
    assert torch.cuda.is_available(), "GPU tests need a GPU (no CPU fallback exists)"
    return gsv.kernels()


def ok(rc):
    assert rc == 0, k().gs_strerror(rc).decode()


def st():
    return torch.cuda.current_stream().cuda_stream


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


def rand_field(rng, dims, lo, hi, interior_only=True):
    a = np.zeros(tuple(d + 2 for d in dims))
    if interior_only:
        a[1:-1, 1:-1, 1:-1] = rng.uniform(lo, hi, dims)
    else:
        a[:] = rng.uniform(lo, hi, a.shape)
    return a


def bfac(w, gamma, dims, h):
    b = DevField(*dims, fill=np.nan)
    ok(k().gs_newton_bfac(C.byref(w.level(h)), gamma, w.ptr, b.ptr, st()))
    return b


@pytest.mark.parametrize("dims,gamma", [((64, 32, 16), 1.0), ((37, 11, 5), 2.5), ((130, 7, 3), 0.25)])
def test_bfac_values(dims, gamma):
    """b = gamma (1 + w) exp(w) at every element of planes -1 .. nz+2 (ghost planes and row padding included),
    against numpy's exp: ocml's and glibc's exp differ by <= 1 ulp, the product by a few."""
    rng = np.random.default_rng(7)
    w = DevField(*dims)
    w.zyx_ext.copy_(torch.from_numpy(rng.uniform(-3, 3, tuple(w.zyx_ext.shape))))
    b = bfac(w, gamma, dims, 1.0 / (dims[1] + 1))
    torch.cuda.synchronize()
    wv, bv = w.zyx_ext.cpu().numpy(), b.zyx_ext.cpu().numpy()
    ref = gamma * (1 + wv) * np.exp(wv)
    assert np.all(np.isfinite(bv))
    np.testing.assert_allclose(bv, ref, rtol=4e-16 * 8, atol=1e-300)


def level_pair(rng, dims):
    h = 1.0 / (dims[1] + 1)
    v = DevField(*dims).from_xyz(rand_field(rng, dims, -0.5, 0.5))
    f = DevField(*dims).from_xyz(rand_field(rng, dims, -2, 2))
    w = DevField(*dims).from_xyz(rand_field(rng, dims, -0.8, 0.8))
    return h, v, f, w


def close(a, b, rel=1e-13):
    a, b = a.to_xyz(), b.to_xyz()
    scale = np.nanmax(np.abs(b))
    assert np.all(np.isfinite(a) == np.isfinite(b))
    d = np.nanmax(np.abs(a - b))
    assert d <= rel * scale, (d, scale)


@pytest.mark.parametrize("dims", [(128, 64, 32), (256, 32, 30), (700, 12, 10), (33, 31, 29)])
def test_mode3_kernels_match_mode2(dims):
    """Pair (+ norm partials), one sweep, residual, residual + restriction, fused prolongation pair: mode 3 on
    B = bfac(w) against mode 2 on w, to a few ulps of the fields."""
    S = gsv.Stencil().to_abi()
    rng = np.random.default_rng(sum(dims))
    h, v, f, w = level_pair(rng, dims)
    b = bfac(w, 1.0, dims, h)
    L = v.level(h)
    cd = tuple(d // 2 for d in dims)
    out2, out3 = DevField(*dims, fill=0.0), DevField(*dims, fill=0.0)
    # one sweep and the residual (every level shape)
    ok(k().gs_jacobi_sweep(C.byref(S), C.byref(L), NEWTON, 0.8, 1.0, v.ptr, out2.ptr, f.ptr, w.ptr, st()))
    ok(k().gs_jacobi_sweep(C.byref(S), C.byref(L), NEWTON_B, 0.8, 1.0, v.ptr, out3.ptr, f.ptr, b.ptr, st()))
    close(out3, out2)
    ok(k().gs_residual(C.byref(S), C.byref(L), NEWTON, 1.0, v.ptr, f.ptr, w.ptr, out2.ptr, None, st()))
    ok(k().gs_residual(C.byref(S), C.byref(L), NEWTON_B, 1.0, v.ptr, f.ptr, b.ptr, out3.ptr, None, st()))
    close(out3, out2, 1e-12)  # (a residual is a difference of O(1) terms: relative to the largest)
    # the fused pair, where the level has one
    if k().gs_jacobi_sweep2_supported_mode(C.byref(S), C.byref(L), NEWTON):
        for vin in (v.ptr, None):  # a loaded iterate and the zero iterate
            ok(k().gs_jacobi_sweep2(C.byref(S), C.byref(L), NEWTON, 0.8, 1.0, vin, out2.ptr, f.ptr, w.ptr, 0, 0, st()))
            ok(k().gs_jacobi_sweep2(C.byref(S), C.byref(L), NEWTON_B, 0.8, 1.0, vin, out3.ptr, f.ptr, b.ptr, 0, 0,
                                    st()))
            close(out3, out2)
    # residual + restriction
    if all(c >= 1 for c in cd):
        c2, c3 = DevField(*cd, fill=0.0), DevField(*cd, fill=0.0)
        Lc = c2.level(1.0 / (cd[1] + 1))
        ok(k().gs_residual_restrict(C.byref(S), C.byref(L), NEWTON, 1.0, v.ptr, f.ptr, w.ptr, c2.ptr, None,
                                    C.byref(Lc), st()))
        ok(k().gs_residual_restrict(C.byref(S), C.byref(L), NEWTON_B, 1.0, v.ptr, f.ptr, b.ptr, c3.ptr, None,
                                    C.byref(Lc), st()))
        close(c3, c2, 1e-12)
        # the fused prolongation pair
        if k().gs_jacobi_sweep2_prolong_supported(C.byref(S), C.byref(L), NEWTON):
            cv = DevField(*cd).from_xyz(rand_field(rng, cd, -0.1, 0.1))
            wsn = k().gs_jacobi_sweep2_prolong_ws_elems(C.byref(S), C.byref(L), NEWTON)
            ws = torch.empty(max(1, wsn), dtype=torch.float64, device="cuda")
            for mode, wp, o in ((NEWTON, w.ptr, out2), (NEWTON_B, b.ptr, out3)):
                ok(k().gs_jacobi_sweep2_prolong_ws(C.byref(S), C.byref(L), mode, 0.8, 1.0, v.ptr, cv.ptr, None,
                                                   C.byref(Lc), o.ptr, f.ptr, wp, 0, 0, ws.data_ptr(), wsn, st()))
            close(out3, out2)


def solve(params, **e):
    with env(**e):
        with gsv.HipGridData(params) as g:
            hist = gsv.NewtonSolver.solve(g)
            fields = {(l, n): g.field(l, n) for l in range(g.numLevels()) for n in ("v", "newtonV")}
    return hist, fields


@pytest.mark.parametrize("dims,pre,post", [((127, 127, 127), 2, 2), ((64, 64, 64), 3, 3), ((130, 66, 34), 2, 3),
                                           ((1100, 20, 18), 2, 2)])
def test_newton_solve_b_matches_reference_mode(dims, pre, post):
    """Whole Newton solves: the default (GS_NEWTON_B inner solves) against GS_NO_NEWTON_B (mode 2, the reference's
    expressions) — histories to 1e-11, level-0 fields to 1e-11 of their magnitude."""
    p = gsv.GridParams(maxiter=3, tol=0.0, gridDim=dims, mode=NEWTON, preSmoothing=pre, postSmoothing=post)
    h_ref, f_ref = solve(p, GS_NO_NEWTON_B=1)
    h_b, f_b = solve(p)
    assert np.all(np.isfinite(h_ref)), h_ref
    assert len(h_b) == len(h_ref)
    for a, c in zip(h_b, h_ref):
        assert abs(a - c) <= 1e-11 * abs(c), (a, c)
    for n in ("v", "newtonV"):
        a, c = f_b[(0, n)], f_ref[(0, n)]
        assert np.abs(a - c).max() <= 1e-11 * np.abs(c).max(), n


@pytest.mark.parametrize("dims,gamma", [((128, 64, 32), 1.0), ((256, 32, 30), 0.7), ((700, 12, 10), 1.3),
                                        ((1100, 20, 18), 1.0), ((33, 31, 29), 2.0)])
def test_mode_g_matches_mode_b_on_a_gamma_field(dims, gamma):
    """GS_NEWTON_G (the first Newton iteration: B = gamma everywhere) against GS_NEWTON_B on a factor field filled
    with gamma: the pair (loaded and zero iterate, with norm partials), the fused prolongation pair (column blocks
    on the long rows), residual + restriction, one sweep and the residual — bit for bit. Where the kernel honours
    the constant (k_tb2y pairs, k_rr2), it must not read the field at all: the same outputs with the field NaN."""
    S = gsv.Stencil().to_abi()
    rng = np.random.default_rng(len(dims) + dims[0])
    h, v, f, _ = level_pair(rng, dims)
    L = v.level(h)
    g_field = DevField(*dims, fill=gamma * (1 + 0.0) * np.exp(0.0))
    nan_field = DevField(*dims, fill=np.nan)
    cd = tuple(d // 2 for d in dims)

    def same(a, b):
        torch.cuda.synchronize()
        assert a.zyx_ext.cpu().numpy().tobytes() == b.zyx_ext.cpu().numpy().tobytes()

    outs = {}
    for tag, mode, wf in (("b", NEWTON_B, g_field), ("g", NEWTON_G, g_field), ("gnan", NEWTON_G, nan_field)):
        o = outs[tag] = {}
        o["sweep"] = DevField(*dims, fill=0.0)
        if tag != "gnan":  # one sweep / the residual read the field (k_rb)
            ok(k().gs_jacobi_sweep(C.byref(S), C.byref(L), mode, 0.8, gamma, v.ptr, o["sweep"].ptr, f.ptr, wf.ptr,
                                   st()))
            o["res"] = DevField(*dims, fill=0.0)
            ok(k().gs_residual(C.byref(S), C.byref(L), mode, gamma, v.ptr, f.ptr, wf.ptr, o["res"].ptr, None, st()))
        kname = k().gs_jacobi_sweep2_kernel(C.byref(S), C.byref(L), NEWTON_B).decode()
        if k().gs_jacobi_sweep2_supported_mode(C.byref(S), C.byref(L), NEWTON_B) and \
                (tag != "gnan" or kname.startswith("k_tb2y")):
            npart = k().gs_jacobi_sweep2_num_partials(C.byref(S), C.byref(L), NEWTON_B)
            for i, vin in enumerate((v.ptr, None)):
                o[f"pair{i}"] = DevField(*dims, fill=0.0)
                o[f"part{i}"] = torch.zeros(max(1, npart), dtype=torch.float64, device="cuda")
                ok(k().gs_jacobi_sweep2_norm(C.byref(S), C.byref(L), mode, 0.8, gamma, vin, o[f"pair{i}"].ptr, f.ptr,
                                             wf.ptr, 0, 0, o[f"part{i}"].data_ptr(), st()))
        if all(c >= 1 for c in cd):
            Lc = DevField(*cd).level(1.0 / (cd[1] + 1))
            o["rr"] = DevField(*cd, fill=0.0)
            if tag != "gnan" or k().gs_residual_restrict_slab_supported(C.byref(S), C.byref(L)):
                ok(k().gs_residual_restrict(C.byref(S), C.byref(L), mode, gamma, v.ptr, f.ptr, wf.ptr, o["rr"].ptr,
                                            None, C.byref(Lc), st()))
            if k().gs_jacobi_sweep2_prolong_supported(C.byref(S), C.byref(L), NEWTON_B):
                cv = DevField(*cd).from_xyz(np.random.default_rng(3).uniform(-0.1, 0.1, tuple(c + 2 for c in cd)))
                wsn = k().gs_jacobi_sweep2_prolong_ws_elems(C.byref(S), C.byref(L), mode)
                ws = torch.empty(max(1, wsn), dtype=torch.float64, device="cuda")
                o["pro"] = DevField(*dims, fill=0.0)
                ok(k().gs_jacobi_sweep2_prolong_ws(C.byref(S), C.byref(L), mode, 0.8, gamma, v.ptr, cv.ptr, None,
                                                   C.byref(Lc), o["pro"].ptr, f.ptr, wf.ptr, 0, 0, ws.data_ptr(), wsn,
                                                   st()))
    assert set(outs["g"]) == set(outs["b"])
    for key in outs["b"]:
        a, b = outs["g"][key], outs["b"][key]
        if isinstance(a, torch.Tensor):
            torch.cuda.synchronize()
            assert torch.equal(a, b), key
        else:
            same(a, b)
    for key, a in outs["gnan"].items():
        if key in ("sweep",) or (key == "rr" and not k().gs_residual_restrict_slab_supported(C.byref(S), C.byref(L))):
            continue
        b = outs["b"][key]
        if isinstance(a, torch.Tensor):
            torch.cuda.synchronize()
            assert torch.equal(a, b), key
        else:
            same(a, b)


@pytest.mark.parametrize("dims", [(127, 127, 127), (130, 66, 34), (1100, 20, 18)])
def test_newton_solve_g_bit_identical(dims):
    """Whole Newton solves: the first iteration's inner solve in GS_NEWTON_G (default) against GS_NO_NEWTON_G
    (GS_NEWTON_B on the gamma-filled factor fields): histories and every level's fields bit for bit."""
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=NEWTON, preSmoothing=2, postSmoothing=2)
    h_b, f_b = solve(p, GS_NO_NEWTON_G=1)
    h_g, f_g = solve(p)
    assert h_g == h_b
    for key in f_b:
        assert f_g[key].tobytes() == f_b[key].tobytes(), key


@pytest.mark.parametrize("dims", [(63, 63, 63), (130, 66, 34)])
def test_solve_upload_newtonv_solve(dims):
    """A solve, then newtonV replaced through the C ABI (gs_grid_upload), then a second solve on the same grid: the
    second solve must linearise at the uploaded newtonV on every level — level 0's factor the first solve's last update
    pass left behind (bfacFresh_) and its level-1 restriction (newtonR1_) are stale — so it equals the same sequence
    with level 0's factor formed by its own pass (GS_NEWTON_B_FUSED=0), bit for bit. A download of newtonV between
    the solves (read-only: no state dropped) leaves the second solve unchanged too."""
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=NEWTON, preSmoothing=2, postSmoothing=2)
    x = rand_field(np.random.default_rng(5), dims, -0.2, 0.2)

    def run(upload, **e):
        with env(**e):
            with gsv.HipGridData(p) as g:
                gsv.NewtonSolver.solve(g)
                g.field(0, "newtonV")  # read-only
                if upload:
                    g.set_field(0, "newtonV", x)
                hist = gsv.NewtonSolver.solve(g)
                return hist, {n: g.field(0, n) for n in ("v", "newtonV")}

    h_fused, f_fused = run(True)
    h_sep, f_sep = run(True, GS_NEWTON_B_FUSED=0)
    assert np.all(np.isfinite(h_sep)), h_sep
    assert h_fused == h_sep
    for n in f_sep:
        assert f_fused[n].tobytes() == f_sep[n].tobytes(), n
    h_plain, _ = run(False)
    h_plain_sep, _ = run(False, GS_NEWTON_B_FUSED=0)
    assert h_plain == h_plain_sep
    assert h_plain != h_fused  # (the upload did change the linearisation point)


def test_nb_quotient_ulps():
    """The GS_NEWTON_B Jacobi quotient (nb_quot: r times the refined reciprocal of den clamped at 2^1000) against the
    IEEE quotient: within 1 ulp over the denominators the solver forms (preFac + B, from the coarsest level's ~24
    up to 2^40) and numerators of every magnitude; the non-finite cases stay non-finite where the IEEE quotient is
    (NaN in, NaN out; den = 0), and den = inf gives a quotient below |r| 2^-999 (the IEEE one is 0)."""
    rng = np.random.default_rng(11)
    n = 400_000
    # the solver's range (preFac + B from ~24 up), then (r06) negative denominators — B < 0 where w < -1 — and
    # small magnitudes of either sign down to 2^-990, where the reciprocal is still normal
    m = n // 2
    den = np.exp(rng.uniform(np.log(20.0), np.log(2.0 ** 40), m))
    mag = np.exp2(rng.uniform(-990.0, 40.0, n - m))
    den = np.concatenate([den, np.where(rng.random(n - m) < 0.5, -mag, mag)])
    r = rng.normal(0, 1, n) * np.exp(rng.uniform(-200, 200, n))
    edge_r = np.array([1.0, -2.0, 0.0, 1e300, -1e-300])
    edge_den = np.array([np.inf, -np.inf, np.nan, 0.0])
    den = np.concatenate([den, np.repeat(edge_den, edge_r.size), np.full(3, 1e6)])
    r = np.concatenate([r, np.tile(edge_r, edge_den.size), [np.nan, np.inf, -np.inf]])
    dr, dd = torch.from_numpy(r).cuda(), torch.from_numpy(den).cuda()
    q = torch.empty_like(dr)
    assert gsv.diag().gs_debug_nb_quot(dr.data_ptr(), dd.data_ptr(), dr.numel(), q.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    got = q.cpu().numpy()
    with np.errstate(all="ignore"):
        want = r / den
    body = slice(0, n)
    fin = np.isfinite(want[body]) & (np.abs(want[body]) >= np.finfo(float).tiny)
    ulp = np.spacing(np.abs(want[body][fin]))
    worst = np.max(np.abs(got[body][fin] - want[body][fin]) / ulp)
    print(f"nb_quot: max {worst} ulp, {np.mean(got[body][fin] != want[body][fin]):.4f} of the quotients differ from r / den")
    assert worst <= NB_QUOT_ULPS, worst
    ne = edge_den.size * edge_r.size
    e = slice(n, n + ne)
    ge, de, re_ = got[e], den[e], r[e]
    inf_d = np.isinf(de)
    assert np.all(np.abs(ge[inf_d]) <= np.abs(re_[inf_d]) * 2.0 ** -999)
    nz = inf_d & (re_ != 0)  # the clamp keeps the denominator's sign: r / -inf is -r 2^-1000 (or -0), not +
    assert np.all(np.signbit(ge[nz]) == (np.signbit(re_[nz]) ^ np.signbit(de[nz])))
    assert np.all(np.isnan(ge[np.isnan(de)]))
    assert not np.any(np.isfinite(ge[(de == 0) & (re_ != 0)]))
    tail = got[n + ne:]
    assert np.isnan(tail[0]) and np.isinf(tail[1]) and np.isinf(tail[2])
