"""NEWTON's fused prolongation pair inside whole solves. The driver takes it only on levels of at
least GS_NEWTON_PRO_POINTS points (default 2^21 since r06, 2^24 before: below that gs_prolong_add + the plain pair is
faster); forcing it on every level (0) must leave every field and every residual bit-identical to
the unfused sequence (a threshold no level reaches), on one GPU and on Z-slabs. The unfused
sequence is itself pinned to the reference (test_gpu_solver.py: src/cpu/NewtonSolver.cpp)."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402


class env:
    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kw}
        os.environ.update({k: str(v) for k, v in self.kw.items()})

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def solve(params):
    with gsv.HipGridData(params) as g:
        hist = gsv.NewtonSolver.solve(g)
        fields = {(l, n): g.field(l, n) for l in range(g.numLevels()) for n in ("v", "newtonV")}
    return hist, fields


@pytest.mark.parametrize("dims,pre,post", [((64, 64, 64), 2, 2), ((33, 31, 29), 3, 3), ((40, 24, 48), 1, 2),
                                           ((130, 66, 34), 2, 3),
                                           # rows > 512 points: the column-block NEWTON prolongation pair (r04)
                                           ((1400, 12, 10), 2, 2), ((1100, 20, 18), 2, 2), ((1024, 16, 16), 2, 3)])
def test_newton_fused_prolong_bit_identical(dims, pre, post):
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=gsv.GS_NEWTON, preSmoothing=pre, postSmoothing=post)
    with env(GS_NEWTON_PRO_POINTS=1 << 62):
        h_ref, f_ref = solve(p)
    with env(GS_NEWTON_PRO_POINTS=0):
        h_got, f_got = solve(p)
    assert np.all(np.isfinite(h_ref)), h_ref
    assert h_got == h_ref
    for key, a in f_ref.items():
        np.testing.assert_array_equal(f_got[key], a, err_msg=str(key))


@pytest.mark.parametrize("dims", [(64, 128, 128), (1030, 18, 16)])  # (1030: column-block prolongation pairs)
def test_newton_fused_prolong_slabs(dims):
    """Z-slab loopback (2 ranks) with the fused NEWTON pair on every slab level == without it."""
    d = gsv.driver()
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=gsv.GS_NEWTON).to_abi()
    out = []
    for thr in (1 << 62, 0):
        v = np.zeros((dims[2] + 2, dims[1] + 2, dims[0] + 2))
        hist = (C.c_double * 64)()
        cnt = C.c_int(0)
        with env(GS_NEWTON_PRO_POINTS=thr):
            rc = d.gs_zslab_loopback_run(C.byref(p), 2, -1, 0, 1, hist, 64, C.byref(cnt),
                                         v.ctypes.data_as(gsv._abi.dptr))
        assert rc == 0, d.gs_last_error().decode()
        out.append((list(hist[: cnt.value]), v))
    assert np.all(np.isfinite(out[0][0])), out[0][0]
    assert out[0][0] == out[1][0]
    np.testing.assert_array_equal(out[0][1], out[1][1])
