"""The one-launch coarse end of the V-cycle (gs_coarse_cycle, HipSolver::coarseCycle) against the
per-operator launch sequence it replaces (GS_COARSE_POINTS=0): every level's iterate and every
residual of whole solves must be bit-identical, in all three modes, for several hierarchy shapes,
smoothing counts and coarse-start thresholds. The per-operator path is itself pinned to the
reference (test_gpu_solver.py), so this pins the fused kernel to src/cpu/CpuSolver.cpp:85-139."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402


def solve_with(params, coarse_points):
    old = os.environ.get("GS_COARSE_POINTS")
    os.environ["GS_COARSE_POINTS"] = str(coarse_points)
    try:
        with gsv.HipGridData(params) as g:
            hist = gsv.HipSolver.solve(g)
            names = ("v", "newtonV") if params.mode == gsv.GS_NEWTON else ("v",)
            fields = {(l, n): g.field(l, n) for l in range(g.numLevels()) for n in names}
    finally:
        if old is None:
            del os.environ["GS_COARSE_POINTS"]
        else:
            os.environ["GS_COARSE_POINTS"] = old
    return hist, fields


CASES = [
    # dims, mode, pre, post, threshold (points of the first level inside the launch)
    ((64, 64, 64), 0, 2, 2, 4096),
    ((64, 64, 64), 0, 2, 2, 512),  # the default start level (8^3)
    ((64, 64, 64), 0, 2, 2, 40000),  # the 32^3 level inside the launch too
    ((31, 31, 31), 0, 3, 3, 4096),
    ((33, 31, 29), 0, 1, 0, 4096),
    ((17, 9, 12), 0, 2, 1, 1 << 30),  # every level but the finest
    ((40, 24, 48), 0, 0, 2, 4096),  # no pre-smoothing: zero iterates made real in the kernel
    ((130, 66, 34), 0, 2, 2, 4096),
    ((33, 31, 29), 1, 2, 2, 4096),  # FAS
    ((64, 64, 64), 1, 1, 2, 40000),
    ((33, 31, 29), 2, 2, 2, 4096),  # Newton (inner solves)
    ((31, 31, 31), 2, 3, 3, 1 << 30),
]


@pytest.mark.parametrize("dims,mode,pre,post,thr", CASES)
def test_coarse_cycle_bit_identical(dims, mode, pre, post, thr):
    p = gsv.GridParams(maxiter=3, tol=0.0, gridDim=dims, mode=mode, preSmoothing=pre, postSmoothing=post)
    h_ref, f_ref = solve_with(p, 0)
    h_got, f_got = solve_with(p, thr)
    assert h_got == h_ref
    for key, a in f_ref.items():
        np.testing.assert_array_equal(f_got[key], a, err_msg=str(key))


def test_coarse_cycle_rejects_bad_arguments():
    kl = gsv.kernels()
    st = gsv.Stencil().to_abi()
    lv = (gsv._abi.gs_coarse_level * 2)()
    mx = kl.gs_coarse_cycle_max_levels()
    assert mx >= 4
    E = gsv._abi.GS_EINVAL
    assert kl.gs_coarse_cycle(C.byref(st), lv, 0, 0, 0.8, 1.0, 2, 2, None) == E  # no levels
    assert kl.gs_coarse_cycle(C.byref(st), lv, mx + 1, 0, 0.8, 1.0, 2, 2, None) == E  # too many
    assert kl.gs_coarse_cycle(C.byref(st), lv, 2, 0, 0.8, 1.0, 2, 2, None) == E  # null fields
    bad = gsv.Stencil(offsets=[(0, 0, 0), (2, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)])
    assert kl.gs_coarse_cycle(C.byref(bad.to_abi()), lv, 1, 0, 0.8, 1.0, 2, 2, None) == E
