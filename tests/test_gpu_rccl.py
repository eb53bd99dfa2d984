"""The RCCL communicator on ONE GPU (one rank): ncclGetUniqueId / ncclCommInitRank through the C ABI
(gs_rccl_unique_id, gs_grid_create_rccl — the calls bench.py makes on every rank at N > 1) and a solve
on the resulting grid, which must be bit-identical to the plain single-GPU grid. Send/recv halos and
the broadcast of replicated levels between real rank processes: test_gpu_rccl_multirank.py."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402


def rccl_grid(params):
    drv = gsv.driver()
    uid = (C.c_ubyte * 128)()
    assert drv.gs_rccl_unique_id(uid) == 0, drv.gs_last_error().decode()
    g = gsv.HipGridData.__new__(gsv.HipGridData)
    g.params = params
    g._abi_params = params.to_abi()
    g.handle = drv.gs_grid_create_rccl(C.byref(g._abi_params), 0, 1, uid)
    assert g.handle, drv.gs_last_error().decode()
    return g


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_rccl_one_rank_solve_bit_identical(mode):
    p = gsv.GridParams(maxiter=3 if mode == 2 else 4, tol=0.0, gridDim=(40, 33, 48), mode=mode)
    with gsv.HipGridData(p) as g:
        ref_h = gsv.NewtonSolver.solve(g) if mode == 2 else gsv.HipSolver.solve(g)
        ref_v = g.field(0, "v")
    g = rccl_grid(p)
    try:
        h = gsv.NewtonSolver.solve(g) if mode == 2 else gsv.HipSolver.solve(g)
        v = g.field(0, "v")
    finally:
        g.close()
    assert h == ref_h
    np.testing.assert_array_equal(v, ref_v)


def test_rccl_injected_error_aborts(monkeypatch):
    """GS_COMM_INJECT_ERROR=1: the first settle of the non-blocking communicator (its initialisation)
    sees ncclInternalError; the communicator is aborted and the grid creation fails with the message
    GpuSolve-hip would print after "Exception: " instead of hanging."""
    monkeypatch.setenv("GS_COMM_INJECT_ERROR", "1")
    drv = gsv.driver()
    uid = (C.c_ubyte * 128)()
    assert drv.gs_rccl_unique_id(uid) == 0
    p = gsv.GridParams(maxiter=1, gridDim=(16, 16, 16)).to_abi()
    assert not drv.gs_grid_create_rccl(C.byref(p), 0, 1, uid)
    msg = drv.gs_last_error().decode()
    assert "RCCL" in msg and "internal error" in msg and "rank 0 of 1" in msg and "aborted" in msg, msg
    monkeypatch.delenv("GS_COMM_INJECT_ERROR")
    g = rccl_grid(gsv.GridParams(maxiter=1, gridDim=(16, 16, 16)))  # a healthy communicator afterwards
    g.close()


def test_rccl_bad_rank_rejected():
    drv = gsv.driver()
    uid = (C.c_ubyte * 128)()
    p = gsv.GridParams(maxiter=1, gridDim=(8, 8, 8)).to_abi()
    assert not drv.gs_grid_create_rccl(C.byref(p), 1, 1, uid)
    assert b"bad arguments" in drv.gs_last_error()


def test_executable_rccl_path_matches_reference_stdout(tmp_path):
    """GpuSolve-hip's multi-process path (WORLD_SIZE / RANK from a launcher, RCCL id through a file) with
    one rank (GS_FORCE_RCCL=1): the reference's stdout line for line, as the single-GPU path, and the id
    file removed afterwards (two ranks: test_gpu_rccl_multirank.py)."""
    import re
    import subprocess
    from conftest import load_json
    from test_gpu_solver import _norm_lines, params_from_case
    exe = gsv._abi.EXECUTABLE
    uid = tmp_path / "uid"
    env = dict(os.environ, GS_FORCE_RCCL="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", GS_UID_FILE=str(uid))
    cases = load_json("stdout.json")
    for name in ("m0_n31_2+2", "m1_n15_2+2", "example_data-2nd_order"):
        case = cases[name]
        conf = tmp_path / f"{name}.conf"
        conf.write_text(params_from_case(case["config"]).config_text())
        out = subprocess.run([exe, str(conf)], capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode == 0 and "Exception" not in out.stderr, out.stderr
        assert _norm_lines(out.stdout.splitlines()) == case["stdout"], (name, out.stdout)
        assert not uid.exists()
    # a rank outside the world is an error line, not a hang
    bad = dict(env, WORLD_SIZE="2", RANK="5")
    conf = tmp_path / "m0_n31_2+2.conf"
    out = subprocess.run([exe, str(conf)], capture_output=True, text=True, timeout=60, env=bad)
    assert out.returncode == 0 and re.search(r"Exception: RANK 5 outside WORLD_SIZE 2", out.stderr)
