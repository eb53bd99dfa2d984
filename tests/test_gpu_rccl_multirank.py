"""RCCL between ranks, on one GPU: 2-8 processes (one per rank, as bench.py and GpuSolve-hip run at N > 1)
build their Z-slabs with gs_grid_create_rccl and solve; the assembled level-0 field must be bit-identical
to the single-GPU solve and the history agree to 1e-12 (rank partials of the norm summed in rank order).

RCCL refuses two ranks on one GPU of one host ("Duplicate GPU detected"); a distinct NCCL_HOSTID per
process makes each rank its own host, so the ranks connect through RCCL's socket transport over loopback
(NCCL_SOCKET_IFNAME=lo) instead of xGMI. The transport differs from the 8-GPU node's; everything above it
— the non-blocking communicator's init and settle loop, the grouped ghost-plane send/recv of the
overlapped sweeps, the in-place broadcast group that assembles replicated levels, the norm allgather —
is the product's own code (gs_comm.cpp, gs_grid.cpp) moving real bytes between ranks."""
import math
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, rel

pytestmark = pytest.mark.gpu

# torch before the library, as in every GPU test module: the process then runs one HIP runtime (torch's
# bundled libamdhip64.so.7, which the library's same-soname dependency resolves to) for its whole life
torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
PROBE = os.path.join(REPO, "tests", "rccl_rank_probe.py")


def rank_env(rank, world, extra=None):
    env = dict(os.environ)
    env.update({"NCCL_HOSTID": f"gs-test-rank-{rank}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0", "WORLD_SIZE": str(world), "RANK": str(rank),
                "LOCAL_RANK": "0", "GS_COMM_INIT_TIMEOUT_S": "90", "GS_COMM_TIMEOUT_S": "60"})
    env.update(extra or {})
    return env


def start_ranks(tmp_path, world, mode, dims, maxiter, extra=None, die=False, digest=False):
    uid = str(tmp_path / "uid")
    procs = []
    for r in range(world):
        out = str(tmp_path / f"rank{r}.npz")
        args = [sys.executable, PROBE, out, str(r), str(world), uid, str(mode), *map(str, dims), str(maxiter)]
        args += ["die"] if die else (["digest"] if digest else [])
        procs.append((subprocess.Popen(args, env=rank_env(r, world, extra), stdout=subprocess.PIPE,
                                       stderr=subprocess.PIPE, text=True), out))
    return procs


def run_ranks(tmp_path, world, mode, dims, maxiter, extra=None):
    procs = start_ranks(tmp_path, world, mode, dims, maxiter, extra)
    errs = []
    for p, _ in procs:
        try:
            _, err = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            raise
        if p.returncode != 0:
            errs.append(err[-3000:])
    assert not errs, "\n---\n".join(errs)
    parts = [np.load(o) for _, o in procs]
    parts.sort(key=lambda d: int(d["z0"]))
    z = 0
    for d in parts:  # the slabs tile the z axis in rank order
        assert int(d["z0"]) == z, (int(d["z0"]), z)
        z += d["v"].shape[2]
    assert z == dims[2]
    hists = [list(d["hist"]) for d in parts]
    # (np.array_equal with equal_nan: a diverging NONLINEAR draw ends in NaN on every rank alike)
    assert all(np.array_equal(h, hists[0], equal_nan=True) for h in hists), ("ranks disagree on the history", hists)
    return hists[0], np.concatenate([d["v"] for d in parts], axis=2)


def same_history(h, ref_h):
    assert len(h) == len(ref_h)
    for a, b in zip(h, ref_h):
        assert a == b or (math.isnan(a) and math.isnan(b)) or rel(a, b) < 1e-12, (a, b)  # inf / NaN: diverged alike


def single(mode, dims, maxiter):
    p = gsv.GridParams(maxiter=maxiter, tol=0.0, gridDim=dims, mode=mode)
    with gsv.HipGridData(p) as g:
        h = gsv.NewtonSolver.solve(g) if mode == 2 else gsv.HipSolver.solve(g)
        v = g.field(0, "v")[:, :, 1:-1]
    return h, v


@pytest.mark.parametrize("world,mode,dims,maxiter,extra", [
    (2, 0, (32, 32, 32), 4, None),
    (2, 1, (31, 33, 40), 4, None),
    (2, 2, (32, 32, 32), 2, None),
    # slabs large enough for the fused pairs, their depth-2 ghosts and the overlapped boundary planes;
    # levels kept partitioned down to 8^3 points (GS_ZSLAB_MIN_POINTS) and the default agglomeration
    (2, 0, (64, 256, 64), 3, {"GS_ZSLAB_MIN_POINTS": "512"}),
    (2, 0, (64, 256, 64), 3, None),
    (3, 0, (48, 512, 70), 3, None),
    (3, 1, (40, 24, 50), 3, None),
    # the driver's 8-GPU rank count (config #5 decomposes 1024^3 the same way: 8 slabs, default agglomeration)
    (8, 0, (64, 96, 256), 3, None),
    (4, 2, (32, 32, 64), 2, None),
    # larger slabs: two 256^3 ranks (one-round chunks on rank 0, the slab rule past it), and BASELINE
    # config #3's grid on 8 ranks (512x512x64 slabs)
    (2, 0, (256, 256, 512), 3, None),
    (8, 0, (512, 512, 512), 2, None),
])
def test_rccl_ranks_match_single_gpu(tmp_path, world, mode, dims, maxiter, extra):
    h, v = run_ranks(tmp_path, world, mode, dims, maxiter, extra)
    ref_h, ref_v = single(mode, dims, maxiter)
    same_history(h, ref_h)
    np.testing.assert_array_equal(v, ref_v)


def test_executable_two_ranks_match_reference_stdout(tmp_path):
    """GpuSolve-hip under a launcher's WORLD_SIZE / RANK with two real ranks: rank 0 prints the
    reference's stdout line for line (the other rank prints nothing), both exit 0."""
    from conftest import load_json
    from test_gpu_solver import _norm_lines, params_from_case
    exe = gsv._abi.EXECUTABLE
    case = load_json("stdout.json")["m0_n31_2+2"]
    conf = tmp_path / "m0.conf"
    conf.write_text(params_from_case(case["config"]).config_text())
    uid = str(tmp_path / "uid")
    procs = [subprocess.Popen([exe, str(conf)], env=rank_env(r, 2, {"GS_UID_FILE": uid}), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=150))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0 and "Exception" not in e, e[-3000:]
    assert _norm_lines(outs[0][0].splitlines()) == case["stdout"], outs[0][0]
    assert outs[1][0].strip() == "", outs[1][0]


def test_lost_peer_is_an_error_not_a_hang(tmp_path):
    """Rank 1 leaves right after the communicator and its slab exist; rank 0's solve must not wait for
    it forever: its bounded wait (GS_COMM_TIMEOUT_S) or RCCL's own error report aborts the communicator
    and the solve fails with the RCCL message GpuSolve-hip would print after "Exception: "."""
    import time
    t0 = time.time()
    procs = start_ranks(tmp_path, 2, 0, (64, 64, 64), 50, {"GS_COMM_TIMEOUT_S": "20"}, die=True)
    res = []
    for p, _ in procs:
        try:
            res.append(p.communicate(timeout=150))
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            raise
    assert procs[1][0].returncode == 3
    assert procs[0][0].returncode not in (0, None), res[0][1][-2000:]
    err = res[0][1]
    assert "RCCL" in err and "rank 0 of 2" in err and "aborted" in err, err[-2000:]
    assert time.time() - t0 < 140


def rccl_cases(n=None, seed=None):
    """Seeded random multi-rank problems: 2-5 ranks, all modes, shapes whose slabs hit uneven plane
    counts and both agglomeration choices (GS_RCCL_FUZZ_N / GS_RCCL_FUZZ_SEED draw more)."""
    import numpy as np
    n = int(os.environ.get("GS_RCCL_FUZZ_N", 6)) if n is None else n
    rng = np.random.default_rng(int(os.environ.get("GS_RCCL_FUZZ_SEED", 20261017)) if seed is None else seed)
    out = []
    for i in range(n):
        world = int(rng.integers(2, 6))
        dims = (int(rng.integers(8, 80)), int(rng.integers(8, 80)), int(rng.integers(4 * world, 120)))
        mode = int(rng.integers(0, 3))
        extra = {"GS_ZSLAB_MIN_POINTS": str(int(rng.choice([512, 4096, 32768])))}
        out.append((i, world, mode, dims, 2 if mode == 2 else 3, extra))
    return out


@pytest.mark.parametrize("case", rccl_cases(), ids=lambda c: f"r{c[0]}-w{c[1]}-m{c[2]}-{'x'.join(map(str, c[3]))}")
def test_rccl_random_vs_single_gpu(tmp_path, case):
    _, world, mode, dims, maxiter, extra = case
    h, v = run_ranks(tmp_path, world, mode, dims, maxiter, extra)
    ref_h, ref_v = single(mode, dims, maxiter)
    same_history(h, ref_h)
    np.testing.assert_array_equal(v, ref_v)


def test_rccl_config5_eight_ranks_match_single_gpu(tmp_path):
    """BASELINE config #5's decomposition over RCCL: 1024^3 linear 2+2 on 8 rank processes (1024x1024x128
    slabs, column-block pairs, default agglomeration), 2 V-cycles; every owned plane of level 0 bit for bit
    (SHA-1 per plane) against the single-GPU 1024^3 solve, histories to 1e-12."""
    import rccl_rank_probe as probe
    dims, world, maxiter = (1024, 1024, 1024), 8, 2
    procs = start_ranks(tmp_path, world, 0, dims, maxiter, digest=True)
    errs = []
    for p, _ in procs:
        try:
            _, err = p.communicate(timeout=280)
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            raise
        if p.returncode != 0:
            errs.append(err[-3000:])
    assert not errs, "\n---\n".join(errs)
    parts = sorted((np.load(o) for _, o in procs), key=lambda d: int(d["z0"]))
    hists = [list(d["hist"]) for d in parts]
    assert all(np.array_equal(h, hists[0]) for h in hists)
    ref_h, ref_v = single(0, dims, maxiter)
    same_history(hists[0], ref_h)
    ref = probe.plane_digests(ref_v)
    got = [h for d in parts for h in d["digests"]]
    assert len(got) == dims[2] and [int(d["z0"]) for d in parts] == [128 * r for r in range(world)]
    assert got == ref
