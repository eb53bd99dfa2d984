"""CPU coverage of the Z-slab decomposition:

1. the ownership plan (gs_zslab_plan, the driver's own host code) covers every plane exactly once
   on every level, honours the "coarse plane zc belongs to the owner of fine plane 2 zc" rule, and
   keeps every stencil / transfer read inside [lo-1, hi+1] (one ghost plane);
2. the driver's own Z-slab schedule (gs_zslab_schedule: HipSolver in trace mode, every launch, plane
   range, ghost exchange, gather and norm reduction of gs_grid.cpp) replayed on world_size 2 / 3
   torch.distributed (gloo) ranks with the oracle's point arithmetic (tests/zslab_exec.py) reproduces
   the single-domain oracle solve bit for bit.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import gpusolve as gsv
import oracle as O


def plan(dims, nranks, min_points=0):
    d = gsv.driver()
    L = 16
    distributed = (C.c_int * L)()
    lo = (C.c_int64 * (L * nranks))()
    hi = (C.c_int64 * (L * nranks))()
    n = d.gs_zslab_plan((C.c_int64 * 3)(*dims), nranks, min_points, L, distributed, lo, hi)
    return n, [distributed[l] for l in range(n)], [[(lo[l * nranks + r], hi[l * nranks + r]) for r in range(nranks)]
                                                   for l in range(n)]


@pytest.mark.parametrize("dims,nranks", [((64, 64, 64), 2), ((1024, 1024, 1024), 8), ((512, 512, 1024), 2),
                                         ((31, 31, 63), 4), ((48, 40, 64), 3), ((7, 7, 7), 2), ((16, 16, 9), 8)])
def test_plan_properties(dims, nranks):
    n, distributed, own = plan(dims, nranks)
    nz = dims[2]
    for l in range(n):
        if l:
            nz //= 2
        if l + 1 == n:
            assert not distributed[l], "coarsest level is always replicated"
        if l and not distributed[l - 1]:
            assert not distributed[l], "replicated levels stay replicated"
        covered = []
        for r in range(nranks):
            lo, hi = own[l][r]
            covered += list(range(lo, hi + 1))
            if l:
                plo, phi = own[l - 1][r]
                assert lo == (plo + 1) // 2 and hi == phi // 2      # zc owned iff 2 zc owned
            if distributed[l]:
                assert hi >= lo
                # restriction reads fine planes 2zc-1..2zc+1, prolongation coarse floor(z/2)..+1
                if l:
                    plo, phi = own[l - 1][r]
                    assert 2 * lo - 1 >= plo - 1 and 2 * hi + 1 <= phi + 1
                if l + 1 < n:
                    clo, chi = own[l + 1][r]
                    assert lo // 2 >= clo - 1 and hi // 2 + 1 <= chi + 1
        if l == 0 or distributed[l - 1]:
            assert sorted(covered) == list(range(1, nz + 1)), "every plane owned exactly once"


def test_plan_baseline_config5():
    """1024^3 on 8 GPUs: 128 planes per rank; agglomeration below 32^3-sized levels."""
    n, distributed, own = plan((1024, 1024, 1024), 8, -1)
    assert own[0] == [(1 + 128 * r, 128 * (r + 1)) for r in range(8)]
    assert distributed[:6] == [1] * 6 and not any(distributed[6:])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _replay_worker(rank, world, port, params, min_points, q, mutation=None, stop_after=None):
    """One gloo rank: replay this rank's schedule from the driver (gs_zslab_schedule) on its slab."""
    import zslab_exec as X
    if stop_after is not None:  # the traced loop stops after cycle `stop_after` (HipGridData::traceNorm)
        os.environ["GS_TRACE_STOP_AFTER"] = str(stop_after)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops = X.schedule(params, world, rank, min_points)
        if mutation:
            ops = X.mutate(ops, mutation)
        R = X.Rank(params, rank, world, min_points)
        R.run(ops)
        lo, hi, v = R.owned_v()
        q.put((rank, lo, hi, v, R.history, sorted({op for op, _ in ops})))
    except Exception as e:  # reported to the parent, which fails the test
        import traceback
        q.put((rank, None, None, None, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


REPLAY_CASES = [
    # fused pairs, slab residual+restriction, fused prolongation pair on slabs, gather + coarse cycle
    ((64, 256, 64), 2, -1, 2, 2),
    # single sweeps (levels too small for pairs), unfused prolongation
    ((40, 36, 64), 2, 0, 2, 2),
    # odd smoothing counts: a pair plus a single sweep; odd coarse-cycle count (its result in vAlt)
    ((64, 256, 64), 2, -1, 3, 2),
    # three ranks, uneven slabs
    ((48, 256, 70), 3, -1, 2, 2),
]


def _replay(dims, world, min_points, pre, post, cycles=2, mutation=None, stop_after=None):
    import gpusolve as gsv
    params = gsv.GridParams(maxiter=cycles, tol=0.0, gridDim=dims, mode=0, preSmoothing=pre, postSmoothing=post)
    ran = cycles if stop_after is None else stop_after + 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replay_worker, args=(r, world, port, params, min_points, q, mutation, stop_after))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] is not None, r[4]
    for p in procs:
        assert p.exitcode == 0
    og = O.Grid(dims, mode=O.LINEAR, maxiter=ran, pre=pre, post=post)
    ref_hist = og.solve()
    ref_v = og.field(0, "v").copy()  # (a view into the oracle grid, which dies with og)
    got = np.full_like(ref_v, np.nan)
    got[:, :, 0] = ref_v[:, :, 0]
    got[:, :, -1] = ref_v[:, :, -1]
    ops_seen = set()
    hists = []
    for rank, lo, hi, v, hist, ops in res:
        got[:, :, lo: hi + 1] = v
        ops_seen |= set(ops)
        hists.append(hist)
    return got, ref_v, hists, ref_hist, ops_seen


@pytest.mark.parametrize("dims,world,min_points,pre,post", REPLAY_CASES)
def test_gloo_replay_of_driver_schedule(dims, world, min_points, pre, post):
    """The Z-slab schedule the driver itself issues (HipSolver in trace mode, gs_grid.cpp), replayed on
    `world` gloo ranks with the oracle's point arithmetic: level-0 fields bit-identical to the
    single-domain oracle solve and the residual history to 1e-12. A changed exchange order, plane
    range or ghost depth in gs_grid.cpp that breaks the decomposition fails here, on the CPU."""
    got, ref_v, hists, ref_hist, ops_seen = _replay(dims, world, min_points, pre, post)
    for hist in hists:
        assert len(hist) == len(ref_hist)
        for a, b in zip(hist, ref_hist):
            assert abs(a - b) <= 1e-12 * abs(b), (a, b)
    np.testing.assert_array_equal(got, ref_v)
    if dims == (64, 256, 64) and pre == 2:
        assert {"pair", "pro", "resrestrict", "halo", "gather", "coarse"} <= ops_seen, ops_seen


def _random_replay_cases(n=4, seed=11):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        world = int(rng.integers(2, 4))
        dims = (int(rng.integers(8, 48)), int(rng.integers(8, 200)), int(rng.integers(6 * world, 72)))
        out.append((dims, world, int(rng.choice([-1, 0, 4096])), int(rng.integers(1, 4)), int(rng.integers(1, 4))))
    return out


@pytest.mark.parametrize("dims,world,min_points,pre,post", _random_replay_cases())
def test_gloo_replay_random_shapes(dims, world, min_points, pre, post):
    """Seeded random shapes, rank counts, thresholds and smoothing counts through the same replay."""
    got, ref_v, hists, ref_hist, _ = _replay(dims, world, min_points, pre, post)
    for hist in hists:
        assert len(hist) == len(ref_hist)
        for a, b in zip(hist, ref_hist):
            assert abs(a - b) <= 1e-12 * abs(b), (a, b)
    np.testing.assert_array_equal(got, ref_v)


@pytest.mark.parametrize("stop_after", [0, 1])
def test_gloo_replay_early_stop(stop_after):
    """A loop that stops after cycle `stop_after` of 4 while the next cycle's down-leg is already
    enqueued (HipSolver::runCycles): the recorded schedule contains that down-leg and the undo of the
    adoption of the speculative pair; replayed, level 0 must equal the oracle's after stop_after + 1
    cycles, bit for bit."""
    got, ref_v, hists, ref_hist, _ = _replay((64, 256, 64), 2, -1, 2, 2, cycles=4, stop_after=stop_after)
    for hist in hists:
        assert len(hist) == len(ref_hist) == stop_after + 2
        for a, b in zip(hist, ref_hist):
            assert abs(a - b) <= 1e-12 * abs(b), (a, b)
    np.testing.assert_array_equal(got, ref_v)


@pytest.mark.parametrize("mutation", ["halo", "depth", "range"])
def test_gloo_replay_catches_a_broken_schedule(mutation):
    """The same replay with one deliberate schedule defect must NOT reproduce the oracle."""
    got, ref_v, hists, ref_hist, _ = _replay((64, 256, 64), 2, -1, 2, 2, mutation=mutation)
    same_field = np.array_equal(got, ref_v)
    same_hist = all(abs(a - b) <= 1e-12 * abs(b) for a, b in zip(hists[0], ref_hist))
    assert not (same_field and same_hist), "a broken schedule went unnoticed"


@pytest.mark.parametrize("order", ["1", "2"])
@pytest.mark.parametrize("dims,world,min_points,pre,post", [((64, 256, 64), 2, -1, 4, 3), ((48, 256, 70), 3, -1, 6, 2)])
def test_gloo_replay_halo_orders(monkeypatch, order, dims, world, min_points, pre, post):
    """Multi-step smoothing calls (several overlapped pair steps per HipSolver::jacobi call) with the
    pipelined sequence's two dispatch orders forced (GS_HALO_ORDER=1: interior k before boundary k, as when
    exchange k-1 is still settling on the host; 2: boundary first): the recorded schedule replays bit for
    bit, and order 1 really puts an interior launch ahead of its step's boundary planes."""
    import zslab_exec as X
    monkeypatch.setenv("GS_HALO_ORDER", order)
    params = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=0, preSmoothing=pre, postSmoothing=post)
    ops = X.schedule(params, world, 0, min_points)
    # the first launch of a step that follows another in the same call (after the previous step's exchange
    # and swap): boundary planes (z1 == 1) or the interior range
    firsts = [ops[i + 2] for i in range(len(ops) - 2)
              if ops[i][0] == "halo" and ops[i][1].get("field") == "vAlt" and ops[i + 1][0] == "swap"
              and ops[i + 2][0] == "pair"]
    interior_first = any(kv["z1"] > 2 for _, kv in firsts)
    assert firsts and interior_first == (order == "1"), firsts
    got, ref_v, hists, ref_hist, _ = _replay(dims, world, min_points, pre, post)
    for hist in hists:
        assert len(hist) == len(ref_hist)
        for a, b in zip(hist, ref_hist):
            assert abs(a - b) <= 1e-12 * abs(b), (a, b)
    np.testing.assert_array_equal(got, ref_v)


def test_newton_slab_schedule_fuses_the_update(monkeypatch):
    """NEWTON on Z-slabs (trace mode): findError's newtonV += v is fused into the next compF
    (newtonFupdate) and the new newtonV's two ghost planes are formed from both operands (ghostsum, planes 0
    and nz+1) instead of a whole-array axpy; GS_NO_NEWTON_FUSED_UPDATE restores the two passes."""
    import zslab_exec as X
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=(512, 128, 128), mode=2)
    ops = X.schedule(p, 2, 0, -1)
    names = [op for op, _ in ops]
    assert names.count("newtonFupdate") == 2 and "axpy" not in names
    ghost = [kv["plane"] for op, kv in ops if op == "ghostsum"]
    assert ghost == [0, 65, 0, 65], ghost
    monkeypatch.setenv("GS_NO_NEWTON_FUSED_UPDATE", "1")
    names = [op for op, _ in X.schedule(p, 2, 0, -1)]
    assert "newtonFupdate" not in names and names.count("axpy") == 2


@pytest.mark.parametrize("mode,dims,world", [(0, (64, 256, 64), 2), (0, (48, 256, 70), 3), (2, (255, 511, 63), 2),
                                             (2, (64, 128, 96), 3)])
def test_schedules_agree_on_collectives(mode, dims, world):
    """Every rank's schedule issues the same exchanges, gathers and norm reductions in the same order (a rank
    that skipped one — a rank-dependent branch in the driver — would deadlock or fail the real RCCL run)."""
    import zslab_exec as X
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=mode)
    seqs = []
    for r in range(world):
        ops = X.schedule(p, world, r, -1)
        seqs.append([(op, kv.get("L"), kv.get("field"), kv.get("depth"), kv.get("allgather"))
                     for op, kv in ops if op in ("halo", "gather", "norm")])
    assert all(s == seqs[0] for s in seqs[1:])


def _replay_newton_worker(rank, world, port, params, min_points, q, env):
    import zslab_exec as X
    os.environ.update(env)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops = X.schedule(params, world, rank, min_points)
        if env.get("GS_TEST_MUTATE"):
            ops = X.mutate(ops, env["GS_TEST_MUTATE"])
        R = X.Rank(params, rank, world, min_points)
        R.run(ops)
        lo, hi, v = R.owned_v("v")
        _, _, w = R.owned_v("newtonV")
        q.put((rank, lo, hi, v, w, R.newton_history, sorted({op for op, _ in ops})))
    except Exception:
        import traceback
        q.put((rank, None, None, None, None, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fused,stale", [(True, False), (True, True)])  # (fused False, the two-pass axpy path,
def test_gloo_replay_newton_schedule(fused, stale):                        # replays too: ~2 min more)
    """NEWTON's Z-slab schedule (NewtonSolver: newtonF, the inner solves, findError's newtonV += v — fused into
    the next compF with the new newtonV's ghost planes formed from both operands, or the two-pass axpy with
    GS_NO_NEWTON_FUSED_UPDATE — and the per-level newtonV restriction) replayed on two gloo ranks with the
    oracle's point expressions: Newton history, newtonV and v against the single-domain oracle solve. numpy's
    exp stands in for libm's, so the comparison is to 1e-10, not bit for bit. A power-of-two grid: its inner
    solves never meet their tol-0.1 exit, so the traced schedule — whose placeholder norms
    never stop a loop — runs the ten inner V-cycles the oracle runs. The inner solves read the GS_NEWTON_B
    factors ("bfac" ops, replayed as a snapshot of the newtonV each was computed from); stale: the schedule with
    the second iteration's level-0 factor dropped must NOT reproduce the oracle."""
    dims, world = ((64, 128, 64) if stale else (256, 512, 64)), 2
    params = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=2)
    # (the fused run also takes the NEWTON prolongation pair on every slab level: GS_NEWTON_PRO_POINTS=0)
    env = {"GS_NEWTON_PRO_POINTS": "0"} if fused else {"GS_NO_NEWTON_FUSED_UPDATE": "1"}
    if stale:
        env["GS_TEST_MUTATE"] = "bfac"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replay_newton_worker, args=(r, world, port, params, -1, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=900) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] is not None, r[5]
    og = O.Grid(dims, mode=O.NEWTON, maxiter=2)
    ref_hist = og.solve()
    ref_v, ref_w = og.field(0, "v").copy(), og.field(0, "newtonV").copy()
    if stale:
        same = all(all(abs(a - b) <= 1e-10 * abs(b) for a, b in zip(r[5], ref_hist)) for r in res)
        assert not same, "a stale GS_NEWTON_B factor went unnoticed"
        return
    for rank, lo, hi, v, w, hist, ops in res:
        assert ("newtonFupdate" in ops and "ghostsum" in ops) == fused and ("axpy" in ops) != fused, ops
        assert ("pro" in ops) == fused and "bfac" in ops, ops
        assert len(hist) == len(ref_hist)
        for a, b in zip(hist, ref_hist):
            assert abs(a - b) <= 1e-10 * abs(b), (a, b)
        np.testing.assert_allclose(w, ref_w[:, :, lo: hi + 1], rtol=0, atol=1e-10 * np.abs(ref_w).max())
        np.testing.assert_allclose(v, ref_v[:, :, lo: hi + 1], rtol=0, atol=1e-9 * np.abs(ref_v).max())
