"""CPU coverage of the Z-slab decomposition:

1. the ownership plan (gs_zslab_plan, the driver's own host code) covers every plane exactly once
   on every level, honours the "coarse plane zc belongs to the owner of fine plane 2 zc" rule, and
   keeps every stencil / transfer read inside [lo-1, hi+1] (one ghost plane);
2. a world_size-2 torch.distributed (gloo) run of the slab protocol — sweeps on slabs with one
   ghost plane, ghost exchange after every write, rank-ordered norm — reproduces the single-domain
   oracle bit for bit. The per-slab arithmetic is the oracle's; the schedule mirrors
   HipSolver::jacobi / finishNorm.
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


def _slab_worker(rank, world, port, dims, sweeps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nx, ny, nz = dims
    _, distributed, own = plan(dims, world)
    lo, hi = own[0][rank]
    h = 1.0 / (ny + 1)
    f_full = O.rhs(nx, ny, nz, O.LINEAR)
    rng = np.random.default_rng(1)
    v_full = O.zeros(nx, ny, nz)
    v_full[1:-1, 1:-1, 1:-1] = rng.uniform(-1, 1, (nx, ny, nz))
    # slab with one ghost plane each side (reference layout: z is the last axis)
    v = np.ascontiguousarray(v_full[:, :, lo - 1: hi + 2])
    f = np.ascontiguousarray(f_full[:, :, lo - 1: hi + 2])
    nzl = hi - lo + 1

    def halo(a):
        reqs = []
        recv_lo = torch.zeros(a.shape[0] * a.shape[1], dtype=torch.float64)
        recv_hi = torch.zeros_like(recv_lo)
        if rank > 0:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a[:, :, 1]).ravel()), rank - 1))
            reqs.append(dist.irecv(recv_lo, rank - 1))
        if rank + 1 < world:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a[:, :, nzl]).ravel()), rank + 1))
            reqs.append(dist.irecv(recv_hi, rank + 1))
        for r_ in reqs:
            r_.wait()
        if rank > 0:
            a[:, :, 0] = recv_lo.numpy().reshape(a.shape[0], a.shape[1])
        if rank + 1 < world:
            a[:, :, nzl + 1] = recv_hi.numpy().reshape(a.shape[0], a.shape[1])

    for _ in range(sweeps):
        v = O.jacobi(v, f, h, O.LINEAR, 0.8, 1.0, 1)  # one sweep on the slab (ghosts are read-only)
        halo(v)
    _, n = O.residual(v, f, h, O.LINEAR)
    part = torch.tensor([n * n], dtype=torch.float64)
    allp = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(allp, part)
    total = 0.0
    for t in allp:  # rank order, as HipSolver::finishNorm
        total += t.item()
    q.put((rank, lo, hi, v[:, :, 1: nzl + 1].copy(), float(np.sqrt(total))))
    dist.destroy_process_group()


def test_gloo_two_rank_slab_sweeps():
    dims, sweeps, world = (23, 18, 30), 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_worker, args=(r, world, port, dims, sweeps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nx, ny, nz = dims
    f_full = O.rhs(nx, ny, nz, O.LINEAR)
    rng = np.random.default_rng(1)
    v_full = O.zeros(nx, ny, nz)
    v_full[1:-1, 1:-1, 1:-1] = rng.uniform(-1, 1, (nx, ny, nz))
    ref = O.jacobi(v_full, f_full, 1.0 / (ny + 1), O.LINEAR, 0.8, 1.0, sweeps)
    _, ref_norm = O.residual(ref, f_full, 1.0 / (ny + 1), O.LINEAR)
    got = O.zeros(nx, ny, nz)
    for rank, lo, hi, slab, norm in res:
        got[:, :, lo: hi + 1] = slab
        assert abs(norm - ref_norm) <= 1e-13 * ref_norm
    np.testing.assert_array_equal(got, ref)
