"""One rank of a multi-process RCCL Z-slab solve (child process of tests/test_gpu_rccl_multirank.py).

    python rccl_rank_probe.py <out.npz> <rank> <world> <uid file> <mode> <nx> <ny> <nz> <maxiter> [die]

(`die`: the last rank leaves right after its communicator and slab exist — a peer lost mid-run;
`digest`: save a SHA-1 per owned z-plane of level 0's interior v instead of the planes — config #5's size.)

Rank 0 creates the RCCL id and publishes it through the file (gs_uid_publish, as GpuSolve-hip's launcher
path does), the others wait for it (gs_uid_await); every rank then builds its slab with
gs_grid_create_rccl — the call bench.py makes at N > 1 — solves, and saves its owned planes of level 0's
v with their global offset and the residual history. The parent sets a distinct NCCL_HOSTID per rank so
that RCCL accepts several ranks on one GPU (it refuses duplicate GPUs only among ranks of one host): the
ranks then talk through RCCL's socket transport over loopback instead of xGMI, but every byte of the
halo exchanges, the broadcast of replicated levels and the norm allgather goes through the product's
RCCL communicator (gs_comm.cpp)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402


def plane_digests(v):
    """SHA-1 of every z-plane's interior (x, y) values of a field indexed [x][y][z]."""
    import hashlib
    return [hashlib.sha1(np.ascontiguousarray(v[1:-1, 1:-1, k]).tobytes()).hexdigest() for k in range(v.shape[2])]


def main():
    out, rank, world, uidp, mode, nx, ny, nz, maxiter = sys.argv[1:10]
    rank, world, mode, maxiter = int(rank), int(world), int(mode), int(maxiter)
    drv = gsv.driver()
    uid = (C.c_ubyte * 128)()
    if rank == 0:
        assert drv.gs_rccl_unique_id(uid) == 0, drv.gs_last_error().decode()
        assert drv.gs_uid_publish(uidp.encode(), uid) == 0, drv.gs_last_error().decode()
    else:
        assert drv.gs_uid_await(uidp.encode(), 120.0, uid) == 0, drv.gs_last_error().decode()
    p = gsv.GridParams(maxiter=maxiter, tol=0.0, gridDim=(int(nx), int(ny), int(nz)), mode=mode)
    g = gsv.HipGridData.__new__(gsv.HipGridData)
    g.params = p
    g._abi_params = p.to_abi()
    g.handle = drv.gs_grid_create_rccl(C.byref(g._abi_params), rank, world, uid)
    if not g.handle:
        raise SystemExit("gs_grid_create_rccl: " + drv.gs_last_error().decode())
    if len(sys.argv) > 10 and sys.argv[10] == "die" and rank == world - 1:
        os._exit(3)
    try:
        hist = gsv.NewtonSolver.solve(g) if mode == 2 else gsv.HipSolver.solve(g)
        geom = g.getLevel(0).geom
        v = g.field(0, "v")[:, :, 1:geom.nz + 1]
        if len(sys.argv) > 10 and sys.argv[10] == "digest":
            np.savez(out, digests=np.array(plane_digests(v)), nz=geom.nz, z0=geom.z0,
                     hist=np.array(hist, dtype=np.float64))
        else:
            np.savez(out, v=v, z0=geom.z0, hist=np.array(hist, dtype=np.float64))
    finally:
        g.close()


if __name__ == "__main__":
    main()
