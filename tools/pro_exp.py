"""Timing-only: the 512^3 level-0 prolongation pair and the plain pair from the product library and
from the GS_PRO_EXP builds (tools/pro_exp_build.sh; exp4 = GS_PRO_HALF=0, whose output must equal the
product's bit for bit), interleaved, HIP events on one stream.
    python tools/pro_exp.py [reps]"""
import ctypes as C
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve import _abi  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
libs = {"prod": gsv.kernels()}
for e in (1, 2, 3, 4):
    p = os.path.join(HERE, "..", "gpu-solve_amd", "build", "exp", f"libgs_exp{e}.so")
    if os.path.exists(p):
        lib = C.CDLL(p, mode=C.RTLD_LOCAL)
        for name in ("gs_jacobi_sweep2_prolong", "gs_jacobi_sweep2", "gs_residual_restrict"):
            res, args = _abi.KERNEL_API[name]
            getattr(lib, name).restype, getattr(lib, name).argtypes = res, args
        libs[f"exp{e}"] = lib

n = 512
prm = gsv.GridParams(maxiter=2, tol=0.0, gridDim=(n, n, n), mode=0)
out = {}
with gsv.HipGridData(prm) as grid:
    gsv.HipSolver.solve(grid)
    drv = gsv.driver()
    L0, L1 = grid.getLevel(0).geom, grid.getLevel(1).geom
    S = prm.stencil.to_abi()
    v, f = drv.gs_grid_field(grid.handle, 0, 0), drv.gs_grid_field(grid.handle, 0, 3)
    cv = drv.gs_grid_field(grid.handle, 1, 0)
    o = DevField(L0.nx, L0.ny, L0.nz)
    st = grid.stream()
    stream = torch.cuda.ExternalStream(st)

    def timed(fn, k=20):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    for r in range(reps):
        for name, lib in libs.items():
            def pro():
                assert lib.gs_jacobi_sweep2_prolong(C.byref(S), C.byref(L0), 0, prm.omega, prm.gamma, v, cv, None,
                                                    C.byref(L1), o.ptr, f, None, 0, 0, st) == 0

            def pair():
                assert lib.gs_jacobi_sweep2(C.byref(S), C.byref(L0), 0, prm.omega, prm.gamma, v, o.ptr, f, None,
                                            0, 0, st) == 0
            def rr():
                assert lib.gs_residual_restrict(C.byref(S), C.byref(L0), 0, prm.gamma, v, f, None, o.ptr, None,
                                                C.byref(L1), st) == 0
            for kind, fn in (("pro", pro), ("pair", pair), ("rr", rr)):
                ms = timed(fn)
                out.setdefault(f"{name}_{kind}", []).append(round(ms, 4))
                print(f"rep {r} {name:5s} {kind:4s} {ms:.4f} ms", flush=True)
    if "exp4" in libs:  # the A/B pair of builds computes the same bits
        res = {}
        for name in ("prod", "exp4"):
            assert libs[name].gs_jacobi_sweep2_prolong(C.byref(S), C.byref(L0), 0, prm.omega, prm.gamma, v, cv, None,
                                                       C.byref(L1), o.ptr, f, None, 0, 0, st) == 0
            torch.cuda.synchronize()
            res[name] = o.to_xyz().copy()
        same = res["prod"].tobytes() == res["exp4"].tobytes()
        out["prod_vs_exp4_bit_identical"] = [same]
        print("prod vs exp4 (GS_PRO_HALF=0) bit-identical:", same, flush=True)
    del o
print(json.dumps({k: sorted(v)[len(v) // 2] for k, v in out.items()}))
