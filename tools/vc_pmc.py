"""A few 512^3 linear 2+2 V-cycles (no bench extras) for per-kernel PMC passes:
    tools/pmc_run.sh <tag> tools/vc_pmc.py [n] [cycles]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 4
p = gsv.GridParams(maxiter=cycles, tol=0.0, gridDim=(n, n, n), mode=gsv.GS_LINEAR, preSmoothing=2, postSmoothing=2)
with gsv.HipGridData(p) as g:
    print(gsv.HipSolver.solve(g)[-1])
