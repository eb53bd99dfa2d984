"""Child process of tests/test_gpu_switches.py: one solve under the environment it was started with
(the library reads its A/B switches once per process), level 0's iterate and the history saved to an
.npz.   python tests/switch_probe.py <out.npz> <mode> <nx> <ny> <nz> <maxiter> [pre post]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402

out, mode, nx, ny, nz, maxiter = sys.argv[1], *map(int, sys.argv[2:7])
pre, post = (int(sys.argv[7]), int(sys.argv[8])) if len(sys.argv) > 8 else (2, 2)
p = gsv.GridParams(maxiter=maxiter, tol=0.0, gridDim=(nx, ny, nz), mode=mode, preSmoothing=pre, postSmoothing=post)
with gsv.HipGridData(p) as g:
    hist = gsv.NewtonSolver.solve(g) if mode == gsv.GS_NEWTON else gsv.HipSolver.solve(g)
    v = g.field(0, "newtonV" if mode == gsv.GS_NEWTON else "v")
np.savez(out, v=v, hist=np.array(hist))
