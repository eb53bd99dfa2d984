"""Child process of tests/test_gpu_switches.py: one solve under the environment it was started with
(the library reads its A/B switches once per process), level 0's iterate and the history saved to an
.npz.   python tests/switch_probe.py <out.npz> <mode> <nx> <ny> <nz> <maxiter> [pre post [ranks]]
ranks > 1: the Z-slab solve of that many loopback ranks on this device (gs_zslab_loopback_run), the
assembled level-0 v."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402

out, mode, nx, ny, nz, maxiter = sys.argv[1], *map(int, sys.argv[2:7])
pre, post = (int(sys.argv[7]), int(sys.argv[8])) if len(sys.argv) > 8 else (2, 2)
ranks = int(sys.argv[9]) if len(sys.argv) > 9 else 1
p = gsv.GridParams(maxiter=maxiter, tol=0.0, gridDim=(nx, ny, nz), mode=mode, preSmoothing=pre, postSmoothing=post)
if ranks > 1:
    d = gsv.driver()
    ap = p.to_abi()
    v = np.zeros((nz + 2, ny + 2, nx + 2))
    hist = (C.c_double * (maxiter + 1))()
    cnt = C.c_int(0)
    rc = d.gs_zslab_loopback_run(C.byref(ap), ranks, -1, 0, 1, hist, maxiter + 1, C.byref(cnt),
                                 v.ctypes.data_as(gsv._abi.dptr))
    assert rc == 0, d.gs_last_error().decode()
    np.savez(out, v=v, hist=np.array(hist[: cnt.value]))
    sys.exit(0)
with gsv.HipGridData(p) as g:
    hist = gsv.NewtonSolver.solve(g) if mode == gsv.GS_NEWTON else gsv.HipSolver.solve(g)
    v = g.field(0, "newtonV" if mode == gsv.GS_NEWTON else "v")
np.savez(out, v=v, hist=np.array(hist))
