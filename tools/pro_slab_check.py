"""One Z-slab loopback solve (2 ranks, LINEAR, 2+2) for a kernel trace: under rocprofv3 the fused
prolongation pair (k_tb2y ... PRO) shows up once per rank and distributed fine level per cycle."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, "gpu-solve_amd")
import gpusolve as gsv  # noqa: E402

dims = (64, 128, 128)
p = gsv.GridParams(maxiter=4, tol=0.0, gridDim=dims, mode=0).to_abi()
v = np.zeros((dims[2] + 2, dims[1] + 2, dims[0] + 2))
hist = (C.c_double * 32)()
cnt = C.c_int(0)
d = gsv.driver()
rc = d.gs_zslab_loopback_run(C.byref(p), 2, -1, 0, 1, hist, 32, C.byref(cnt), v.ctypes.data_as(gsv._abi.dptr))
assert rc == 0, d.gs_last_error().decode()
print(list(hist[: cnt.value]))
