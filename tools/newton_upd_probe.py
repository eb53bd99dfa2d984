"""The Newton update pass alone at 512^3: gs_newton_F_update (k_newton_upd, w' = w + e and f = F - N(w')) and,
for comparison, gs_newton_F (compF, k_rb KIND 1) and gs_axpy, each timed over `reps` launches with HIP events.
Run once per GS_NEWTON_UPD_XCD value (the library reads it when it loads).
    python tools/newton_upd_probe.py [n] [reps]"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
k = gsv.kernels()
S = gsv.GridParams(gridDim=(n, n, n)).stencil.to_abi()
w, e, F, wo, f = (DevField(n, n, n) for _ in range(5))
for a in (w, e, F):
    a.buf.uniform_(-0.5, 0.5)
L = w.level(1.0 / (n + 1))
np_ = k.gs_residual_num_partials(C.byref(S), C.byref(L))
parts = torch.zeros(np_, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


res = {"GS_NEWTON_UPD_XCD": os.environ.get("GS_NEWTON_UPD_XCD", "1"),
       "newton_F_update_ms": timed(lambda: k.gs_newton_F_update(C.byref(S), C.byref(L), 1.0, w.ptr, e.ptr, F.ptr, wo.ptr,
                                                                f.ptr, parts.data_ptr(), st)),
       "newton_F_ms": timed(lambda: k.gs_newton_F(C.byref(S), C.byref(L), 1.0, w.ptr, F.ptr, f.ptr, parts.data_ptr(), st)),
       "axpy_ms": timed(lambda: k.gs_axpy(wo.ptr, e.ptr, 1.0, wo.span, st))}
res["update_GBps_40B"] = round(40 * n ** 3 / res["newton_F_update_ms"] / 1e6, 1)
print(json.dumps(res))
