"""Level-0 pre-smoothing + restriction at n^3 (default 512): the fused pass (gs_jacobi_sweep2_restrict)
against the two-pass path it replaces (gs_jacobi_sweep2_norm + gs_residual_restrict), HIP-event
timed on one stream, interleaved rounds. Prints one JSON line."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
k = gsv.kernels()
kd = gsv.diag()
S = gsv.Stencil().to_abi()
h = 1.0 / (n + 1)
v, f, out = DevField(n, n, n, fill=0.5), DevField(n, n, n, fill=1.0), DevField(n, n, n)
c = DevField(n // 2, n // 2, n // 2)
L, CL = v.level(h), c.level(2 * h)
p1 = torch.zeros(k.gs_jacobi_sweep2_num_partials(C.byref(S), C.byref(L), 0), dtype=torch.float64, device="cuda")
p2 = torch.zeros(kd.gs_jacobi_sweep2_restrict_num_partials(C.byref(S), C.byref(L), C.byref(CL)), dtype=torch.float64,
                 device="cuda")
st = torch.cuda.current_stream()


def two():
    assert k.gs_jacobi_sweep2_norm(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, out.ptr, f.ptr, None, 0, 0,
                                   p1.data_ptr(), st.cuda_stream) == 0
    assert k.gs_residual_restrict(C.byref(S), C.byref(L), 0, 1.0, out.ptr, f.ptr, None, c.ptr, None, C.byref(CL),
                                  st.cuda_stream) == 0


def fused():
    assert kd.gs_jacobi_sweep2_restrict(C.byref(S), C.byref(L), 0.8, v.ptr, out.ptr, f.ptr, p2.data_ptr(), c.ptr,
                                       None, C.byref(CL), st.cuda_stream) == 0


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for fn in (two, fused, two, fused):
    fn()
torch.cuda.synchronize()
res = {"two": [], "fused": []}
for _ in range(3):
    res["two"].append(timed(two))
    res["fused"].append(timed(fused))
t2, tf = min(res["two"]), min(res["fused"])
pts = float(n) ** 3
print(json.dumps({"n": n, "two_pass_ms": round(t2, 4), "fused_ms": round(tf, 4),
                  "fused_GBps_25B": round(25 * pts / (tf * 1e-3) / 1e9, 1), "saving_ms": round(t2 - tf, 4),
                  "rounds": res}))
