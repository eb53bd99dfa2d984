#!/usr/bin/env python3
"""Where does the LINEAR pair lose against the flat triad? (verdict r05 item 2, r06)

Times, interleaved in one process on the bench grid (512^3 padded fields), the production pair (k_tb2y,
gs_jacobi_sweep2), its memory skeleton without arithmetic (gs_debug_march: the same tiles, z-march, loads and
stores; variants of prefetch depth, per-step barrier, store / f-load policy, z-chunk length) and the flat
streaming triad (gs_debug_bw, the guide's shape). GB/s at 24 B per point.

    python tools/march_probe.py [--n 512] [--rounds 3] [--reps 10]
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--variants", default="", help="pfd,bar,nts,ntf,zc;... (default: the r06e set)")
    a = ap.parse_args()
    n = a.n
    k, kd = gsv.kernels(), gsv.diag()
    st = torch.cuda.current_stream()
    S = gsv.Stencil().to_abi()
    h = 1.0 / (n + 1)
    v, f, o = DevField(n, n, n), DevField(n, n, n), DevField(n, n, n)
    L = v.level(h)
    assert k.gs_rhs_init(C.byref(L), f.ptr, 0, h, 1.0, st.cuda_stream) == 0
    g = torch.Generator(device="cuda").manual_seed(5)
    inner = v.zyx[1:-1, 1:-1, 1:n + 1]
    inner.copy_(torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) * 1e-3)
    m = n * n * n
    A = torch.rand(m, dtype=torch.float64, device="cuda")
    B = torch.rand(m, dtype=torch.float64, device="cuda")
    O = torch.empty(m, dtype=torch.float64, device="cuda")
    sink = torch.zeros(1, dtype=torch.float64, device="cuda")
    cases = {"pair (k_tb2y)": lambda: k.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, o.ptr, f.ptr,
                                                          None, 0, 0, st.cuda_stream),
             "triad flat nt": lambda: kd.gs_debug_bw(3, 1, 1, 0, O.data_ptr(), A.data_ptr(), B.data_ptr(), m,
                                                     sink.data_ptr(), st.cuda_stream),
             "copy flat nt (16 B/elem)": lambda: kd.gs_debug_bw(2, 1, 1, 0, O.data_ptr(), A.data_ptr(), None, m,
                                                                sink.data_ptr(), st.cuda_stream)}
    variants = [(2, 1, 1, 0, zc) for zc in (256, 128)] + \
               [(2, 1, 1, 6, zc) for zc in (512, 256, 128)] + [(1, 1, 1, 7, zc) for zc in (256, 128, 64)]
    if a.variants:
        variants = [tuple(int(x) for x in v.split(",")) for v in a.variants.split(";")]
    for pfd, bar, nts, ntf, zc in variants:
        tag = {0: "", 1: " nt-f", 2: " LEAN", 3: " sync2", 4: " sync4", 5: " sync8", 6: " RY1", 7: " RY4"}[ntf]
        name = f"march pfd{pfd} bar{bar} {'nt' if nts else 'plain'}-st zc{zc}{tag}"
        cases[name] = (lambda pfd=pfd, bar=bar, nts=nts, ntf=ntf, zc=zc:
                       kd.gs_debug_march(pfd, bar, nts, ntf, zc, C.byref(L), v.ptr, f.ptr, o.ptr, st.cuda_stream))
    res = {name: [] for name in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for name, fn in cases.items():
            for _ in range(2):
                assert fn() == 0, name
            e0.record(st)
            for _ in range(a.reps):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / a.reps)
    out = {}
    for name, ms in res.items():
        b = (16.0 if "copy" in name else 24.0) * m
        best = min(ms)
        out[name] = {"ms": [round(x, 4) for x in ms], "gbps_best": round(b / (best * 1e-3) / 1e9, 1)}
        print(f"{name:40s} {best:8.4f} ms  {b / (best * 1e-3) / 1e9:8.1f} GB/s")
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
