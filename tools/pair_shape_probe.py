#!/usr/bin/env python3
"""The LINEAR pair in other occupancy shapes (r06, verdict r05 item 2: close the pair to 0.70 of 8 TB/s).

The production pair (k_tb2y: 4 x-waves x 2 mirrored y-waves of 2 rows, two plane steps of prefetch, 210 VGPRs, one
8-wave block per CU = two waves per SIMD) against the same kernel at one row per y-wave, whose register budget fits
128 VGPRs, so that TWO blocks share a CU (four waves per SIMD: one block's arithmetic under the other's loads, and
the two blocks are not coupled by a barrier). gs_debug_pair_shape launches it (libgpusolve_diag.so); every shape's
output is compared bit for bit with gs_jacobi_sweep2's. GB/s at 24 B per point.

    python tools/pair_shape_probe.py [--n 512] [--rounds 3] [--reps 10] [--out f.json]
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
    ap.add_argument("--shapes", default="1,1,4,256;1,1,4,128;1,1,4,64;1,1,0,512;1,2,4,256;1,2,0,512;2,2,0,256;2,1,0,256")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    n = a.n
    k, kd = gsv.kernels(), gsv.diag()
    st = torch.cuda.current_stream()
    S = gsv.Stencil().to_abi()
    h = 1.0 / (n + 1)
    v, f, o, ref = DevField(n, n, n), DevField(n, n, n), DevField(n, n, n), DevField(n, n, n)
    L = v.level(h)
    assert k.gs_rhs_init(C.byref(L), f.ptr, 0, h, 1.0, st.cuda_stream) == 0
    g = torch.Generator(device="cuda").manual_seed(5)
    inner = v.zyx[1:-1, 1:-1, 1:n + 1]
    inner.copy_(torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) * 1e-3)
    prod = lambda out: k.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, out.ptr, f.ptr, None, 0, 0,
                                          st.cuda_stream)
    assert prod(ref) == 0
    torch.cuda.synchronize()
    cases = {"production pair (gs_jacobi_sweep2)": lambda: prod(o)}
    ident = {}
    for spec in a.shapes.split(";"):
        ry, pfd, wpe, zc = (int(x) for x in spec.split(","))
        name = f"ry{ry} pfd{pfd} wpe{wpe} zc{zc}"
        fn = (lambda ry=ry, pfd=pfd, wpe=wpe, zc=zc:
              kd.gs_debug_pair_shape(C.byref(S), C.byref(L), 0.8, v.ptr, o.ptr, f.ptr, ry, pfd, wpe, zc,
                                     st.cuda_stream))
        o.buf.zero_()
        rc = fn()
        torch.cuda.synchronize()
        if rc != 0:
            print(f"{name}: rc {rc}, skipped")
            continue
        ident[name] = bool(torch.equal(o.buf, ref.buf))
        cases[name] = fn
    res = {name: [] for name in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
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
    b = 24.0 * n ** 3
    for name, ms in res.items():
        best = min(ms)
        out[name] = {"ms": [round(x, 4) for x in ms], "gbps_best": round(b / (best * 1e-3) / 1e9, 1),
                     "frac_best": round(b / (best * 1e-3) / 8e12, 4), "bit_identical": ident.get(name, True)}
        print(f"{name:40s} {best:8.4f} ms  {b / (best * 1e-3) / 1e9:8.1f} GB/s  identical={ident.get(name, True)}")
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
