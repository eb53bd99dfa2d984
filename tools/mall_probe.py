"""Does the Infinity Cache (256 MiB) carry planes from one fused-pair launch to the next when consecutive
launches march the planes in opposite orders? 512^3 LINEAR pairs ping-ponging v <-> vAlt as the solver's
smoother does: every launch ascending (the product), vs alternating ascending / descending
(gs_debug_pair_reverse: timing only, the descending launch swaps the z-terms of the sum).
    python tools/mall_probe.py [--size 512] [--pairs 20] [--rounds 5]"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--pairs", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    n = a.size
    kd = gsv.diag()
    S = gsv.GridParams(gridDim=(n, n, n)).stencil.to_abi()
    v, w, f = DevField(n, n, n), DevField(n, n, n), DevField(n, n, n)
    v.buf.uniform_(-1, 1)
    f.buf.uniform_(-1, 1)
    L = v.level(1.0 / (n + 1))
    st = torch.cuda.current_stream().cuda_stream

    def run(key):
        alternate, cached = "alternating" in key, "cached" in key
        src, dst = v, w
        for i in range(a.pairs):
            rc = kd.gs_debug_pair_reverse(C.byref(S), C.byref(L), 0.8, src.ptr, dst.ptr, f.ptr,
                                          (1 if (alternate and i % 2) else 0) | (2 if cached else 0), st)
            assert rc == 0, rc
            src, dst = dst, src

    res = {"ascending": [], "alternating": [], "ascending cached-stores": [], "alternating cached-stores": []}
    for _ in range(2):
        for key in res:
            run(key)
    for _ in range(a.rounds):
        for key in res:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(key)
            e1.record()
            torch.cuda.synchronize()
            res[key].append(e0.elapsed_time(e1) / a.pairs)
    out = {k: {"median_ms": round(statistics.median(x), 4), "all": [round(y, 4) for y in x]} for k, x in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
