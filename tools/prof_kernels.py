"""Minimal launcher for counter collection: the level-0 smoother kernels of bench.py's workload
(512^3 linear) launched back to back, nothing else on the GPU.

    rocprofv3 --pmc <counters> -d <dir> -o run --output-format csv -- python tools/prof_kernels.py
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--which", default="pair,single,residual")
    ap.add_argument("--pair-variants", default="", help="also launch these gs_debug_pair_variant ids")
    ap.add_argument("--zc", type=int, default=0, help="z-chunk of the pair variants (0 = auto)")
    a = ap.parse_args()
    n = a.size
    kl = gsv.kernels()
    kd = gsv.diag()
    p = gsv.GridParams(gridDim=(n, n, n))
    S = p.stencil.to_abi()
    v, v2, f, r = (DevField(n, n, n) for _ in range(4))
    g = torch.Generator(device="cuda").manual_seed(1)
    for d in (v, f):
        d.buf.copy_(torch.rand(d.buf.shape, generator=g, device="cuda", dtype=torch.float64))
    L = v.level(1.0 / (n + 1))
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(a.reps):
        if "pair" in a.which:
            assert kl.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, v2.ptr, f.ptr, None, 0, 0, st) == 0
        if "single" in a.which:
            assert kl.gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, v2.ptr, f.ptr, None, st) == 0
        for i in filter(None, a.pair_variants.split(",")):
            assert kd.gs_debug_pair_variant(int(i), C.byref(S), C.byref(L), 0.8, v.ptr, v2.ptr, f.ptr, a.zc, st) == 0
        if "rr" in a.which.split(","):
            c = DevField(n // 2, n // 2, n // 2)
            Lc = c.level(2.0 / (n + 1))
            assert kl.gs_residual_restrict(C.byref(S), C.byref(L), 0, 1.0, v.ptr, f.ptr, None, c.ptr, None,
                                           C.byref(Lc), st) == 0
        if "residual" in a.which:
            assert kl.gs_residual(C.byref(S), C.byref(L), 0, 1.0, v.ptr, f.ptr, None, r.ptr, None, st) == 0
    torch.cuda.synchronize()
    print("ok", n, a.reps, a.which)


if __name__ == "__main__":
    main()
