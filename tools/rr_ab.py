#!/usr/bin/env python3
"""A/B of the level-0 residual + restriction (gs_residual_restrict, LINEAR, 512^3 -> 256^3) between the
in-tree kernel library and another build of it (argv[1], linked -Wl,-Bsymbolic), interleaved rounds in
one process, outputs compared bit for bit.   python tools/rr_ab.py gpu-solve_amd/lib_ab/libgpusolve_hip_old.so
"""
import ctypes as C
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve._abi import KERNEL_API  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def main():
    new = gsv.kernels()
    old = C.CDLL(os.path.abspath(sys.argv[1]), mode=C.RTLD_LOCAL)
    for name, (res, args) in KERNEL_API.items():
        if hasattr(old, name):
            getattr(old, name).restype = res
            getattr(old, name).argtypes = args
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    nc = n // 2
    h, hc = 1.0 / (n + 1), 1.0 / (nc + 1)
    st = torch.cuda.current_stream().cuda_stream
    S = gsv.Stencil().to_abi()
    v, f = DevField(n, n, n), DevField(n, n, n)
    ca, cb = DevField(nc, nc, nc), DevField(nc, nc, nc)
    L, Lc = v.level(h), ca.level(hc)
    assert new.gs_rhs_init(C.byref(L), f.ptr, 0, h, 1.0, st) == 0
    g = torch.Generator(device="cuda").manual_seed(7)
    inner = v.zyx[1:-1, 1:-1, 1:n + 1]
    inner.copy_(torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) * 1e-3)

    def run(lib, out):
        rc = lib.gs_residual_restrict(C.byref(S), C.byref(L), 0, 1.0, v.ptr, f.ptr, None, out.ptr, None,
                                      C.byref(Lc), st)
        assert rc == 0, rc
    run(new, ca)
    run(old, cb)
    torch.cuda.synchronize()
    same = bool(torch.equal(ca.buf, cb.buf))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t = {"new": [], "old": []}
    for _ in range(7):
        for name, lib in (("new", new), ("old", old)):
            run(lib, ca)
            ev[0].record()
            for _ in range(10):
                run(lib, ca)
            ev[1].record()
            torch.cuda.synchronize()
            t[name].append(ev[0].elapsed_time(ev[1]) / 10)
    for name, xs in t.items():
        med = statistics.median(xs)
        print(f"rr {n}^3 {name}: median {med:.4f} ms  min {min(xs):.4f}  {16 * n ** 3 / med / 1e6:.0f} GB/s (16 B/pt)")
    print("bitwise_equal", same)

    # the production fused pair (gs_jacobi_sweep2) of both builds
    a1, a2 = DevField(n, n, n), DevField(n, n, n)

    def pair(lib, src, dst):
        rc = lib.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, src.ptr, dst.ptr, f.ptr, None, 0, 0, st)
        assert rc == 0, rc
    pair(new, v, a1)
    pair(old, v, a2)
    torch.cuda.synchronize()
    same = bool(torch.equal(a1.buf, a2.buf))
    t = {"new": [], "old": []}
    for _ in range(7):
        for name, lib in (("new", new), ("old", old)):
            pair(lib, v, a1)
            ev[0].record()
            for i in range(10):
                pair(lib, a1 if i % 2 else a2, a2 if i % 2 else a1)
            ev[1].record()
            torch.cuda.synchronize()
            t[name].append(ev[0].elapsed_time(ev[1]) / 10)
    for name, xs in t.items():
        med = statistics.median(xs)
        print(f"pair {n}^3 {name}: median {med:.4f} ms  min {min(xs):.4f}  {24 * n ** 3 / med / 1e6:.0f} GB/s (24 B/pt)")
    print("bitwise_equal", same)

    # NEWTON: the fused prolongation pair (gs_jacobi_sweep2_prolong, mode 2) of both builds
    w = DevField(n, n, n)
    inner = w.zyx[1:-1, 1:-1, 1:n + 1]
    inner.copy_(torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) * 1e-2)
    c = DevField(nc, nc, nc)
    cin = c.zyx[1:-1, 1:-1, 1:nc + 1]
    cin.copy_(torch.rand(cin.shape, generator=g, device="cuda", dtype=torch.float64) * 1e-3)
    Lc2 = c.level(hc)

    for mode, label in ((0, "linear"), (2, "newton")):
        def pro(lib, src, dst):
            rc = lib.gs_jacobi_sweep2_prolong(C.byref(S), C.byref(L), mode, 0.8, 1.0, src.ptr, c.ptr, None,
                                              C.byref(Lc2), dst.ptr, f.ptr, w.ptr if mode == 2 else None, 0, 0, st)
            assert rc == 0, rc
        pro(new, v, a1)
        pro(old, v, a2)
        torch.cuda.synchronize()
        same = bool(torch.equal(a1.buf, a2.buf))
        t = {"new": [], "old": []}
        for _ in range(5):
            for name, lib in (("new", new), ("old", old)):
                pro(lib, v, a1)
                ev[0].record()
                for i in range(6):
                    pro(lib, v, a1 if i % 2 else a2)
                ev[1].record()
                torch.cuda.synchronize()
                t[name].append(ev[0].elapsed_time(ev[1]) / 6)
        for name, xs in t.items():
            med = statistics.median(xs)
            print(f"{label} prolongation pair {n}^3 {name}: median {med:.4f} ms  min {min(xs):.4f}")
        print("bitwise_equal", same)

if __name__ == "__main__":
    main()
