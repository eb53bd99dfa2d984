#!/usr/bin/env python3
"""k_rr2 vs k_rr2d (GS_RR_DMA, read once per process): times gs_residual_restrict alone on the bench-size levels
(512^3 LINEAR = the V-cycle's level 0, 256^3 LINEAR = its level 1, 512^3 GS_NEWTON_B / GS_NEWTON_G = the Newton
inner cycle's level 0) and prints a SHA-1 of each coarse result, so two runs (GS_RR_DMA=0 / 1) can be compared for
bit-identity.      python tools/rr_probe.py [--reps 20] [--rounds 3]
"""
import argparse
import ctypes as C
import hashlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    k = gsv.kernels()
    st = torch.cuda.current_stream()
    S = gsv.Stencil().to_abi()
    cases = [("linear512", 512, gsv.GS_LINEAR, 17.0), ("linear256", 256, gsv.GS_LINEAR, 17.0),
             ("newtonB512", 512, gsv.GS_NEWTON_B, 25.0), ("newtonG512", 512, gsv.GS_NEWTON_G, 17.0),
             ("linear511", 511, gsv.GS_LINEAR, 17.0)]
    env = os.environ.get("GS_RR_DMA", "default")
    for name, n, mode, bpp in cases:
        h = 1.0 / (n + 1)
        g = torch.Generator(device="cuda").manual_seed(n + mode)
        v, f, w = DevField(n, n, n), DevField(n, n, n), DevField(n, n, n)
        for fld, sc, off in ((v, 1e-3, 0.0), (f, 1.0, 0.0), (w, 0.1, 1.0)):
            inner = fld.zyx[1:-1, 1:-1, 1:n + 1]
            inner.copy_(torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) * sc + off)
        cd = n // 2
        ca = DevField(cd, cd, cd)
        L, Lc = v.level(h), ca.level(2 * h)
        wp = w.ptr if mode in (gsv.GS_NEWTON_B, gsv.GS_NEWTON_G, gsv.GS_NEWTON) else None

        def run():
            rc = k.gs_residual_restrict(C.byref(S), C.byref(L), mode, 1.0, v.ptr, f.ptr, wp, ca.ptr, None, C.byref(Lc),
                                        st.cuda_stream)
            assert rc == 0, rc
        run()
        torch.cuda.synchronize()
        digest = hashlib.sha1(ca.buf.cpu().numpy().tobytes()).hexdigest()[:16]
        best = None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            e0.record(st)
            for _ in range(a.reps):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            best = ms if best is None else min(best, ms)
        gbps = bpp * n ** 3 / (best * 1e-3) / 1e9
        print(f"GS_RR_DMA={env} {name:11s} {best:.4f} ms  {gbps:7.1f} GB/s ({bpp:.0f} B/pt) frac {gbps / 8000:.3f} "
              f"sha1 {digest}", flush=True)
        del v, f, w, ca


if __name__ == "__main__":
    main()
