#!/usr/bin/env python3
"""Kernel tuning bench: times every tiling variant of the LINEAR fused Jacobi sweep
(gs_debug_sweep_variant) in interleaved rounds in ONE process, checks each is bit-identical to the
production kernel, and measures the achievable HBM ceiling for the same byte pattern
(gs_debug_stream_triad: out = a + 0.8*b, 24 B per element).

    python tools/kbench.py [--n 512] [--rounds 5] [--sweeps 10] [--out gpurun_out/kbench.json]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--nz", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sweeps", type=int, default=10)
    ap.add_argument("--variants", type=str, default="")
    ap.add_argument("--out", type=str, default="")
    ap.add_argument("--bw", action="store_true", help="also sweep the streaming-ceiling kernels")
    ap.add_argument("--pairs", action="store_true", help="also time the fused-pair shape variants")
    ap.add_argument("--zc", type=str, default="0", help="fused-pair z-chunks to try (comma list, 0 = auto)")
    a = ap.parse_args()
    k = gsv.kernels()
    kd = gsv.diag()
    nx = a.n
    ny = a.ny or a.n
    nz = a.nz or a.n
    h = 1.0 / (ny + 1)
    st = torch.cuda.current_stream().cuda_stream
    S = gsv.Stencil().to_abi()

    f = DevField(nx, ny, nz)
    v = DevField(nx, ny, nz)
    alt = DevField(nx, ny, nz)
    L = v.level(h)
    assert k.gs_rhs_init(C.byref(L), f.ptr, 0, h, 1.0, st) == 0
    g = torch.Generator(device="cuda").manual_seed(5)
    inner = v.zyx[1:-1, 1:-1, 1:nx + 1]
    inner.copy_(torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) * 1e-3)
    torch.cuda.synchronize()

    nv = kd.gs_debug_num_variants()
    variants = [int(x) for x in a.variants.split(",")] if a.variants else list(range(nv))
    names = {i: kd.gs_debug_variant_name(i).decode() for i in range(nv)}

    # reference output: production kernel (gs_jacobi_sweep)
    ref = DevField(nx, ny, nz)
    assert k.gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, ref.ptr, f.ptr, None, st) == 0
    torch.cuda.synchronize()
    result = {"n": [nx, ny, nz], "build": gsv.build_info(), "variants": {}}
    for i in variants:
        alt.buf.fill_(float("nan"))
        alt.zyx[:, :, :].zero_() if False else None
        # the sweep writes the interior only: give alt the same zero boundary
        alt.buf.zero_()
        rc = kd.gs_debug_sweep_variant(i, C.byref(S), C.byref(L), 0.8, v.ptr, alt.ptr, f.ptr, st)
        assert rc == 0, k.gs_strerror(rc)
        torch.cuda.synchronize()
        same = bool(torch.equal(alt.zyx[:, :, :nx + 2], ref.zyx[:, :, :nx + 2]))
        result["variants"][names[i]] = {"id": i, "bitwise_equal_to_production": same, "ms": []}

    lups = float(nx) * ny * nz
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for r in range(a.rounds):
        for i in variants:
            a_, b_ = v, alt
            for _ in range(2):
                kd.gs_debug_sweep_variant(i, C.byref(S), C.byref(L), 0.8, a_.ptr, b_.ptr, f.ptr, st)
                a_, b_ = b_, a_
            ev[0].record()
            for _ in range(a.sweeps):
                kd.gs_debug_sweep_variant(i, C.byref(S), C.byref(L), 0.8, a_.ptr, b_.ptr, f.ptr, st)
                a_, b_ = b_, a_
            ev[1].record()
            torch.cuda.synchronize()
            result["variants"][names[i]]["ms"].append(ev[0].elapsed_time(ev[1]) / a.sweeps)
    for name, d in result["variants"].items():
        med = statistics.median(d["ms"])
        d["median_ms"] = round(med, 4)
        d["min_ms"] = round(min(d["ms"]), 4)
        d["glups"] = round(lups / med / 1e6, 2)
        d["gbps"] = round(24 * lups / med / 1e6, 1)
        d["pct_peak"] = round(100 * 24 * lups / med / 1e6 / PEAK, 1)
        del d["ms"]

    if a.pairs:
        # reference: two production single sweeps of the current v
        ref1, ref2 = DevField(nx, ny, nz), DevField(nx, ny, nz)
        assert k.gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, ref1.ptr, f.ptr, None, st) == 0
        assert k.gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, ref1.ptr, ref2.ptr, f.ptr, None, st) == 0
        torch.cuda.synchronize()
        pv = {}
        cases = [("production", -1, 0)] + [(kd.gs_debug_pair_variant_name(i).decode() + f" zc{zc}", i, int(zc))
                                            for i in range(kd.gs_debug_num_pair_variants())
                                            for zc in a.zc.split(",")]

        def launch(i, zc, src, dst):
            if i < 0:
                return k.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, src.ptr, dst.ptr, f.ptr, None, 0, 0, st)
            return kd.gs_debug_pair_variant(i, C.byref(S), C.byref(L), 0.8, src.ptr, dst.ptr, f.ptr, zc, st)
        for name, i, zc in cases:
            alt.buf.zero_()
            rc = launch(i, zc, v, alt)
            if rc != 0:
                continue
            torch.cuda.synchronize()
            pv[name] = {"bitwise_equal_to_two_sweeps": bool(torch.equal(alt.zyx[:, :, :nx + 2],
                                                                         ref2.zyx[:, :, :nx + 2])), "ms": []}
        for r in range(a.rounds):
            for name, i, zc in cases:
                if name not in pv:
                    continue
                a_, b_ = v, alt
                launch(i, zc, a_, b_)
                ev[0].record()
                for _ in range(a.sweeps):
                    launch(i, zc, a_, b_)
                    a_, b_ = b_, a_
                ev[1].record()
                torch.cuda.synchronize()
                pv[name]["ms"].append(ev[0].elapsed_time(ev[1]) / a.sweeps)
        for name, d in pv.items():
            med = statistics.median(d["ms"])
            d["median_ms_per_pair"] = round(med, 4)
            d["gbps_24B"] = round(24 * lups / med / 1e6, 1)
            d["glups"] = round(2 * lups / med / 1e6, 1)
            del d["ms"]
        result["pairs"] = pv

    # achievable ceiling for the same byte pattern (2 streamed reads + 1 streamed write)
    n = (v.span // 2) * 2
    A = torch.rand(n, dtype=torch.float64, device="cuda")
    B = torch.rand(n, dtype=torch.float64, device="cuda")
    O = torch.empty(n, dtype=torch.float64, device="cuda")
    for _ in range(3):
        kd.gs_debug_stream_triad(O.data_ptr(), A.data_ptr(), B.data_ptr(), n, st)
    ts = []
    for _ in range(a.rounds):
        ev[0].record()
        for _ in range(a.sweeps):
            kd.gs_debug_stream_triad(O.data_ptr(), A.data_ptr(), B.data_ptr(), n, st)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) / a.sweeps)
    med = statistics.median(ts)
    result["triad"] = {"elements": n, "median_ms": round(med, 4), "gbps": round(24 * n / med / 1e6, 1),
                       "pct_peak": round(100 * 24 * n / med / 1e6 / PEAK, 1)}
    if a.bw:
        sink = torch.zeros(1, dtype=torch.float64, device="cuda")
        bytes_per = {0: 8, 1: 8, 2: 16, 3: 24}
        names_k = {0: "read", 1: "write", 2: "copy", 3: "triad"}
        bw = {}
        for kind in (0, 1, 2, 3):
            for unroll in (1, 4):
                for nt in (0, 1):
                    for blocks in (1024, 2048, 4096, 8192, 16384):
                        def run():
                            kd.gs_debug_bw(kind, unroll, nt, blocks, O.data_ptr(), A.data_ptr(), B.data_ptr(), n,
                                          sink.data_ptr(), st)
                        run()
                        ts = []
                        for _ in range(3):
                            ev[0].record()
                            for _ in range(a.sweeps):
                                run()
                            ev[1].record()
                            torch.cuda.synchronize()
                            ts.append(ev[0].elapsed_time(ev[1]) / a.sweeps)
                        med = statistics.median(ts)
                        bw[f"{names_k[kind]} u{unroll} nt{nt} b{blocks}"] = round(bytes_per[kind] * n / med / 1e6, 1)
        result["bw"] = bw
        best = {}
        for key, val in bw.items():
            kk = key.split()[0]
            if val > best.get(kk, (0, ""))[0]:
                best[kk] = (val, key)
        result["bw_best"] = best
    # torch's own copy as a second reference point
    for _ in range(2):
        O.copy_(A)
    ev[0].record()
    for _ in range(a.sweeps):
        O.copy_(A)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.sweeps
    result["torch_copy"] = {"gbps": round(16 * n / ms / 1e6, 1)}
    js = json.dumps(result, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(js)


if __name__ == "__main__":
    main()
