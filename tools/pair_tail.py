"""How evenly the blocks of one pair launch finish: per-block start / end wall clock (100 MHz) of the
production 512^3 LINEAR pair (gs_debug_pair_timestamps, libgpusolve_diag.so), per z-chunk length.

    python tools/pair_tail.py [--size 512] [--zc 0,128,64] [--reps 5] [--out gpurun_out/tail.json]
Prints, per chunk length: launch ms (HIP events), block duration min / median / max, the spread of start and end
times, and the mean end time per XCD (hardware block index % 8)."""
import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import ctypes as C  # noqa: E402
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--zc", default="0")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    n = a.size
    kd = gsv.diag()
    p = gsv.GridParams(gridDim=(n, n, n))
    S = p.stencil.to_abi()
    v, o, f = DevField(n, n, n), DevField(n, n, n), DevField(n, n, n)
    v.buf.uniform_(-1, 1)
    f.buf.uniform_(-1, 1)
    L = v.level(1.0 / (n + 1))
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for zc in (int(z) for z in a.zc.split(",")):
        nb = kd.gs_debug_pair_blocks(C.byref(S), C.byref(L), zc)
        ts = torch.zeros(4 * nb, dtype=torch.float64, device="cuda")
        rows = []
        for rep in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = kd.gs_debug_pair_timestamps(C.byref(S), C.byref(L), 0.8, v.ptr, o.ptr, f.ptr, zc, ts.data_ptr(), st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            if rep < 2:
                continue
            t = ts.view(nb, 4).cpu().numpy()
            t0 = t[:, 0].min()
            start, end = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # us
            dur = end - start
            xcd = (t[:, 2].astype(np.int64) % 8)
            rows.append({"launch_ms": e0.elapsed_time(e1), "start_spread_us": float(start.max()),
                         "end_min_us": float(end.min()), "end_median_us": float(np.median(end)),
                         "end_max_us": float(end.max()), "dur_min_us": float(dur.min()),
                         "dur_median_us": float(np.median(dur)), "dur_max_us": float(dur.max()),
                         "end_p90_us": float(np.percentile(end, 90)),
                         "xcd_mean_end_us": [float(end[xcd == i].mean()) for i in range(8)]})
        agg = {k: statistics.median(r[k] for r in rows) for k in rows[0] if k != "xcd_mean_end_us"}
        agg["xcd_mean_end_us"] = rows[-1]["xcd_mean_end_us"]
        agg["blocks"] = nb
        res[f"zc{zc}"] = agg
        print(f"zc={zc} blocks={nb}", json.dumps({k: (round(x, 1) if isinstance(x, float) else x) for k, x in agg.items()}))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
