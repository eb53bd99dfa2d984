"""Regenerate profiles/config5_single_gpu.json — the driver's one-GPU 1024^3 MLUPS, the SECONDARY denominator of
the N=8 bench line's strong-scaling ratio (speedup_vs_1gpu_same_grid.vs_driver_record; its `value` divides by
rank 0's same-job measurement) — from a DRIVER record of bench.py's N=1 run:
    python tools/config5_denominator.py BENCH_r03.json
The driver's own record is the only accepted source (tests/test_config5_denominator.py checks it)."""
import json
import os
import re
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def bench_line(record):
    """The JSON line bench.py printed, from a driver BENCH_rNN.json record."""
    for text in (record["run"]["stdout_tail"], record.get("tail", "")):
        for ln in text.splitlines():
            ln = ln.strip()
            if ln.startswith("{") and '"config5_single_gpu"' in ln:
                return json.loads(ln)
    raise ValueError("no bench.py line with config5_single_gpu in the record")


def main(path):
    name = os.path.basename(path)
    if not re.fullmatch(r"BENCH_r\d\d\.json", name):
        raise SystemExit(f"{name}: not a driver bench record (BENCH_rNN.json)")
    rec = json.load(open(path))
    c5 = bench_line(rec)["config5_single_gpu"]
    out = {"mlups": c5["mlups"], "pair_kernel_ms": c5["pair_kernel_ms"], "pair_frac": c5.get("pair_frac"),
           "vcycle_ms": c5.get("vcycle_ms"), "grid": c5["grid"], "source": name, "source_kind": "driver",
           "source_detail": f"the driver's round-end bench ({rec.get('cmd', '?')}, {rec.get('where', '?')}, "
                            f"head {rec.get('head', '?')}): its config5_single_gpu object",
           "note": "1024^3 linear 2+2 on ONE MI355X, the driver's record: the secondary denominator of the N=8 "
                   "line's strong-scaling ratio (speedup_vs_1gpu_same_grid.vs_driver_record; `value` divides by "
                   "rank 0's same-job measurement). Regenerate with tools/config5_denominator.py <BENCH_rNN.json>."}
    with open(os.path.join(REPO, "profiles", "config5_single_gpu.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
