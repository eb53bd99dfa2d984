"""The N=8 bench line's strong-scaling ratio (speedup_vs_1gpu_same_grid, bench.py): its `value` divides by rank
0's same-job one-GPU measurement of the 1024^3 grid; the secondary `vs_driver_record` divides by
profiles/config5_single_gpu.json, which must be the DRIVER's own N=1 measurement of config #5's grid (a
BENCH_rNN.json record), never a builder box's."""
import json
import os
import re
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "tools"))


def test_denominator_is_a_driver_record():
    from config5_denominator import bench_line

    d = json.load(open(os.path.join(REPO, "profiles", "config5_single_gpu.json")))
    assert re.fullmatch(r"BENCH_r\d\d\.json", d["source"]), d["source"]
    assert d.get("source_kind") == "driver"
    rec_path = os.path.join(REPO, d["source"])
    assert os.path.exists(rec_path), f"{d['source']} (the driver's record) is missing"
    c5 = bench_line(json.load(open(rec_path)))["config5_single_gpu"]
    assert d["mlups"] == c5["mlups"] and d["pair_kernel_ms"] == c5["pair_kernel_ms"]
    assert d["grid"] == [1024, 1024, 1024]

