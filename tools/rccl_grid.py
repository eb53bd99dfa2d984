"""RCCL's kernels in the per-rank kernel traces of tools/bench_ranks.sh (PROF=1): launches, workgroup grid
(grid size / workgroup size) and mean duration per kernel name, per rank, with the launch count per
workgroup count (the bulk halo send/recv groups are the launches of the largest grid):
    python tools/rccl_grid.py gpurun_out/<tag>"""
import collections
import csv
import glob
import os
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "prof_r*"))):
    agg = collections.defaultdict(lambda: [0, 0.0, collections.Counter()])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "nccl" not in name.lower() and "rccl" not in name.lower():
                continue
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            a = agg[name.split("(")[0][:60]]
            a[0] += 1
            a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a[2][(g // max(1, wg), wg)] += 1
    print(os.path.basename(d))
    for name, (n, t, grids) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        hist = ", ".join(f"{w}x{th}: {c}" for (w, th), c in sorted(grids.items()))
        print(f"  {name:60s} n={n:5d} mean {t / n:8.1f} us  (workgroups x threads: launches) {hist}")
