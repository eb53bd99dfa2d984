"""Per-kernel totals of a rocprofv3 kernel trace (name truncated, grid size), largest first."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:50]
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    a = agg[(name, g)]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"total kernel time {tot:.1f} us")
for (name, g), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{name:52s} grid={g:>10d} n={n:4d} {t:10.1f} us")
