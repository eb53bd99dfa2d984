"""Launch sequence of one norm-to-norm segment of a rocprofv3 kernel trace (segments end at a
k_sumsq_finish launch), with full template arguments:
    python tools/trace_seq.py <kernel_trace.csv> [segment index, default -2] [--agg]
--agg: also the per-(kernel, grid) totals over every segment of the trace, full names."""
import collections
import csv
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].replace(" ", "")


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seg = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else -2
names = [short(r["Kernel_Name"]) for r in rows]
t0 = [int(r["Start_Timestamp"]) for r in rows]
t1 = [int(r["End_Timestamp"]) for r in rows]
grid = [int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) for r in rows]
fin = [i for i, n in enumerate(names) if "sumsq_finish" in n]
bounds = [-1] + fin
a, b = bounds[seg - 1] + 1, bounds[seg]
print(f"segment {seg}: launches {a}..{b}, kernel time {sum(t1[i] - t0[i] for i in range(a, b + 1)) / 1e3:.1f} us, "
      f"wall {(t1[b] - t0[a]) / 1e3:.1f} us")
for i in range(a, b + 1):
    gap = (t0[i] - t1[i - 1]) / 1e3 if i > a else 0.0
    print(f"  {names[i][:86]:88s} grid={grid[i]:>9d} {(t1[i] - t0[i]) / 1e3:9.1f} {gap:6.1f}")
if "--agg" in sys.argv:
    agg = collections.defaultdict(lambda: [0, 0.0])
    for i in range(len(rows)):
        v = agg[(names[i], grid[i])]
        v[0] += 1
        v[1] += (t1[i] - t0[i]) / 1e3
    print(f"\nall launches: {sum(v[1] for v in agg.values()):.1f} us")
    for (n, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"  {n[:86]:88s} grid={g:>9d} n={c:4d} {t:10.1f} us  ({t / c:8.1f} per launch)")
