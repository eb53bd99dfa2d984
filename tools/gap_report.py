#!/usr/bin/env python3
"""Inter-kernel gaps of a rocprofv3 kernel trace (verdict r04 item 7: is a hipGraph worth building?).
    python tools/gap_report.py <kernel_trace.csv> [label] [--json out.json]
Segments end at a k_sumsq_finish launch (one norm-to-norm V-cycle; Newton: one inner V-cycle, the last one of
an inner solve merged with the update pass that follows it). Per segment: launches, the sum of kernel
durations, the wall span (first start -> last end) and their difference = the time the GPU queue sat between
kernels (dependent-kernel boundaries + any wait for the host). A hipGraph can only remove host-side launch
latency that the GPU waits on; the boundary itself costs the same eager or replayed (MI355X_MICROARCH.md,
row 'boundary'). Gaps >= 20 us are listed: the host was behind the GPU there (the norm readback)."""
import csv
import json
import statistics
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].replace(" ", "")


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path, label = args[0], (args[1] if len(args) > 1 else "")
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [short(r["Kernel_Name"]) for r in rows]
    t0 = [int(r["Start_Timestamp"]) for r in rows]
    t1 = [int(r["End_Timestamp"]) for r in rows]
    fin = [i for i, n in enumerate(names) if "sumsq_finish" in n]
    segs = []
    for a, b in zip(fin[:-1], fin[1:]):
        lo, hi = a + 1, b
        kern = sum(t1[i] - t0[i] for i in range(lo, hi + 1)) / 1e3
        wall = (t1[hi] - t0[lo]) / 1e3
        gaps = [(t0[i] - t1[i - 1]) / 1e3 for i in range(lo + 1, hi + 1)]
        big = [(names[i], round((t0[i] - t1[i - 1]) / 1e3, 1)) for i in range(lo + 1, hi + 1)
               if (t0[i] - t1[i - 1]) / 1e3 >= 20.0]
        segs.append({"launches": hi - lo + 1, "kernel_us": round(kern, 1), "wall_us": round(wall, 1),
                     "gap_us": round(wall - kern, 1), "gap_frac": round((wall - kern) / wall, 4) if wall else 0.0,
                     "boundaries": len(gaps), "gap_per_boundary_us": round(statistics.mean(gaps), 2) if gaps else 0.0,
                     "max_gap_us": round(max(gaps), 1) if gaps else 0.0, "big_gaps": big})
    # the typical segment: the median by wall time of the segments with the most common launch count
    common = statistics.mode([s["launches"] for s in segs]) if segs else 0
    typ = sorted([s for s in segs if s["launches"] == common], key=lambda s: s["wall_us"])
    med = typ[len(typ) // 2] if typ else None
    out = {"trace": path, "label": label, "segments": len(segs), "typical_launches": common, "typical": med,
           "gap_frac_all_segments": (round(sum(s["gap_us"] for s in segs) / sum(s["wall_us"] for s in segs), 4)
                                     if segs else None),
           "per_segment": segs}
    print(f"{label}: {len(segs)} segments; typical ({common} launches): {json.dumps(med)}")
    print(f"  gap fraction over all segments: {out['gap_frac_all_segments']}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
