"""Per-kernel mean of every counter collected by tools/pmc_session.sh.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc [--md out.md]
"""
import argparse
import collections
import csv
import glob
import os
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([A-Za-z0-9_]+<[^(]*>|[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--md")
    a = ap.parse_args()
    # counter values per (kernel, dispatch): summed over the dimensions rocprof reports per row
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for fn in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(fn)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            x = float(r["Counter_Value"])
            # GRBM_* are chip-wide clocks repeated per XCD: take one copy; everything else adds up
            per[key] = max(per[key], x) if r["Counter_Name"].startswith("GRBM") else per[key] + x
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (d, c), v in per.items():
            vals[names[d]][c].append(v)
    lines = []
    for k in sorted(vals):
        lines.append(f"### {k}")
        for c in sorted(vals[k]):
            xs = vals[k][c]
            lines.append(f"- {c}: {sum(xs) / len(xs):.6g}  (n={len(xs)})")
        cs = {c: sum(x) / len(x) for c, x in vals[k].items()}
        if "SQ_ACTIVE_INST_VALU" in cs and "GRBM_GUI_ACTIVE" in cs:
            lines.append(f"- VALUBusy% (256 CUs): {100 * cs['SQ_ACTIVE_INST_VALU'] / 256 / cs['GRBM_GUI_ACTIVE']:.1f}")
        if "SQ_WAIT_INST_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
            lines.append(f"- wait_inst/wave_cycles: {cs['SQ_WAIT_INST_ANY'] / cs['SQ_WAVE_CYCLES']:.3f}")
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            lines.append(f"- L2 hit rate: {cs['TCC_HIT_sum'] / (cs['TCC_HIT_sum'] + cs['TCC_MISS_sum']):.3f}")
        lines.append("")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out)


if __name__ == "__main__":
    main()
