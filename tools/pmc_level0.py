"""Per-kernel PMC means over a V-cycle's level-0 launches only, from a tools/pmc_run.sh directory: a
launch counts as level 0 when it writes at least half the bytes of that kernel's largest launch
(every pass runs the same program, so a Dispatch_Id names the same launch in every pass); traffic
against the kernel's algorithmic bytes.
    python tools/pmc_level0.py gpurun_out/<tag>/pmc <points> [name-substring=bytes_per_point ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    d, pts = sys.argv[1], float(sys.argv[2])
    bpp = dict((kv.rsplit("=", 1)[0], float(kv.rsplit("=", 1)[1])) for kv in sys.argv[3:])
    per = collections.defaultdict(float)  # (kernel, dispatch, counter) -> value summed over rows
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            per[(r["Kernel_Name"], int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    writes = collections.defaultdict(dict)
    for (k, disp, c), v in per.items():
        if c == "WRITE_SIZE":
            writes[k][disp] = v
    for name in sorted(writes):
        top = max(writes[name].values())
        sel = {disp for disp, w in writes[name].items() if w >= 0.5 * top}
        m = collections.defaultdict(list)
        for (k, disp, c), v in per.items():
            if k == name and disp in sel:
                m[c].append(v)
        m = {c: sum(v) / len(v) for c, v in m.items()}
        short = name.replace("(anonymous namespace)::", "").replace("void ", "")
        short = short[: short.find("(")] if "(" in short else short
        line = f"{short}: level-0 launches={len(sel)}"
        if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_INST_ANY" in m:
            line += f" wait_inst/wave_cycles={m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f}"
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
            line += f" valu_active/wave_cycles={m['SQ_ACTIVE_INST_VALU'] / m['SQ_WAVE_CYCLES']:.3f}"
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and m["TCC_HIT_sum"] + m["TCC_MISS_sum"] > 0:
            line += f" L2_hit={m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}"
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            rd, wr = 2 * m["FETCH_SIZE"] * 1024, m["WRITE_SIZE"] * 1024
            line += f" read={rd / 1e9:.3f}GB write={wr / 1e9:.3f}GB"
            for key, b in bpp.items():
                if key in short:
                    line += f" traffic/algorithmic={(rd + wr) / (b * pts):.3f} ({b:g} B/pt)"
        print(line)


if __name__ == "__main__":
    main()
