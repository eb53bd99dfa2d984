#!/usr/bin/env python3
"""Condense one gpu_session.sh output directory into the committed evidence under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `bench.py`
  profiles/<tag>_summary.md         the same as a table + the bench line + kbench results
  profiles/pmc_smoother.json        HBM bytes per launch of the level-0 sweep from the two PMC
                                    passes (bench.py reads it for roofline.traffic)

PMC correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly half the bytes of a
wide coalesced (16 B/lane) streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE reads
exactly for 16-B-per-lane streaming stores. Both counters include Infinity-Cache hits.

    python tools/profile_summary.py gpurun_out/r01 r01
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sweep_kernel(name):
    """The level-0 smoother of bench.py's headline: the fused LINEAR pair (k_tb2y whole-row shape, not the
    column blocks of config #5's 1024-point rows, not the prolongation / zero-iterate forms, or k_tb2) or,
    without it, the one-sweep k_rb."""
    if "k_tb2<0," in name:
        return True
    if "k_tb2y<0," not in name:
        return False
    args = [a.strip() for a in name[name.index("k_tb2y<") + 7:].split(">")[0].split(",")]
    # k_tb2y<MODE, RY, WXMAX, NT, NTF, ZV, SPEC, PRO, PFD, XH, UN>
    return len(args) < 10 or (args[5] == "false" and args[7] == "0" and args[9] == "false")


def single_kernel(name):
    return "k_rb<0, 0, false" in name


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(src, "prof", "run_kernel_stats.csv")
    lines = []
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
        rows = list(csv.DictReader(open(stats)))
        lines.append("| kernel | calls | avg us | min us | max us | % time |")
        lines.append("|---|---|---|---|---|---|")
        for r in rows:
            nm = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
            lines.append(f"| `{nm}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['MinNs'])/1e3:.1f} | "
                         f"{float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    # PMC: the level-0 sweep launches of the bench (largest grid among the sweep kernels)
    pmc = {}
    for counter, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        fn = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(fn):
            continue
        allrows = list(csv.DictReader(open(fn)))
        rows = [r for r in allrows if sweep_kernel(r["Kernel_Name"]) and r["Counter_Name"] == counter]
        if not rows:
            rows = [r for r in allrows if single_kernel(r["Kernel_Name"]) and r["Counter_Name"] == counter]
        if not rows:
            continue
        big = max(int(r["Grid_Size"]) for r in rows)
        vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == big]
        pmc[counter] = (sum(vals) / len(vals), len(vals), rows[0]["Kernel_Name"])
    bench = None
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj):
        txt = open(bj).read().strip().splitlines()
        bench = json.loads(txt[-1]) if txt else None
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch_kb, nf, kname = pmc["FETCH_SIZE"]
        write_kb, nw, _ = pmc["WRITE_SIZE"]
        read_bytes = 2.0 * fetch_kb * 1024
        write_bytes = write_kb * 1024
        n = bench["config"]["grid"][0] if bench else 512
        alg = 24.0 * n ** 3
        d = {"n": n, "kernel": kname.replace("(anonymous namespace)::", "").split("(")[0],
             "launches_averaged": min(nf, nw),
             "fetch_size_kb": fetch_kb, "write_size_kb": write_kb,
             "read_bytes_per_launch": read_bytes, "write_bytes_per_launch": write_bytes,
             "hbm_bytes_per_launch": read_bytes + write_bytes, "algorithmic_bytes_per_launch": alg,
             "traffic_over_algorithmic": (read_bytes + write_bytes) / alg,
             "correction": "read = 2 x FETCH_SIZE (gfx950 half-count of 16-B/lane streams), write = WRITE_SIZE; "
                           "Infinity-Cache hits are included by both counters",
             "source": f"profiles/{tag}_summary.md (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes)"}
        with open(os.path.join(prof, "pmc_smoother.json"), "w") as f:
            json.dump(d, f, indent=1)
        lines += ["", "## PMC (level-0 sweep, bench.py config)", "", "```", json.dumps(d, indent=1), "```"]
    if bench:
        lines += ["", "## bench.py line", "", "```", json.dumps(bench, indent=1), "```"]
    # the profiled bench run's timed launches (the last steps/2 pair launches of its kernel trace) against
    # the kernel_ms that run measured itself with HIP events on the solver's stream
    trace, bp = os.path.join(src, "prof", "run_kernel_trace.csv"), os.path.join(src, "bench_prof.json")
    if os.path.exists(trace) and os.path.exists(bp):
        b2 = json.loads(open(bp).read().strip().splitlines()[-1])
        rows = [r for r in csv.DictReader(open(trace)) if sweep_kernel(r["Kernel_Name"])]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        k = b2["steps"] // 2 + b2["steps"] % 2
        if len(rows) >= k > 0:
            timed = rows[-k:]
            avg = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed) / k / 1e6
            lines += ["", "## rocprofv3 vs bench.py's own HIP-event timing (same profiled run)", "",
                      f"- timed pair launches in the trace (last {k} of {len(rows)}): average {avg:.4f} ms",
                      f"- bench.py roofline.kernel_ms of that run: {b2['roofline']['kernel_ms']:.4f} ms "
                      f"(ratio {b2['roofline']['kernel_ms'] / avg:.3f}); the stats table's average also "
                      f"includes the warm-up launches"]
    vct = os.path.join(src, "prof_vc", "run_kernel_trace.csv")
    if os.path.exists(vct):
        import subprocess
        out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "vc_breakdown.py"), vct, "30"],
                             capture_output=True, text=True).stdout
        shutil.copy(os.path.join(src, "prof_vc", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_vcycle_stats.csv"))
        lines += ["", "## One 512^3 linear 2+2 V-cycle, kernel by kernel (rocprofv3 kernel trace, last cycle)", "",
                  "```", out.strip(), "```"]
    kb = os.path.join(src, "kbench.json")
    if os.path.exists(kb):
        k = json.load(open(kb))
        shutil.copy(kb, os.path.join(prof, f"{tag}_kbench.json"))
        lines += ["", "## kbench (sweep variants, 512^3, median of interleaved rounds)", "",
                  "| variant | ms | GB/s | % of 8 TB/s | bit-identical |", "|---|---|---|---|---|"]
        for nm, v in sorted(k["variants"].items(), key=lambda kv: kv[1]["median_ms"]):
            lines.append(f"| {nm} | {v['median_ms']} | {v['gbps']} | {v['pct_peak']} | "
                         f"{v['bitwise_equal_to_production']} |")
        if "bw_best" in k:
            lines += ["", "streaming ceilings (best config each): " +
                      ", ".join(f"{kk} {vv[0]} GB/s ({vv[1]})" for kk, vv in k["bw_best"].items())]
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write(f"# {tag}: rocprofv3 + bench evidence\n\n" + "\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
