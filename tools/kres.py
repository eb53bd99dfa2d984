#!/usr/bin/env python3
"""Code-object facts of the kernel library (CPU only): VGPRs, spill bytes, waves per SIMD and LDS per
block of every kernel, from hipcc's -Rpass-analysis=kernel-resource-usage remarks.

  python3 tools/kres.py [filter-regex] [--src gs_kernels.hip] [--remarks file]   (writes nothing)
"""
import argparse
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(REPO, "gpu-solve_amd", "csrc")


def remarks(src, extra):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950",
           "-I" + os.path.join(REPO, "include"), "-I" + CSRC, "-shared", os.path.join(CSRC, src), "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"] + extra
    return subprocess.run(cmd, capture_output=True, text=True, check=True).stderr


def parse(text):
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?(?: \[[^\]]+\])?): (\w+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        n = n.replace("(anonymous namespace)::", "")
        r["demangled"] = re.sub(r"\((Coef|double|int|const|CcPlan).*", "", n)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("filter", nargs="?", default="")
    ap.add_argument("--src", default="gs_kernels.hip")
    ap.add_argument("--remarks", help="read saved remarks instead of compiling")
    ap.add_argument("-D", action="append", default=[], help="extra -D defines")
    a = ap.parse_args()
    text = open(a.remarks).read() if a.remarks else remarks(a.src, ["-D" + d for d in a.D])
    print(f"{'VGPR':>4} {'AGPR':>4} {'spill':>5} {'w/SIMD':>6} {'LDS':>7}  kernel")
    for r in parse(text):
        if a.filter and not re.search(a.filter, r["demangled"]):
            continue
        print(f"{r.get('VGPRs', '?'):>4} {r.get('AGPRs', '?'):>4} {r.get('ScratchSize [bytes/lane]', '?'):>5} "
              f"{r.get('Occupancy [waves/SIMD]', '?'):>6} {r.get('LDS Size [bytes/block]', '?'):>7}  {r['demangled']}")


if __name__ == "__main__":
    sys.exit(main())
