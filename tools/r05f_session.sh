#!/bin/bash
# r05f: GS_NEWTON_B prolongation pairs without the RECOMP LDS state (sweep 2's B / f rows of plane z-1 kept in
# registers, as the plain pairs do; the coarse X-pass rows stay in LDS): 246 instead of 234 VGPRs, no spill, 84 instead
# of 116 KB of LDS (gpu-solve_amd/lib_exp/norecomp, -DGS_EXP_B_NORECOMP). The level-0 kernels alone in both builds and
# an interleaved bench A/B with two Newton iterations.
set -o pipefail
OUT=gpurun_out/${1:-r05f}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step kprobe
for r in 1 2; do
for lib in product norecomp; do
  L=gpu-solve_amd/lib/libgpusolve_hip.so; [ $lib = norecomp ] && L=gpu-solve_amd/lib_exp/norecomp/libgpusolve_hip.so
  GS_KPROBE_LIB=$PWD/$L timeout -k 10 300 python tools/newton_kprobe.py 3 10 512 > "$OUT/kprobe_${lib}_r$r.json" 2> "$OUT/kprobe_${lib}_r$r.err" || { tail "$OUT/kprobe_${lib}_r$r.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/kprobe_${lib}_r$r.json'))['ms']; print('$lib r$r', {k: min(v) for k, v in d.items() if k.startswith('newtonb') and not k.endswith('GBps')})"
done
done
step lib-ab
timeout -k 10 1000 bash tools/lib_ab_session.sh r05f/libab 3 2 gpu-solve_amd/lib_exp/norecomp/libgpusolve_hip.so || exit 1
step done
