#!/bin/bash
# r05j (timing): GS_NEWTON_B pairs and k_rr2 taking k.gamma instead of loading the factor (the first Newton iteration's
# B = gamma; lib_exp/wconst, -DGS_EXP_WCONST forces the flag on every launch, so its mode-3 timings are that iteration's)
# against the product: the level-0 kernels alone, 3 interleaved rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05j}; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2 3; do
for lib in product wconst; do
  L=gpu-solve_amd/lib/libgpusolve_hip.so; [ $lib = wconst ] && L=gpu-solve_amd/lib_exp/wconst/libgpusolve_hip.so
  GS_KPROBE_LIB=$PWD/$L timeout -k 10 300 python tools/newton_kprobe.py 2 10 512 > "$OUT/kp_${lib}_r$r.json" 2> "$OUT/kp_${lib}_r$r.err" || { tail "$OUT/kp_${lib}_r$r.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/kp_${lib}_r$r.json'))['ms']; print('$lib r$r', {k: min(v) for k, v in d.items() if k.startswith('newtonb') and not k.endswith('GBps')})"
done
done
