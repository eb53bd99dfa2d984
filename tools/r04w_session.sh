#!/bin/bash
# r04w: k_rr2's z-chunk on >= 2^26-point levels (GS_RR_ZC_BIG; the rule gives 16 coarse planes at 512^3 and the
# cap of 32 at 1024^3): bench.py's level-0 kernel timings and V-cycle at 1024^3 and 512^3, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r04w}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for s in 1024 512; do
    for v in 0 8 16 64 128; do
      GS_RR_ZC_BIG=$v timeout -k 10 300 python bench.py --size $s --steps 4 --warmup 2 --vcycles 6 --cpu-sweeps 0 --newton-iters 0 --config5 0 \
        > "$OUT/b_${s}_${v}_r$r.json" 2> "$OUT/b_${s}_${v}_r$r.err" || { tail "$OUT/b_${s}_${v}_r$r.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/b_${s}_${v}_r$r.json')); k=d['vcycle']['level0_kernels']; print('$s GS_RR_ZC_BIG=$v r$r vcycle', d['vcycle']['ms'], 'rr2', k['residual_restrict']['ms'])"
    done
  done
done
