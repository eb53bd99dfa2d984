#!/bin/bash
# r04y: k_rr2's z-chunk on levels below 2^26 points (GS_RR_ZC; the 256^3 level: 8 coarse planes = 2048 blocks =
# 1.33 rounds at six blocks per CU; 11 planes = one round; 16 = 2/3 of one), V-cycle and Newton, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r04y}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/knob_ab.sh ${1:-r04y}/vc GS_RR_ZC 3 0 11 16 || exit 1
for r in 1 2; do
  for v in 0 11 16; do
    GS_RR_ZC=$v timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/n_${v}_r$r.json" 2> "$OUT/n_${v}_r$r.err" || { tail "$OUT/n_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/n_${v}_r$r.json')); print('GS_RR_ZC=$v r$r newton', d['newton']['ms_per_iteration'])"
  done
done
