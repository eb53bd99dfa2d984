#!/bin/bash
# r04aa: NEWTON k_rr2 in one round of blocks at 512^3 (GS_RR_ZC_BIG=128: 512 blocks of four waves at two per CU)
# against the 64-plane default (two rounds), on bench.py's Newton timing, interleaved, plus the level-0 probe.
set -o pipefail
OUT=gpurun_out/${1:-r04aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 0 128; do
    GS_RR_ZC_BIG=$v timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/n_${v}_r$r.json" 2> "$OUT/n_${v}_r$r.err" || { tail "$OUT/n_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/n_${v}_r$r.json')); print('GS_RR_ZC_BIG=$v r$r newton', d['newton']['ms_per_iteration'])"
    GS_RR_ZC_BIG=$v timeout -k 10 200 python tools/newton_kprobe.py 2 10 > "$OUT/kp_${v}_r$r.json" 2> "$OUT/kp_${v}_r$r.err" || { tail "$OUT/kp_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/kp_${v}_r$r.json'))['ms']; print('GS_RR_ZC_BIG=$v r$r', {k: min(x) for k, x in d.items() if k.endswith('_rr') and isinstance(x, list)})"
  done
done
