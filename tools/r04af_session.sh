#!/bin/bash
# r04af: the one-point passes' z-chunk (GS_RB_ZC; the Newton update pass k_newton_upd runs ~5 rounds of blocks at
# 512^3 with the default 32 planes; 172 planes = one round at three blocks per CU): the Newton update tests under
# the knob, then bench.py's Newton timing interleaved with the default.
set -o pipefail
OUT=gpurun_out/${1:-r04af}
mkdir -p "$OUT"
export TMPDIR=/tmp
GS_RB_ZC=172 timeout -k 10 600 python -u -m pytest tests/test_gpu_newton_update.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2 3; do
  for v in 0 64 172; do
    GS_RB_ZC=$v timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/n_${v}_r$r.json" 2> "$OUT/n_${v}_r$r.err" || { tail "$OUT/n_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/n_${v}_r$r.json')); print('GS_RB_ZC=$v r$r newton', d['newton']['ms_per_iteration'], 'k_rb', d['single_sweep_kernel']['ms'])"
  done
done
