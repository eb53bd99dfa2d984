#!/bin/bash
# r04x: 64-plane k_rr2 chunks on >= 2^26-point levels as the default: the switch / Z-slab / solver tests, then
# bench.py's Newton timing against the old rule (GS_RR_ZC_BIG=32: NEWTON 512^3's old chunk) and the V-cycle
# against GS_RR_ZC_BIG=16 (LINEAR 512^3's old chunk), interleaved, and config #5's slab V-cycle on 8 loopback slabs.
set -o pipefail
OUT=gpurun_out/${1:-r04x}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_zslab.py tests/test_gpu_solver.py tests/test_gpu_pair_restrict.py \
  -m gpu -x -q -k "not switch_bit_identical or RR_ZC_BIG" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2 3; do
  for v in 0 32; do
    GS_RR_ZC_BIG=$v timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/n_${v}_r$r.json" 2> "$OUT/n_${v}_r$r.err" || { tail "$OUT/n_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/n_${v}_r$r.json')); print('GS_RR_ZC_BIG=$v r$r newton', d['newton']['ms_per_iteration'])"
  done
done
bash tools/knob_ab.sh ${1:-r04x}/vc GS_RR_ZC_BIG 2 0 16 || exit 1
