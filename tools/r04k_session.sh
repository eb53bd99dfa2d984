#!/bin/bash
# r04k: NEWTON column-block pairs: the five edge values of a step packed into one register per slot (plain pairs;
# the prolongation pairs load them per step)
# (lane groups, read back by lane permutes): the sweep-2 / prolongation / switch / Newton tests, then the 1023^3
# level-0 kernels and Newton iteration.
set -o pipefail
OUT=gpurun_out/${1:-r04k}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests/test_gpu_sweep2.py tests/test_gpu_newton_pro.py tests/test_gpu_switches.py tests/test_gpu_newton_update.py tests/test_gpu_zslab.py \
  -m gpu -x -q -k "not switch_bit_identical or newton_rows700 or SPEC_CACHED" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
step "kprobe 1023"
timeout -k 10 300 python tools/newton_kprobe.py 2 3 1023 > "$OUT/kp.json" 2> "$OUT/kp.err" || { tail -20 "$OUT/kp.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/kp.json'))['ms']; print({k: min(x) for k, x in d.items() if isinstance(x, list)})"
step newton-1023
for r in 1 2; do
  timeout -k 10 400 python bench.py --size 1023 --steps 2 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
    > "$OUT/n1023_r$r.json" 2> "$OUT/n1023_r$r.err" || { tail "$OUT/n1023_r$r.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/n1023_r$r.json')); print('1023 r$r', d['newton']['ms_per_iteration'], d['newton']['residuals'])"
done
step done
