#!/bin/bash
# r04h: NEWTON on config #5's row length, at 1023^3 (odd: the Newton iteration converges; 1024^3 runs away to
# inf / NaN like the reference at powers of two, and its division / exp slow paths make that timing
# meaningless). The level-0 kernels alone (tools/newton_kprobe.py) and one Newton iteration through bench.py,
# default (column-block prolongation pair, k_tb2 plain pairs) against GS_NEWTON_XH=1 (column-block plain pairs)
# and GS_NEWTON_PRO_POINTS=2^40 (prolongation unfused: gs_prolong_add + k_tb2 pair, the r03 path).
set -o pipefail
OUT=gpurun_out/${1:-r04h}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest-switch
timeout -k 10 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_newton_pro.py -m gpu -x -q -k "newton_rows700 or list_matches or newton_fused_prolong" \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in 0 1; do
  step "kprobe 1023 GS_NEWTON_XH=$v"
  GS_NEWTON_XH=$v timeout -k 10 300 python tools/newton_kprobe.py 2 3 1023 > "$OUT/kp_xh$v.json" 2> "$OUT/kp_xh$v.err" || { tail -20 "$OUT/kp_xh$v.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/kp_xh$v.json'))['ms']; print('xh=$v', {k: (min(x) if isinstance(x, list) else x) for k, x in d.items()})"
done
nrun() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --size 1023 --steps 2 --warmup 2 --vcycles 2 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail "$OUT/$tag.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['newton']['ms_per_iteration'], d['newton']['residuals'], 'vcycle', d['vcycle']['ms'])"
}
step newton-1023
nrun default GS_NONE=1
nrun newton_xh GS_NEWTON_XH=1
nrun unfused GS_NEWTON_PRO_POINTS=1099511627776
step done
