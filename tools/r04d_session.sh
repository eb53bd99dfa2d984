#!/bin/bash
# r04d: NEWTON mid-level chunking A/Bs (GS_MID_ZC for level-1/2 pairs, GS_RR_ZC for their k_rr2), one bench.py
# process per run, interleaved; then a kernel trace of one Newton iteration with the product defaults.
set -o pipefail
OUT=gpurun_out/${1:-r04d}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail "$OUT/$tag.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['newton']['ms_per_iteration'])"
}
for r in 1 2; do
  step "round $r"
  run default_r$r GS_NONE=1
  run midzc32_r$r GS_MID_ZC=32
  run midzc64_r$r GS_MID_ZC=64
  run rrzc4_r$r GS_RR_ZC=4
  run rrzc16_r$r GS_RR_ZC=16
  run npro24_r$r GS_NEWTON_PRO_POINTS=16777216
done
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_newton" -o run --output-format csv -- python tools/newton_prof.py > "$OUT/prof_newton.log" 2>&1 || { tail -20 "$OUT/prof_newton.log"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_newton -name '*kernel_trace.csv' -print -quit)" -4 --agg > "$OUT/newton_seq.txt" && head -45 "$OUT/newton_seq.txt"
step done
