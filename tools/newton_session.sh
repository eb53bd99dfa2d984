#!/bin/bash
# Newton A/B session on the MI355X box (run through gpurun from the repo root):
#   tools/newton_session.sh <tag> [pytest -k expr]
# GPU tests of the Newton paths, bench.py's Newton timing with the default build and under
# GS_NO_NEWTON_FUSED_UPDATE (each its own process), and a kernel trace of one 512^3 Newton iteration.
set -o pipefail
TAG=${1:-newton}
K=${2:-newton}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for rep in 1 2; do
  for sw in default GS_NO_NEWTON_FUSED_UPDATE; do
    step "bench newton $sw rep $rep"
    if [ "$sw" = default ]; then
      timeout -k 10 300 python bench.py --steps 4 --warmup 2 --cpu-sweeps 0 --vcycles 0 --config5 0 --newton-iters 2 > "$OUT/bench_${sw}_$rep.json" 2> "$OUT/bench_${sw}_$rep.err" || { tail -20 "$OUT/bench_${sw}_$rep.err"; exit 1; }
    else
      env $sw=1 timeout -k 10 300 python bench.py --steps 4 --warmup 2 --cpu-sweeps 0 --vcycles 0 --config5 0 --newton-iters 2 > "$OUT/bench_${sw}_$rep.json" 2> "$OUT/bench_${sw}_$rep.err" || { tail -20 "$OUT/bench_${sw}_$rep.err"; exit 1; }
    fi
    python -c "import json,sys; d=json.load(open('$OUT/bench_${sw}_$rep.json')); print('$sw', d['newton']['ms_per_iteration'], d['newton']['residuals'])"
  done
done
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python tools/newton_prof.py > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
python tools/kernel_agg.py "$(find $OUT/prof -name '*kernel_trace.csv' -print -quit)" > "$OUT/newton_kernels.txt" && head -40 "$OUT/newton_kernels.txt"
step done
