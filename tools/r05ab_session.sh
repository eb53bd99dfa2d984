#!/bin/bash
# r05ab: the round's final tree (the prolongation pair shares the reciprocal too). The whole GPU suite, 600 seeded random solves (new
# seed), bench.py with the driver's flags twice and its rocprofv3 kernel-trace summary.
set -o pipefail
OUT=gpurun_out/${1:-r05ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1"; exit 1; }; return 0; }
step pytest-gpu-full
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 20 > "$OUT/pytest.log" 2>&1; rc=$?
tail -6 "$OUT/pytest.log"; fatal $rc
step fuzz
GS_FUZZ_N=600 GS_FUZZ_SEED=20261025 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 900 --timeout-method thread > "$OUT/fuzz.log" 2>&1; rc=$?
tail -2 "$OUT/fuzz.log"; fatal $rc
step bench-driver-flags
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_r$r.json" 2> "$OUT/bench_r$r.err" || { tail -20 "$OUT/bench_r$r.err"; exit 1; }
  python tools/bench_brief.py "$OUT/bench_r$r.json" || true
done
step bench-rocprof-stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --cpu-sweeps 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -20 "$OUT/prof_bench.err"; exit 1; }
python tools/kernel_agg.py "$(find $OUT/prof_bench -name '*kernel_trace.csv' -print -quit)" > "$OUT/prof_bench_agg.txt" && head -12 "$OUT/prof_bench_agg.txt"
step done
