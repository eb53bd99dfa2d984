#!/bin/bash
# r05m: the round's tree after GS_NEWTON_G. The whole GPU suite, 600 seeded random solves (new seed), bench.py with the
# driver's flags twice, its rocprofv3 kernel-trace summary, one 512^3 two-iteration Newton solve's kernel sequence,
# and the 8-rank one-GPU rehearsal of the N > 1 line.
set -o pipefail
OUT=gpurun_out/${1:-r05m}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1"; exit 1; }; return 0; }
step pytest-gpu-full
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 20 > "$OUT/pytest.log" 2>&1; rc=$?
tail -4 "$OUT/pytest.log"; fatal $rc
step fuzz
GS_FUZZ_N=600 GS_FUZZ_SEED=20261021 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 900 --timeout-method thread > "$OUT/fuzz.log" 2>&1; rc=$?
tail -2 "$OUT/fuzz.log"; fatal $rc
step bench-driver-flags
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_r$r.json" 2> "$OUT/bench_r$r.err" || { tail -20 "$OUT/bench_r$r.err"; exit 1; }
  python tools/bench_brief.py "$OUT/bench_r$r.json" || true
done
step bench-rocprof-stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --cpu-sweeps 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -20 "$OUT/prof_bench.err"; exit 1; }
python tools/kernel_agg.py "$(find $OUT/prof_bench -name '*kernel_trace.csv' -print -quit)" > "$OUT/prof_bench_agg.txt" && head -24 "$OUT/prof_bench_agg.txt"
step newton-seq
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_n" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --vcycles 0 --config5 0 --newton-iters 2 > "$OUT/n512.json" 2> "$OUT/n512.err" || { tail -20 "$OUT/n512.err"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_n -name '*kernel_trace.csv' -print -quit)" -4 --agg > "$OUT/n512_seq.txt" && head -40 "$OUT/n512_seq.txt"
step ranks8
bash tools/bench_ranks.sh r05m/ranks8 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/ranks8/rank0.json'))
print(json.dumps({k: d.get(k) for k in ('value','scaling','rccl_cta_ab')})[:1500])" || true
step done
