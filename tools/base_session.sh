#!/bin/bash
# Baseline session on the MI355X box (run through gpurun from the repo root):
#   tools/base_session.sh <tag>
# bench.py with the driver's flags, then kernel traces of one 512^3 Newton iteration and of ten linear
# V-cycles, each printed as a launch sequence of one norm-to-norm segment (tools/trace_seq.py).
set -o pipefail
TAG=${1:-base}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step bench
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python tools/bench_brief.py "$OUT/bench.json" || true
step newton-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_newton" -o run --output-format csv -- python tools/newton_prof.py > "$OUT/prof_newton.log" 2>&1 || { tail -20 "$OUT/prof_newton.log"; exit 1; }
NT=$(find "$OUT/prof_newton" -name '*kernel_trace.csv' -print -quit)
python tools/trace_seq.py "$NT" -4 --agg > "$OUT/newton_seq.txt" && head -60 "$OUT/newton_seq.txt"
step vcycle-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vc" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --newton-iters 0 --config5 0 --vcycles 10 > "$OUT/bench_vc.json" 2> "$OUT/bench_vc.err" || { tail -20 "$OUT/bench_vc.err"; exit 1; }
VT=$(find "$OUT/prof_vc" -name '*kernel_trace.csv' -print -quit)
python tools/trace_seq.py "$VT" -3 > "$OUT/vc_seq.txt" && cat "$OUT/vc_seq.txt"
step done
