#!/bin/bash
# One GPU session on the MI355X box (run through gpurun from the repo root):
#   tools/gpu_session.sh <tag> [steps]
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-20}
WARM=${3:-5}   # the driver runs bench.py --steps 20 --warmup 5
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }

if [ -z "$SKIP_TESTS" ]; then
step pytest-gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
fi

step kbench
timeout -k 10 500 python tools/kbench.py --bw --pairs --zc 0 --out "$OUT/kbench.json" > "$OUT/kbench.log" 2>&1 || { tail -20 "$OUT/kbench.log"; exit 1; }

step bench
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup "$WARM" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"

# kernel statistics of the bench's timed smoother alone (no V-cycles: every launch of the pair kernel
# is a level-0 launch, so its average is the bench's kernel_ms)
step rocprof-kernel-trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps "$STEPS" --warmup "$WARM" --cpu-sweeps 0 --newton-iters 0 --vcycles 0 --config5 0 > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { tail -20 "$OUT/bench_prof.err"; exit 1; }

# the V-cycle's kernels (tools/vc_breakdown.py reads the trace)
step rocprof-vcycle
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vc" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --cpu-sweeps 0 --newton-iters 0 --vcycles 10 --config5 0 > "$OUT/bench_vc.json" 2> "$OUT/bench_vc.err" || { tail -20 "$OUT/bench_vc.err"; exit 1; }

step rocprof-pmc-fetch
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python bench.py --steps 5 --cpu-sweeps 0 --newton-iters 0 --vcycles 0 --config5 0 > "$OUT/pmc_fetch.log" 2>&1 || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }

step rocprof-pmc-write
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python bench.py --steps 5 --cpu-sweeps 0 --newton-iters 0 --vcycles 0 --config5 0 > "$OUT/pmc_write.log" 2>&1 || { tail -20 "$OUT/pmc_write.log"; exit 1; }

step done
