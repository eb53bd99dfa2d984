#!/bin/bash
# A/B V-cycle session on the MI355X box (through gpurun, from the repo root):
#   tools/ab_session.sh <tag> [pytest]
# Kernel traces of 10 V-cycles of bench.py's 512^3 workload under each variant environment
# (tools/vc_breakdown.py reads them); optional GPU test run first. Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }

if [ "${2:-}" = "pytest" ]; then
    step pytest-gpu
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
    tail -2 "$OUT/pytest_gpu.log"
fi

vc() { # name, env...
    local name=$1; shift
    step "vcycle $name"
    env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/vc_$name" -o run --output-format csv -- \
        python bench.py --steps 2 --warmup 2 --cpu-sweeps 0 --newton-iters 0 --vcycles 10 > "$OUT/vc_$name.json" 2> "$OUT/vc_$name.err" \
        || { tail -20 "$OUT/vc_$name.err"; exit 1; }
    python tools/vc_breakdown.py "$OUT/vc_$name/run_kernel_trace.csv" 14 > "$OUT/vc_$name.txt"
    head -1 "$OUT/vc_$name.txt"
}
vc default GS_AB=default
vc nocoarse GS_COARSE_POINTS=0

vc rrlds GS_RR_LDS=1
step done
