#!/bin/bash
# A/B of bench.py under two settings of one environment variable (run through gpurun):
#   tools/ab_env.sh <tag> <VAR> <valA> <valB> [bench.py args...]
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for val in "$A" "$B"; do
    echo "[$(date +%T)] $VAR=$val rep $rep"
    env "$VAR=$val" timeout -k 10 300 python bench.py --cpu-sweeps 0 --newton-iters 0 "$@" > "$OUT/${VAR}_${val}_$rep.json" 2> "$OUT/${VAR}_${val}_$rep.err" || { tail -20 "$OUT/${VAR}_${val}_$rep.err"; exit 1; }
    python tools/bench_brief.py "$OUT/${VAR}_${val}_$rep.json"
  done
done
