#!/bin/bash
# Pair launch time on whole levels under GS_PAIR_ZC (z-chunk override, A/B): tools/zc_sweep.sh <tag> "<zcs>" nx ny nz
set -o pipefail
TAG=$1; ZCS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do
  for zc in $ZCS; do
    echo -n "rep $r zc=$zc: " | tee -a "$OUT/zc.log"
    GS_PAIR_ZC=$zc timeout -k 10 120 python tools/pair_shape.py "$@" 2>&1 | tee -a "$OUT/zc.log" || exit 1
  done
done
