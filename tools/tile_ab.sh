#!/bin/bash
# V-cycle A/B of the tiled small-level steps (GS_TILE_POINTS: 0 = off, else the largest tiled level),
# one bench.py process per setting, interleaved rounds:  tools/tile_ab.sh <tag> [rounds] [thresholds...]
set -o pipefail
O=gpurun_out/${1:-tile}; R=${2:-2}; shift 2; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for t in ${@:-0 32768 262144 2097152}; do
    GS_TILE_POINTS=$t timeout -k 10 120 python bench.py --steps 2 --warmup 2 --ramp-ms 100 --vcycles 30 --cpu-sweeps 0 \
      --newton-iters 0 --config5 0 > $O/vc_t${t}_r$r.json 2> $O/vc_t${t}_r$r.err || { tail $O/vc_t${t}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/vc_t${t}_r$r.json')); print('tile_points=$t round=$r vcycle_ms', d['vcycle']['ms'])"
  done
done
