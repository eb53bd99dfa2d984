#!/bin/bash
# Newton iteration (BASELINE config #4, 512^3) with the tiled small-level steps on / off (GS_TILE_POINTS),
# one bench.py process per setting:   tools/newton_tile_ab.sh <tag> [thresholds...]
set -o pipefail
O=gpurun_out/${1:-ntile}; shift; mkdir -p $O; export TMPDIR=/tmp
for t in ${@:-0 262144}; do
  GS_TILE_POINTS=$t timeout -k 10 200 python bench.py --steps 2 --warmup 2 --ramp-ms 50 --vcycles 10 --cpu-sweeps 0 \
    --newton-iters 2 --config5 0 > $O/n_t$t.json 2> $O/n_t$t.err || { tail $O/n_t$t.err; exit 1; }
  python -c "import json; d=json.load(open('$O/n_t$t.json')); print('tile_points=$t vcycle_ms', d['vcycle']['ms'], 'newton_ms', d['newton']['ms_per_iteration'])"
done
