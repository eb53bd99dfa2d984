#!/bin/bash
# Pair z-chunks on levels of >= 2^26 points: GPU tests, then bench.py (smoother, V-cycle, Newton) with
# the 128-plane rule and with the 64-plane rule (GS_PAIR_BIG_CHUNKS=0), twice each, one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-chunk}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for r in 1 2; do
  for b in 1 0; do
    GS_PAIR_BIG_CHUNKS=$b timeout -k 10 300 python bench.py --steps 40 --warmup 100 --cpu-sweeps 0 --newton-iters 2 --vcycles 20 > $O/b${b}_$r.json 2> $O/b${b}_$r.err || { tail -20 $O/b${b}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b${b}_$r.json')); print('big=$b', d['roofline']['kernel_ms'], d['vcycle']['ms'], d['newton']['ms_per_iteration'])"
  done
done
