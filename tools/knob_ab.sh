#!/bin/bash
# Interleaved A/B of one environment switch on the headline bench (one bench.py process per run):
#   tools/knob_ab.sh <tag> <VAR> <rounds> <value...>      e.g. tools/knob_ab.sh pfd GS_PAIR_PFD 3 2 3
set -o pipefail
O=gpurun_out/${1:-ab}; VAR=$2; R=$3; shift 3; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters 0 \
      --config5 0 > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${v}_r$r.json')); k=d['vcycle']['level0_kernels']; print('$VAR=$v r$r', 'GLUPS', round(d['value']/1e3,1), 'pair_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'vcycle', d['vcycle']['ms'], 'rr2', k['residual_restrict']['ms'], 'pro', k['prolong_pair']['ms'])"
  done
done
