#!/bin/bash
# Interleaved A/B of one environment switch on bench.py's Newton timing (BASELINE config #4, 512^3, 2 outer
# iterations of 10 inner V-cycles), one process per run, plus a kernel trace of one iteration per value:
#   tools/newton_ab.sh <tag> <VAR> <rounds> <value...>        (through gpurun, from the repo root)
set -o pipefail
O=gpurun_out/${1:-nab}; VAR=$2; R=$3; shift 3; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 \
      --newton-iters 2 > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${v}_r$r.json')); print('$VAR=$v r$r newton ms/iter', d['newton']['ms_per_iteration'], d['newton']['residuals'])"
  done
done
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- \
      python tools/newton_prof.py > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  echo "== $VAR=$v"; python tools/kernel_agg.py "$(find $O/prof_$v -name '*kernel_trace.csv' -print -quit)" | head -14 || true
done
