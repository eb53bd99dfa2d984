#!/bin/bash
# k_rr2 under a cap on blocks per CU (GS_RR_SHMEM dynamic LDS): time in the V-cycle and FETCH_SIZE.
#   tools/rr_occ_session.sh <tag> [values...]      (through gpurun, from the repo root)
set -o pipefail
TAG=${1:-rrocc}; shift; VALS=${@:-0 90000}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for v in $VALS; do
    GS_RR_SHMEM=$v timeout -k 10 200 python bench.py --steps 10 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters 0 \
      --config5 0 > $OUT/b_${v}_r$r.json 2> $OUT/b_${v}_r$r.err || { tail $OUT/b_${v}_r$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${v}_r$r.json')); print('GS_RR_SHMEM=$v r$r vcycle', d['vcycle']['ms'], 'rr2 ms', d['vcycle']['level0_kernels']['residual_restrict']['ms'])"
  done
done
for v in $VALS; do
  GS_RR_SHMEM=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_$v -o run --output-format csv -- \
      python tools/prof_kernels.py --size 512 --reps 3 --which rr > $OUT/pmc_$v.log 2>&1 || { tail -20 $OUT/pmc_$v.log; exit 1; }
  python tools/pmc_summary.py $OUT/pmc_$v | grep -A3 "k_rr2" | head -4
done
