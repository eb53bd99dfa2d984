#!/bin/bash
# k_rr2 A/B session (through gpurun): parity tests, bench V-cycle under two settings of one
# environment variable, and a rocprofv3 kernel-trace V-cycle breakdown for each.
#   tools/rr_ab_session.sh <tag> <VAR> <valA> <valB>
set -o pipefail
export TMPDIR=/tmp
TAG=$1; VAR=$2; A=$3; B=$4
O=gpurun_out/$TAG; mkdir -p $O
for val in "$A" "$B"; do
  env "$VAR=$val" timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$val.log 2>&1 || { tail -30 $O/pytest_$val.log; exit 1; }
  tail -1 $O/pytest_$val.log
done
bash tools/ab_multi.sh $TAG $VAR "$A $B" 2 --vcycles 50 || exit 1
for val in "$A" "$B"; do
  env "$VAR=$val" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$val -o run -- python bench.py --steps 20 --vcycles 5 --cpu-sweeps 0 --newton-iters 0 > $O/prof_$val.log 2>&1 || exit 1
  echo "== $VAR=$val"; python tools/vc_breakdown.py $(find $O/prof_$val -name '*kernel_trace.csv' -print -quit) 6
done
