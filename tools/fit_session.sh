#!/bin/bash
# A/B of the round-fitted zero-iterate pair chunks (GS_FIT_ROUNDS 0/1) through gpurun: GPU tests,
# bench V-cycle / Newton, and a rocprofv3 V-cycle breakdown per setting.   tools/fit_session.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fit; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_multi.sh fit GS_FIT_ROUNDS "0 1" 2 --newton-iters 2 || exit 1
for val in 0 1; do
  GS_FIT_ROUNDS=$val timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$val -o run -- python bench.py --steps 2 --warmup 2 --ramp-ms 0 --vcycles 5 --cpu-sweeps 0 --newton-iters 0 > $O/prof_$val.log 2>&1 || exit 1
  echo "== $val"; python tools/vc_breakdown.py $(find $O/prof_$val -name '*kernel_trace.csv' -print -quit) 14
done
