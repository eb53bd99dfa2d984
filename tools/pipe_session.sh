#!/bin/bash
# A/B of the overlapped solve loop (GS_NO_PIPELINE unset / set) through gpurun: GPU tests, bench
# V-cycle / Newton, and a rocprofv3 V-cycle breakdown.   tools/pipe_session.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pipe; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --vcycles 100 --cpu-sweeps 0 --newton-iters 2 > $O/on_$rep.json 2>$O/on_$rep.err || exit 1
  echo "pipe on  $(python tools/bench_brief.py $O/on_$rep.json)"
  GS_NO_PIPELINE=1 timeout -k 10 300 python bench.py --steps 20 --vcycles 100 --cpu-sweeps 0 --newton-iters 2 > $O/off_$rep.json 2>$O/off_$rep.err || exit 1
  echo "pipe off $(python tools/bench_brief.py $O/off_$rep.json)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 2 --warmup 2 --ramp-ms 0 --vcycles 5 --cpu-sweeps 0 --newton-iters 0 > $O/prof.log 2>&1 || exit 1
python tools/vc_breakdown.py $(find $O/prof -name '*kernel_trace.csv' -print -quit) 8
