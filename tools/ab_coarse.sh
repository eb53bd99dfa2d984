#!/bin/bash
set -o pipefail
OUT=gpurun_out/abcc
mkdir -p $OUT
export TMPDIR=/tmp
for thr in 4096 512 64 8 1; do
  GS_COARSE_POINTS=$thr timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t$thr -o run --output-format csv -- python bench.py --steps 2 --warmup 2 --cpu-sweeps 0 --newton-iters 0 --vcycles 10 > $OUT/t$thr.json 2>/dev/null || exit 1
  python tools/vc_breakdown.py $OUT/t$thr/run_kernel_trace.csv 40 > $OUT/t$thr.txt
  echo "thr $thr: $(head -1 $OUT/t$thr.txt) $(grep coarse $OUT/t$thr.txt)"
done
