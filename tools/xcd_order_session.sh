#!/bin/bash
# XCD-aware tile order (production) vs the hardware order, on the headline bench: the second library is
# built here with -DGS_XCD_IDENTITY into gpu-solve_amd/lib_noxcd/ and swapped in between interleaved runs.
#   tools/xcd_order_session.sh <tag> [rounds]          (through gpurun, from the repo root)
set -o pipefail
O=gpurun_out/${1:-xcd}; R=${2:-3}; mkdir -p $O; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so $O/prod.so
for r in $(seq 1 $R); do
  for v in prod noxcd; do
    if [ $v = prod ]; then cp $O/prod.so $L/libgpusolve_hip.so; else cp gpu-solve_amd/lib_noxcd/libgpusolve_hip.so $L/libgpusolve_hip.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters 0 --config5 0 \
      > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { cp $O/prod.so $L/libgpusolve_hip.so; tail $O/b_${v}_r$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${v}_r$r.json')); k=d['vcycle']['level0_kernels']; print('$v r$r', 'pair_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'vcycle', d['vcycle']['ms'], 'rr2', k['residual_restrict']['ms'], 'pro', k['prolong_pair']['ms'], 'k_rb', d['single_sweep_kernel']['ms'])"
  done
done
cp $O/prod.so $L/libgpusolve_hip.so
