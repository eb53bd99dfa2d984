#!/bin/bash
# r06z: LINEAR plain-pair load orders (p1: v rows, halo, f rows + the prolongation pairs' coarse rows issued first;
# p2: f rows, halo, v rows; p3: halo, then row by row) against the product, with config #5's 1024^3 pair leg.
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so $O/product.so
restore() { cp $O/product.so $L/libgpusolve_hip.so; }
trap restore EXIT INT TERM
for r in 1 2 3; do
  for v in product p1 p2 p3; do
    if [ $v = product ]; then cp $O/product.so $L/libgpusolve_hip.so; else cp gpu-solve_amd/lib_exp/$v/libgpusolve_hip.so $L/libgpusolve_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters 2 --config5 0 --config2 0 \
      > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    timeout -k 10 200 python tools/c5_pair_zc.py 20 > $O/c5_${v}_r$r.json 2> $O/c5_${v}_r$r.err || { tail $O/c5_${v}_r$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_r$r.json')); c=json.load(open('$O/c5_${v}_r$r.json')); k=d['vcycle']['level0_kernels']
print('%-8s r$r' % '$v', 'pair', d['roofline']['kernel_ms'], 'vcycle', d['vcycle']['ms'], 'pro', k['prolong_pair']['ms'], 'newton', d['newton']['ms_per_iteration'], 'c5 pair', c['pair_kernel_ms'])"
  done
done
