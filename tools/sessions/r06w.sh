#!/bin/bash
# r06w: the grouped load order of the LINEAR plain pairs (product) against the previous build (lib_exp/old):
# the pair tests on the new build, then per round bench.py (no Newton) and config #5's 1024^3 pair leg for each build.
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so $O/product.so
restore() { cp $O/product.so $L/libgpusolve_hip.so; }
trap restore EXIT INT TERM
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep2.py tests/test_gpu_solver.py tests/test_gpu_config5.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for v in product old; do
    if [ $v = product ]; then cp $O/product.so $L/libgpusolve_hip.so; else cp gpu-solve_amd/lib_exp/old/libgpusolve_hip.so $L/libgpusolve_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters 0 --config5 0 --config2 0 \
      > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    timeout -k 10 200 python tools/c5_pair_zc.py 20 > $O/c5_${v}_r$r.json 2> $O/c5_${v}_r$r.err || { tail $O/c5_${v}_r$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_r$r.json')); c=json.load(open('$O/c5_${v}_r$r.json'))
print('%-8s r$r' % '$v', 'pair', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'vcycle', d['vcycle']['ms'], 'c5 pair', c['pair_kernel_ms'], c['pair_frac'])"
  done
done
