#!/bin/bash
# Round-6 product-vs-other-builds session:
#   tools/sessions/r06_libab.sh <tag> <rounds> <newton-iters> "<alt builds>" <pytest files...>
# The given GPU test files on the product build, then per round bench.py and config #5's 1024^3 pair leg for the product
# and each gpu-solve_amd/lib_exp/<alt> build (e.g. old: the build before the change), the order rotated every round.
# The product library is restored however it ends.
set -o pipefail
TAG=$1; R=$2; NI=$3; ALTS=$4; shift 4
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so $O/product.so
restore() { cp $O/product.so $L/libgpusolve_hip.so; }
trap restore EXIT INT TERM
if [ $# -gt 0 ]; then
  timeout -k 10 700 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for r in $(seq 1 $R); do
  all=(product $ALTS); n=${#all[@]}; order=()
  for i in $(seq 0 $((n - 1))); do order+=("${all[$(((i + r) % n))]}"); done  # rotate which build runs first
  for v in "${order[@]}"; do
    if [ $v = product ]; then cp $O/product.so $L/libgpusolve_hip.so; else cp gpu-solve_amd/lib_exp/$v/libgpusolve_hip.so $L/libgpusolve_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters $NI --config5 0 --config2 0 \
      > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    timeout -k 10 200 python tools/c5_pair_zc.py 20 > $O/c5_${v}_r$r.json 2> $O/c5_${v}_r$r.err || { tail $O/c5_${v}_r$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_r$r.json')); c=json.load(open('$O/c5_${v}_r$r.json')); k=d['vcycle']['level0_kernels']
print('%-8s r$r' % '$v', 'pair', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'vcycle', d['vcycle']['ms'], 'rr2', k['residual_restrict']['ms'], 'pro', k['prolong_pair']['ms'], 'newton', (d.get('newton') or {}).get('ms_per_iteration'), 'c5 pair', c['pair_kernel_ms'], c['pair_frac'])"
  done
done
