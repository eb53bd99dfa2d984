#!/bin/bash
# Interleaved A/B/C... of kernel-library builds (gpu-solve_amd/lib_exp/<name>/libgpusolve_hip.so, tools/exp_builds.sh;
# "product" = the in-tree library): per round, for each build, the NEWTON_B level-0 kernels alone (tools/newton_kprobe.py)
# and bench.py with NI Newton iterations. The product library is restored however the session ends.
#   tools/multi_lib_ab.sh <out-dir> <rounds> <newton-iters> name1 name2 ...
set -o pipefail
O=$1; R=$2; NI=$3; shift 3; mkdir -p $O; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so $O/product.so
restore() { cp $O/product.so $L/libgpusolve_hip.so; }
trap restore EXIT INT TERM
for r in $(seq 1 $R); do
  for v in "$@"; do
    if [ $v = product ]; then cp $O/product.so $L/libgpusolve_hip.so; else cp gpu-solve_amd/lib_exp/$v/libgpusolve_hip.so $L/libgpusolve_hip.so; fi
    timeout -k 10 300 python tools/newton_kprobe.py 2 10 512 > $O/kp_${v}_r$r.json 2> $O/kp_${v}_r$r.err || { tail $O/kp_${v}_r$r.err; exit 1; }
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters $NI --config5 0 \
      > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_r$r.json')); k=d['vcycle']['level0_kernels']
p={a: min(b) for a, b in json.load(open('$O/kp_${v}_r$r.json'))['ms'].items() if a.startswith('newtonb') and not a.endswith('GBps')}
print('%-10s r$r' % '$v', 'pair', d['roofline']['kernel_ms'], 'vcycle', d['vcycle']['ms'], 'rr2', k['residual_restrict']['ms'], 'pro', k['prolong_pair']['ms'], 'newton', (d.get('newton') or {}).get('ms_per_iteration'), '| B:', p)"
  done
done
