#!/bin/bash
# Interleaved A/B of two builds of the kernel library on the headline bench (and optionally Newton): the
# alternative libgpusolve_hip.so is built here into gpu-solve_amd/lib_exp/ (tools/exp_builds.sh; scratch, deleted after the round) and swapped in between runs.
#   tools/lib_ab_session.sh <tag> [rounds] [newton-iters] [alt .so]   (through gpurun, from the repo root)
set -o pipefail
O=gpurun_out/${1:-libab}; R=${2:-3}; NI=${3:-0}; ALT=${4:-gpu-solve_amd/lib_exp/alt/libgpusolve_hip.so}; mkdir -p $O; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so $O/new.so
restore() { cp $O/new.so $L/libgpusolve_hip.so; }
# the product library is put back however the session ends (normal exit, failure, timeout signal)
trap restore EXIT INT TERM
for r in $(seq 1 $R); do
  for v in new alt; do
    if [ $v = new ]; then cp $O/new.so $L/libgpusolve_hip.so; else cp $ALT $L/libgpusolve_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters $NI --config5 0 \
      > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_r$r.json')); k=d['vcycle']['level0_kernels']
print('$v r$r', 'GLUPS', round(d['value']/1e3,1), 'pair_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'vcycle', d['vcycle']['ms'], 'rr2', k['residual_restrict']['ms'], 'pro', k['prolong_pair']['ms'], 'k_rb', d['single_sweep_kernel']['ms'], 'newton', (d.get('newton') or {}).get('ms_per_iteration'))"
  done
done
