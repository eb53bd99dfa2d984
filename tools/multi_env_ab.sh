#!/bin/bash
# Interleaved A/B of environment settings of the product library (A/B switches): per round, for
# each setting, the NEWTON_B level-0 kernels alone (tools/newton_kprobe.py) and bench.py with NI Newton iterations.
#   tools/multi_env_ab.sh <out-dir> <rounds> <newton-iters> "name:VAR=val VAR2=val" "name2:" ...
set -o pipefail
O=$1; R=$2; NI=$3; shift 3; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for spec in "$@"; do
    v=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 300 python tools/newton_kprobe.py 2 10 512 > $O/kp_${v}_r$r.json 2> $O/kp_${v}_r$r.err || { tail $O/kp_${v}_r$r.err; exit 1; }
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --vcycles 10 --cpu-sweeps 0 --newton-iters $NI --config5 0 \
      > $O/b_${v}_r$r.json 2> $O/b_${v}_r$r.err || { tail $O/b_${v}_r$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${v}_r$r.json')); k=d['vcycle']['level0_kernels']
p={a: min(b) for a, b in json.load(open('$O/kp_${v}_r$r.json'))['ms'].items() if a.startswith('newtonb') and not a.endswith('GBps')}
print('%-10s r$r' % '$v', 'pair', d['roofline']['kernel_ms'], 'vcycle', d['vcycle']['ms'], 'rr2', k['residual_restrict']['ms'], 'pro', k['prolong_pair']['ms'], 'newton', (d.get('newton') or {}).get('ms_per_iteration'), '| B:', p)"
  done
done
