#!/bin/bash
# r05b: k_rr2 with two groups of coarse rows per block (GS_RR_NG) and the level-0 GS_NEWTON_B factor fused into the
# compF update pass (GS_NEWTON_B_FUSED). The whole GPU suite, then interleaved A/Bs on bench.py (V-cycle, k_rr2 alone,
# Newton iteration) and the PMC passes over the level-0 kernels alone (k_rr2's over-fetch, verdict item 2).
set -o pipefail
OUT=gpurun_out/${1:-r05b}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1"; exit 1; }; return 0; }
step pytest-gpu-full
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 20 > "$OUT/pytest.log" 2>&1; rc=$?
tail -15 "$OUT/pytest.log"; fatal $rc
brief() { python -c "
import json,sys; d=json.load(open(sys.argv[1])); v=d.get('vcycle') or {}; l=v.get('level0_kernels') or {}
print(sys.argv[2], 'pair', d['roofline']['kernel_ms'], 'vcycle', v.get('ms'), 'rr2', (l.get('residual_restrict') or {}).get('ms'), 'pro', (l.get('prolong_pair') or {}).get('ms'), 'newton', (d.get('newton') or {}).get('ms_per_iteration'))" "$@"; }
step ab
for r in 1 2; do
  for v in def ng1 bf0; do
    case $v in def) E="GS_NONE=1";; ng1) E="GS_RR_NG=1";; bf0) E="GS_NEWTON_B_FUSED=0";; esac
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/ab_${v}_r$r.json" 2> "$OUT/ab_${v}_r$r.err" || { tail "$OUT/ab_${v}_r$r.err"; exit 1; }
    brief "$OUT/ab_${v}_r$r.json" "$v r$r"
  done
done
step newton-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_newton" -o run --output-format csv -- python tools/newton_prof.py > "$OUT/prof_newton.log" 2>&1 || { tail -20 "$OUT/prof_newton.log"; exit 1; }
NT=$(find "$OUT/prof_newton" -name '*kernel_trace.csv' -print -quit)
python tools/trace_seq.py "$NT" -4 --agg > "$OUT/newton_seq.txt" && head -45 "$OUT/newton_seq.txt"
step pmc-level0
bash tools/pmc_run.sh r05b/kprobe tools/newton_kprobe.py 1 3 512 > "$OUT/pmc_kprobe.log" 2>&1 || { tail -30 "$OUT/pmc_kprobe.log"; exit 1; }
python tools/pmc_level0.py "$OUT/kprobe/pmc" 134217728 "k_rr2<0=17" "k_rr2<2=25" "k_rr2<3=25" "k_tb2y<3, 2, 4, true, false, false, true, 1=33" "k_tb2y<3, 2, 4, true, false, false, true, 0=32" "k_tb2y<0, 2, 4, true, false, false, true, 0, 2=24" > "$OUT/pmc_level0.txt" 2>&1 || true
cat "$OUT/pmc_level0.txt" || true
step done
