#!/bin/bash
# r05a: the round's first tree on the GPU. The whole GPU suite (the switch tests at HEAD; a test
# failure is reported and the session goes on, a crash ends it), bench.py with the driver's flags (now with the
# copy / read-only ceilings), the Newton iteration with and without the GS_NEWTON_B factors (interleaved), kernel
# traces of ten linear V-cycles and one 512^3 Newton iteration with their inter-kernel gaps (verdict item 7:
# tools/gap_report.py), PMC passes over the level-0 kernels alone (tools/newton_kprobe.py: k_rr2's traffic at the
# 64-plane chunks, verdict item 2; the NEWTON / NEWTON_B kernels), and the 8-rank one-GPU rehearsal of the N > 1
# line (transports + the CTA A/B, verdict item 4).
set -o pipefail
OUT=gpurun_out/${1:-r05a}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1"; exit 1; }; return 0; }
step pytest-gpu-full
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 20 > "$OUT/pytest.log" 2>&1; rc=$?
tail -25 "$OUT/pytest.log"; fatal $rc
step bench-driver-flags
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python tools/bench_brief.py "$OUT/bench.json" || true
step newton-ab
for r in 1 2; do
  for v in b ref; do
    if [ $v = ref ]; then export GS_NO_NEWTON_B=1; else unset GS_NO_NEWTON_B; fi
    timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/newton_${v}_r$r.json" 2> "$OUT/newton_${v}_r$r.err" || { tail "$OUT/newton_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/newton_${v}_r$r.json')); print('newton $v r$r', d['newton']['ms_per_iteration'], d['newton']['residuals'])"
  done
done
unset GS_NO_NEWTON_B
step vcycle-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vc" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --newton-iters 0 --config5 0 --vcycles 10 > "$OUT/bench_vc.json" 2> "$OUT/bench_vc.err" || { tail -20 "$OUT/bench_vc.err"; exit 1; }
VT=$(find "$OUT/prof_vc" -name '*kernel_trace.csv' -print -quit)
python tools/gap_report.py "$VT" vcycle512 --json "$OUT/gaps_vcycle.json"
step newton-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_newton" -o run --output-format csv -- python tools/newton_prof.py > "$OUT/prof_newton.log" 2>&1 || { tail -20 "$OUT/prof_newton.log"; exit 1; }
NT=$(find "$OUT/prof_newton" -name '*kernel_trace.csv' -print -quit)
python tools/gap_report.py "$NT" newton512 --json "$OUT/gaps_newton.json"
python tools/trace_seq.py "$NT" -4 --agg > "$OUT/newton_seq.txt" && head -30 "$OUT/newton_seq.txt"
step kprobe
timeout -k 10 300 python tools/newton_kprobe.py 3 10 512 > "$OUT/kprobe.json" 2> "$OUT/kprobe.err" || { tail "$OUT/kprobe.err"; exit 1; }
cat "$OUT/kprobe.json"
step pmc-level0
bash tools/pmc_run.sh r05a/kprobe tools/newton_kprobe.py 1 3 512 > "$OUT/pmc_kprobe.log" 2>&1 || { tail -30 "$OUT/pmc_kprobe.log"; exit 1; }
python tools/pmc_level0.py "$OUT/kprobe/pmc" 134217728 "k_rr2<0=17" "k_rr2<2=25" "k_rr2<3=25" "k_tb2y<2, 2, 4, true, false, false, true, 1=33" "k_tb2y<3, 2, 4, true, false, false, true, 1=33" "k_tb2y<2, 2, 4, true, false, false, true, 0=32" "k_tb2y<3, 2, 4, true, false, false, true, 0=32" "k_tb2y<0, 2, 4, true, false, false, true, 0, 2=24" > "$OUT/pmc_level0.txt" 2>&1 || true
cat "$OUT/pmc_level0.txt" || true
step ranks8
bash tools/bench_ranks.sh r05a/ranks8 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/ranks8/rank0.json'))
print(json.dumps({k: d.get(k) for k in ('value','scaling','rccl_cta_ab','rccl_transports')})[:3000])
print(d['config']['workload'])" || true
step done
