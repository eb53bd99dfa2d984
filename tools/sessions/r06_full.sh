#!/bin/bash
# Round-6 evidence session on one tree (through gpurun from the repo root): tools/sessions/r06_full.sh <tag> [fuzz_seed]
# The whole GPU suite, 600 seeded random solves, bench.py with the driver's flags twice, the rocprofv3 kernel-trace
# summary of the bench, one V-cycle's launch sequence (per level), one Newton iteration's split, and the level-0 PMC
# of the LINEAR and NEWTON_B kernels (separate counter passes). Every GPU step has its own limit; a fatal rc stops.
set -o pipefail
TAG=${1:-r06x}
SEED=${2:-20261026}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1"; exit 1; }; return 0; }
step pytest-gpu-full
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 20 > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; fatal $rc
step fuzz
GS_FUZZ_N=600 GS_FUZZ_SEED=$SEED timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 900 --timeout-method thread > "$OUT/fuzz.log" 2>&1; rc=$?
tail -2 "$OUT/fuzz.log"; fatal $rc
step bench-driver-flags
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_r$r.json" 2> "$OUT/bench_r$r.err" || { tail -20 "$OUT/bench_r$r.err"; exit 1; }
  python tools/bench_brief.py "$OUT/bench_r$r.json" || true
done
step bench-rocprof-stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --cpu-sweeps 0 --config2 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -20 "$OUT/prof_bench.err"; exit 1; }
python tools/kernel_agg.py "$(find $OUT/prof_bench -name '*kernel_trace.csv' -print -quit)" > "$OUT/prof_bench_agg.txt" && head -12 "$OUT/prof_bench_agg.txt"
step vcycle-sequence
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_vc" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --vcycles 10 --config5 0 --config2 0 --newton-iters 0 > "$OUT/vc.json" 2> "$OUT/vc.err" || { tail -20 "$OUT/vc.err"; exit 1; }
python tools/vc_breakdown.py "$(find $OUT/prof_vc -name '*kernel_trace.csv' -print -quit)" 30 --seq > "$OUT/vc_seq.txt" && head -40 "$OUT/vc_seq.txt"
step newton-seq
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_n" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --vcycles 0 --config5 0 --config2 0 --newton-iters 2 > "$OUT/n512.json" 2> "$OUT/n512.err" || { tail -20 "$OUT/n512.err"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_n -name '*kernel_trace.csv' -print -quit)" -4 --agg > "$OUT/n512_seq.txt" && head -22 "$OUT/n512_seq.txt"
step pmc-level0
bash tools/pmc_run.sh $TAG/kprobe tools/newton_kprobe.py 1 3 512 > "$OUT/pmc_kprobe.log" 2>&1 || { tail -30 "$OUT/pmc_kprobe.log"; exit 1; }
python tools/pmc_level0.py "$OUT/kprobe/pmc" 134217728 "k_rr2<0=17" "k_rr2<2=25" "k_rr2<3=25" "k_tb2y<2, 2, 4, true, false, false, true, 1=33" "k_tb2y<3, 2, 4, true, false, false, true, 1=33" "k_tb2y<2, 2, 4, true, false, false, true, 0=32" "k_tb2y<3, 2, 4, true, false, false, true, 0=32" "k_tb2y<0, 2, 4, true, false, false, true, 0, 2=24" "k_tb2y<0, 2, 4, true, false, false, true, 1, 1=25" > "$OUT/pmc_level0.txt" 2>&1 || true
cat "$OUT/pmc_level0.txt" || true
step done
