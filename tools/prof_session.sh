#!/bin/bash
# Profile session on the MI355X box (run through gpurun from the repo root):
#   tools/prof_session.sh <tag> [pmc]
# 1. rocprofv3 kernel trace + stats of bench.py's default workload (the committed summary's source)
# 2. a V-cycle breakdown (tools/vc_breakdown.py over a kernel trace of 10 V-cycles)
# 3. with "pmc": counter passes over tools/prof_kernels.py (pair, residual+restriction)
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { echo "[$(date +%T)] $*"; }
if [ "$2" != "pmconly" ]; then
step rocprof-bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --cpu-sweeps 0 --newton-iters 0 --vcycles 0 > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { tail -20 "$OUT/bench_prof.err"; exit 1; }
step rocprof-vcycle
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vc" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --newton-iters 0 --vcycles 10 > "$OUT/bench_vc.json" 2> "$OUT/bench_vc.err" || { tail -20 "$OUT/bench_vc.err"; exit 1; }
python tools/vc_breakdown.py "$(find $OUT/prof_vc -name "*kernel_trace.csv" -print -quit)" 40 > "$OUT/vc_breakdown.txt" || true
cat "$OUT/vc_breakdown.txt"
fi
if [ "$2" = "pmc" ] || [ "$2" = "pmconly" ]; then
    mkdir -p "$OUT/pmc"
    i=0
    for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
               "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
               "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i + 1))
        step "pmc pass $i: $set"
        timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/pmc/p$i" -o run --output-format csv -- \
            python tools/prof_kernels.py --size 512 --reps 3 --which pair,rr > "$OUT/pmc/p$i.log" 2>&1 || { tail -20 "$OUT/pmc/p$i.log"; exit 1; }
    done
    python tools/pmc_summary.py "$OUT/pmc" --md "$OUT/pmc_summary.md" > /dev/null && cat "$OUT/pmc_summary.md"
fi
step done
