#!/bin/bash
# rocprofv3 PMC passes (one counter set per run, SQ <= 8 / TCC <= 4 per pass) over one python program,
# then tools/pmc_summary.py per kernel (through gpurun):
#   tools/pmc_run.sh <tag> <script.py> [args...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG/pmc; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    echo "[$(date +%T)] pmc pass $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python "$@" > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
done
python tools/pmc_summary.py "$OUT" --md "$OUT/pmc_summary.md" > /dev/null && cat "$OUT/pmc_summary.md"
