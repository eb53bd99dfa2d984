#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, kernel trace only) over tools/prof_kernels.py:
#   tools/pmc_session.sh <tag> [size]
# Summarise with: python tools/pmc_summary.py gpurun_out/<tag>/pmc
set -o pipefail
TAG=${1:-pmc}
SIZE=${2:-512}
EXTRA=${3:-}   # extra prof_kernels.py arguments, e.g. "--which pair --pair-variants 0,3 --zc 64"
OUT=gpurun_out/$TAG/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr" "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"; do
    i=$((i + 1))
    echo "[$(date +%T)] pass $i: $set"
    timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- \
        python tools/prof_kernels.py --size "$SIZE" --reps 3 $EXTRA > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
done
echo "[$(date +%T)] done"
