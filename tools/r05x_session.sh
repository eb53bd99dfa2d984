#!/bin/bash
# r05x: the chunking knobs re-checked with the round's NEWTON_B kernels (interleaved, 2 rounds): mid-level pair chunks
# (GS_MID_ZC=32), mid-level k_rr2 chunks (GS_RR_ZC=16), the 256^3 level's pairs in one round (GS_PAIR_ONE_ROUND_MID=1),
# the one-point passes' chunks (GS_RB_ZC=64), the fused prolongation pair from 2^21 points (GS_NEWTON_PRO_POINTS).
set -o pipefail
OUT=gpurun_out/${1:-r05x}; mkdir -p $OUT
timeout -k 10 1100 bash tools/multi_env_ab.sh $OUT 2 2 "default:" "midzc32:GS_MID_ZC=32" "rrzc16:GS_RR_ZC=16" \
    "oneroundmid:GS_PAIR_ONE_ROUND_MID=1" "rbzc64:GS_RB_ZC=64" "pro21:GS_NEWTON_PRO_POINTS=2097152"
