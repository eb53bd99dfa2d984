#!/bin/bash
# r05w: k_rr2 non-temporal loads for the rows no neighbouring block reads also in one-row blocks (GS_RR_NTU=2: the
# NEWTON_B level-0 k_rr2 and the LINEAR levels below 2^26 points) against the default (two-row blocks only).
set -o pipefail
OUT=gpurun_out/${1:-r05w}; mkdir -p $OUT
timeout -k 10 1000 bash tools/multi_env_ab.sh $OUT 3 2 "default:" "ntu2:GS_RR_NTU=2"
