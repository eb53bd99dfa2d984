#!/bin/bash
# r05z: the shared Jacobi reciprocal also in the four-x-wave NEWTON_B prolongation pair (ysh4, -DGS_EXP_YSH_PRO4:
# 255 VGPRs, no spill; r05t's yshb4 on the final tree) against the product, 4 interleaved rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05z}; mkdir -p $OUT
timeout -k 10 1100 bash tools/multi_lib_ab.sh $OUT 4 2 product ysh4
