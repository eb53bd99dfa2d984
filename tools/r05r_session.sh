#!/bin/bash
# r05r: GS_NEWTON_B pairs dividing each row's two stencil sums by h^2 in one batch (one range branch per row, as
# LINEAR does; lib_exp/batch3, -DGS_EXP_BATCH3: 218-243 VGPRs, no spill) against the product (one branch per point).
set -o pipefail
OUT=gpurun_out/${1:-r05r}; mkdir -p $OUT
timeout -k 10 900 bash tools/multi_lib_ab.sh $OUT 3 2 product batch3
