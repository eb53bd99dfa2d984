#!/bin/bash
# r05ac: k_rr2's residual dividing a row's two stencil sums by h^2 in one batch (rrb, -DGS_EXP_RRB; every mode)
# against the product, 3 interleaved rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05ac}; mkdir -p $OUT
timeout -k 10 1000 bash tools/multi_lib_ab.sh $OUT 3 2 product rrb
