#!/bin/bash
# r05s: on top of the batched h^2 division (batch3, r05r), the Jacobi reciprocal formed once per point and pair and
# reused by sweep 2 (-DGS_EXP_YSHARE; yshb: plain and prolongation pairs, yshb0: plain pairs only), interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r05s}; mkdir -p $OUT
timeout -k 10 1000 bash tools/multi_lib_ab.sh $OUT 3 2 batch3 yshb yshb0
