#!/bin/bash
# r05n (timing): what NEWTON_B's per-point Jacobi division costs. nodiv (-DGS_EXP_NODIV: r * den, results wrong) and
# rcp1 (-DGS_EXP_RCP1: r times den's reciprocal after one Newton step, within an ulp or two of r / den) against the
# product: the level-0 kernels alone and bench.py with two Newton iterations, 3 interleaved rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05n}; mkdir -p $OUT
timeout -k 10 1100 bash tools/multi_lib_ab.sh $OUT 3 2 product nodiv rcp1
