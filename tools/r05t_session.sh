#!/bin/bash
# r05t: the shared Jacobi reciprocal in the plain pairs (yshb0) vs also in the four-x-wave prolongation pair (yshb4:
# the two-x-wave instance of 256-point rows, which would drop to one wave per SIMD, keeps recomputing), on batch3.
set -o pipefail
OUT=gpurun_out/${1:-r05t}; mkdir -p $OUT
timeout -k 10 1000 bash tools/multi_lib_ab.sh $OUT 3 2 batch3 yshb0 yshb4
