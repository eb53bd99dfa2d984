#!/bin/bash
# r05p: the GS_NEWTON_B Jacobi quotient, branch-free. c1 (product: den clamped at 2^1000, one Newton step of its
# reciprocal), c2 (two steps), br1 (r05o's range branch, one step), ieee (the IEEE division): each one's ulp distance
# to r / den (its own diag build), then the level-0 kernels and bench.py with two Newton iterations, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r05p}; mkdir -p $OUT; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_diag.so $OUT/diag_product.so
trap 'cp $OUT/diag_product.so $L/libgpusolve_diag.so' EXIT INT TERM
for v in c1 c2 br1; do
  cp gpu-solve_amd/lib_exp/$v/libgpusolve_diag.so $L/libgpusolve_diag.so
  echo -n "$v: "; timeout -k 10 200 python -u -m pytest tests/test_gpu_newton_b.py -m gpu -q -s -k ulps --timeout 150 --timeout-method thread 2>&1 | grep -E "^nb_quot|passed|failed" | tr '\n' ' '; echo
done
cp $OUT/diag_product.so $L/libgpusolve_diag.so
timeout -k 10 1000 bash tools/multi_lib_ab.sh $OUT/ab 3 2 c1 c2 br1 ieee || exit 1
