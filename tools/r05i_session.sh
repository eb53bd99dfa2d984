#!/bin/bash
# r05i (diagnosis): what the column-block pair's edge work costs. A timing-only build with every block edge treated as
# a boundary (gpu-solve_amd/lib_exp/noedge, -DGS_EXP_NOEDGE: no edge-column loads or lane-parallel sweep; results wrong)
# against the product, on config #5's per-rank slab (1024x1024x128), 1024^3 and 512^3 (no column blocks), interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r05i}; mkdir -p $OUT; export TMPDIR=/tmp
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so $OUT/product.so
restore() { cp $OUT/product.so $L/libgpusolve_hip.so; }
trap restore EXIT INT TERM
for r in 1 2 3; do
  for v in product noedge; do
    if [ $v = product ]; then cp $OUT/product.so $L/libgpusolve_hip.so; else cp gpu-solve_amd/lib_exp/noedge/libgpusolve_hip.so $L/libgpusolve_hip.so; fi
    for s in "1024 1024 128" "1024 1024 1024" "512 512 512"; do
      echo -n "$v r$r "; timeout -k 10 200 python tools/pair_shape.py $s || exit 1
    done
  done
done
