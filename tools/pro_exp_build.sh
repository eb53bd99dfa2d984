#!/bin/bash
# Timing-only builds of the kernel library with GS_PRO_EXP=1..3 (gs_kernels.hip), and 4 = the product
# with GS_PRO_HALF=0 (the r02 prolongation arithmetic, for A/B), into
# gpu-solve_amd/build/exp/ (git-ignored; travels to the GPU box). Run here, then tools/pro_exp.py there.
set -e
H=$(dirname "$0")/../gpu-solve_amd
mkdir -p $H/build/exp
for e in ${@:-1 2 3 4}; do
  case $e in 4) D="-DGS_PRO_HALF=0" ;; *) D="-DGS_PRO_EXP=$e" ;; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I$H/../include -I$H/csrc \
    $D -shared -Wl,-Bsymbolic $H/csrc/gs_kernels.hip -o $H/build/exp/libgs_exp$e.so &
done
wait
