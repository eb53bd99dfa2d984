#!/bin/bash
# Timing-only experiment builds of the kernel library (CPU, in the build container): one
# gpu-solve_amd/lib_exp/<name>/libgpusolve_hip.so per -D set (GS_EXP_* in gs_device.hpp, plus any
# KFLAGS-style extras). They travel to the GPU box with the tree; tools/newton_kprobe.py loads one
# through GS_KPROBE_LIB. Never the product: their results are wrong by construction.
#   tools/exp_builds.sh name1:"-DGS_EXP_NOBAR" name2:"-DGS_EXP_NOEXP" ...
set -e
cd "$(dirname "$0")/../gpu-solve_amd"
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  mkdir -p lib_exp/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall --offload-arch=gfx950 $defs \
      -I../include -Icsrc -shared csrc/gs_kernels.hip -o lib_exp/$name/libgpusolve_hip.so &
done
wait
ls -la lib_exp/*/libgpusolve_hip.so
