#!/bin/bash
# A/B of the in-tree kernel library against gpu-solve_amd/lib_ab/libgpusolve_hip_old.so (level-0
# residual+restriction and the production pair, tools/rr_ab.py), optionally after the GPU tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-abk}; mkdir -p $O
if [ "${2:-}" = "pytest" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
    tail -2 $O/pt.log
fi
timeout -k 10 300 python tools/rr_ab.py gpu-solve_amd/lib_ab/libgpusolve_hip_old.so 512 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
