#!/bin/bash
# k_rr2 with two coarse rows per block (GS_RR_NR=2) vs one: GPU tests under both, then the level-0
# A/B against the previous build (tools/rr_ab.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-rrnr}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt1.log 2>&1 || { tail -30 $O/pt1.log; exit 1; }
tail -1 $O/pt1.log
GS_RR_NR=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pt2.log 2>&1 || { tail -30 $O/pt2.log; exit 1; }
tail -1 $O/pt2.log
GS_RR_NR=1 timeout -k 10 300 python tools/rr_ab.py gpu-solve_amd/lib_ab/libgpusolve_hip_old.so 512 > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }
head -3 $O/ab1.log
GS_RR_NR=2 timeout -k 10 300 python tools/rr_ab.py gpu-solve_amd/lib_ab/libgpusolve_hip_old.so 512 > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }
head -3 $O/ab2.log
GS_RR_NR=2 timeout -k 10 300 python tools/rr_ab.py gpu-solve_amd/lib_ab/libgpusolve_hip_old.so 256 > $O/ab3.log 2>&1 || { tail -20 $O/ab3.log; exit 1; }
head -3 $O/ab3.log
