#!/bin/bash
# r06y: k_rr2 with its halo rows loaded first (product) — the residual/restriction, solver and Newton tests on it, then
# an interleaved A/B against the previous build (old) and two more orders (r4: halos, f/w, v; r5: halos, v, f/w).
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py tests/test_gpu_newton_b.py \
    tests/test_gpu_zslab.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/multi_lib_ab.sh $O 3 2 product old r4 r5
