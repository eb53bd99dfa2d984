#!/bin/bash
# r05u: the adopted NEWTON_B pair changes (batched h^2 division, shared Jacobi reciprocal) with the zero-iterate pairs
# left out of the sharing (nozv: they keep three waves per SIMD, 166 VGPRs) against the product (177), interleaved;
# then the NEWTON tests on the product.
set -o pipefail
OUT=gpurun_out/${1:-r05u}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_newton_b.py tests/test_gpu_switches.py tests/test_gpu_zslab.py tests/test_gpu_newton_update.py tests/test_gpu_solver.py tests/test_gpu_sweep2.py -m gpu -q --timeout 300 --timeout-method thread -k "newton or Newton or NEWTON or zslab or slab or m2 or mode2 or mode3" > "$OUT/pytest.log" 2>&1; rc=$?
tail -4 "$OUT/pytest.log"; [ $rc -ge 124 ] && exit 1
timeout -k 10 900 bash tools/multi_lib_ab.sh $OUT/ab 3 2 product nozv
