#!/bin/bash
# r05o: the GS_NEWTON_B Jacobi quotient through den's refined reciprocal (nb_quot). Its ulp distance to the IEEE
# quotient (diag probe), the NEWTON tests with it, then an interleaved A/B: product (one Newton step of the
# reciprocal) vs steps2 (-DGS_EXP_NB_STEPS2: two) vs ieee (-DGS_EXP_NB_IEEE: the IEEE division, r05m's arithmetic).
set -o pipefail
OUT=gpurun_out/${1:-r05o}; mkdir -p $OUT; export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step ulps
timeout -k 10 300 python -u -m pytest tests/test_gpu_newton_b.py -m gpu -q -s -k ulps --timeout 200 --timeout-method thread 2>&1 | grep -E "nb_quot|passed|failed|Error" ; 
step pytest-newton
timeout -k 10 900 python -u -m pytest tests/test_gpu_newton_b.py tests/test_gpu_switches.py tests/test_gpu_zslab.py tests/test_gpu_newton_update.py tests/test_gpu_solver.py tests/test_gpu_fuzz.py -m gpu -q --timeout 300 --timeout-method thread -k "newton or Newton or NEWTON or zslab or slab or fuzz or m2 or mode2" > "$OUT/pytest.log" 2>&1; rc=$?
tail -8 "$OUT/pytest.log"; [ $rc -ge 124 ] && exit 1
step ab
timeout -k 10 900 bash tools/multi_lib_ab.sh $OUT/ab 3 2 product steps2 ieee || exit 1
step done
