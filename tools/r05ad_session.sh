#!/bin/bash
# r05ad: the round's final built tree as the driver runs it: smoke(), the default `python bench.py`, and the NEWTON
# and LINEAR GPU test files most tied to the round's changes.
set -o pipefail
OUT=gpurun_out/${1:-r05ad}; mkdir -p $OUT; export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit 1
echo "[$(date +%T)] bench default"
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python tools/bench_brief.py $OUT/bench_default.json || true
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_newton_b.py tests/test_gpu_solver.py tests/test_gpu_sweep2.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -ge 124 ] && exit 1
echo "[$(date +%T)] done"
