#!/bin/bash
# r05ah: the whole GPU suite on the round's final build, as the driver runs it at round end.
set -o pipefail
OUT=gpurun_out/${1:-r05ah}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 20 > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; exit $rc
