#!/bin/bash
# r04r: gs_smooth2_restrict_zero (a LINEAR coarse level's first step from v = 0 in one pass): its bit-identity tests,
# the switch test, the whole-solve tests against the oracle, then the V-cycle with and without it (GS_NO_ZPRR),
# interleaved, and a kernel trace of ten V-cycles.
set -o pipefail
OUT=gpurun_out/${1:-r04r}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests/test_gpu_pair_restrict.py tests/test_gpu_solver.py tests/test_gpu_switches.py tests/test_gpu_coarse.py \
  tests/test_gpu_tiled.py -m gpu -x -q -k "not switch_bit_identical or ZPRR" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
step ab
bash tools/knob_ab.sh ${1:-r04r}/ab GS_NO_ZPRR 3 0 1 || exit 1
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vc" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --newton-iters 0 --config5 0 --vcycles 10 > "$OUT/vc.json" 2> "$OUT/vc.err" || { tail -20 "$OUT/vc.err"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_vc -name '*kernel_trace.csv' -print -quit)" -3 > "$OUT/vc_seq.txt" && cat "$OUT/vc_seq.txt"
step done
