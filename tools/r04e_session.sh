#!/bin/bash
# r04e: Newton-path A/Bs (mid-level chunks, level-1 fused prolongation), column-block wave rotation on config
# #5's slab / grid, k_rr2's reversed chunks, the level-0 kernel probe, an 8-rank RCCL rehearsal under rocprofv3
# (RCCL's kernel grid against GS_RCCL_CTAS) and a kernel trace of one Newton iteration. One process per run.
set -o pipefail
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
nrun() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail "$OUT/$tag.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['newton']['ms_per_iteration'])"
}
step pytest-newton
timeout -k 10 600 python -u -m pytest tests/test_gpu_newton_update.py tests/test_gpu_solver.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
  step "newton round $r"
  nrun default_r$r GS_NONE=1
  nrun npro24_r$r GS_NEWTON_PRO_POINTS=16777216
  nrun midzc32_r$r GS_MID_ZC=32
  nrun rrzc4_r$r GS_RR_ZC=4
  nrun rrzc16_r$r GS_RR_ZC=16
done
step xh-swizzle
for r in 1 2; do
  for v in 0 1; do
    for dims in "1024 1024 128" "1024 1024 1024"; do
      GS_XH_SWIZZLE=$v timeout -k 10 200 python tools/pair_shape.py $dims > "$OUT/swz.txt" 2>&1 || { tail "$OUT/swz.txt"; exit 1; }
      echo "GS_XH_SWIZZLE=$v r$r $(cat $OUT/swz.txt)"
    done
  done
done
step rr-reverse
bash tools/knob_ab.sh r04e/rrrev GS_RR_REVERSE 2 0 1 || exit 1
step kprobe
timeout -k 10 300 python tools/newton_kprobe.py 3 10 > "$OUT/kprobe.json" 2> "$OUT/kprobe.err" || { tail -20 "$OUT/kprobe.err"; exit 1; }
cat "$OUT/kprobe.json"
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_newton" -o run --output-format csv -- python tools/newton_prof.py > "$OUT/prof_newton.log" 2>&1 || { tail -20 "$OUT/prof_newton.log"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_newton -name '*kernel_trace.csv' -print -quit)" -4 --agg > "$OUT/newton_seq.txt" || true
head -30 "$OUT/newton_seq.txt" || true
step ranks8-rocprof
PROF=1 bash tools/bench_ranks.sh r04e/ranks8 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
tail -3 "$OUT/ranks8.log"
python tools/rccl_grid.py gpurun_out/r04e/ranks8 > "$OUT/rccl_grid.txt" || true
head -40 "$OUT/rccl_grid.txt" || true
step done
