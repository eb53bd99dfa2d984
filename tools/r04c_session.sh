#!/bin/bash
# r04c: the full GPU suite, the driver-flag bench, and A/Bs: NEWTON's level-1 fused prolongation pair
# (GS_NEWTON_PRO_POINTS, two-x-wave instance), the column-block wave rotation (GS_XH_SWIZZLE) on config #5's
# slab and grid, k_rr2's reversed chunk order (GS_RR_REVERSE).
set -o pipefail
OUT=gpurun_out/${1:-r04c}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
step bench
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python tools/bench_brief.py "$OUT/bench.json"
step newton-pro-points
bash tools/newton_ab.sh r04c/npro GS_NEWTON_PRO_POINTS 2 67108864 16777216 || exit 1
step xh-swizzle
for r in 1 2; do
  for v in 0 1; do
    for dims in "1024 1024 128" "1024 1024 1024"; do
      GS_XH_SWIZZLE=$v timeout -k 10 200 python tools/pair_shape.py $dims > "$OUT/swz_${v}_r$r.txt" 2>&1 || { tail "$OUT/swz_${v}_r$r.txt"; exit 1; }
      echo "GS_XH_SWIZZLE=$v r$r $(cat $OUT/swz_${v}_r$r.txt)"
    done
  done
done
step rr-reverse
bash tools/knob_ab.sh r04c/rrrev GS_RR_REVERSE 2 0 1 || exit 1
step kprobe
timeout -k 10 300 python tools/newton_kprobe.py 3 10 > "$OUT/kprobe.json" 2> "$OUT/kprobe.err" || { tail -20 "$OUT/kprobe.err"; exit 1; }
cat "$OUT/kprobe.json"
step ranks8-rocprof
PROF=1 bash tools/bench_ranks.sh r04c/ranks8 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
tail -3 "$OUT/ranks8.log"
python tools/rccl_grid.py gpurun_out/r04c/ranks8 | head -40
step done
