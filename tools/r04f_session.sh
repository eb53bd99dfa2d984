#!/bin/bash
# r04f: the whole GPU suite on the new defaults (GS_XH_SWIZZLE=1, GS_RR_REVERSE=1, GS_NEWTON_PRO_POINTS=2^24),
# bench.py with the driver's flags + its kernel-trace summary, the NEWTON fused-prolongation threshold on
# 256^3 and 512^3, PMC passes over the level-0 NEWTON kernels (tools/newton_kprobe.py), and an 8-rank
# rehearsal under rocprofv3 with GS_RCCL_CTAS=2 (does RCCL's kernel grid follow the communicator's cap?).
set -o pipefail
OUT=gpurun_out/${1:-r04f}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
nrun() { # tag size env...
  local tag=$1 size=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --size $size --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail "$OUT/$tag.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['newton']['ms_per_iteration'])"
}
step pytest-gpu-full
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
step bench-driver-flags
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python tools/bench_brief.py "$OUT/bench.json" || true
step bench-rocprof-stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 20 --cpu-sweeps 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -20 "$OUT/prof_bench.err"; exit 1; }
step newton-pro-threshold
for r in 1 2; do
  for s in 256 512; do
    nrun pro26_${s}_r$r $s GS_NEWTON_PRO_POINTS=67108864
    nrun pro24_${s}_r$r $s GS_NONE=1
  done
done
step pmc-newton
bash tools/pmc_run.sh r04f/newton tools/newton_kprobe.py 1 3 512 > "$OUT/pmc_newton.log" 2>&1 || { tail -30 "$OUT/pmc_newton.log"; exit 1; }
tail -20 "$OUT/pmc_newton.log"
python tools/pmc_level0.py "$OUT/newton/pmc" 134217728 > "$OUT/pmc_level0.txt" 2>&1 || true
cat "$OUT/pmc_level0.txt" || true
step ranks8-ctas2
GS_RCCL_CTAS=2 PROF=1 bash tools/bench_ranks.sh r04f/ranks8_ctas2 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
python tools/rccl_grid.py gpurun_out/r04f/ranks8_ctas2 > "$OUT/rccl_grid.txt" || true
head -20 "$OUT/rccl_grid.txt" || true
step done
