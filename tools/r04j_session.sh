#!/bin/bash
# r04j: evidence at the round-4 tree — the whole GPU suite, smoke(), 600 seeded random solves of a new seed against
# the oracle, bench.py as the driver runs it + its kernel-trace summary, three 512^3 Newton timings, and the 8-rank
# rehearsal with bench.py's default p2p channel count (NCCL_NCHANNELS_PER_PEER = GS_RCCL_CTAS / 4).
set -o pipefail
OUT=gpurun_out/${1:-r04j}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest-gpu-full
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
step fuzz
GS_FUZZ_N=600 GS_FUZZ_SEED=20261018 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/fuzz.log" 2>&1 || { tail -30 "$OUT/fuzz.log"; exit 1; }
tail -1 "$OUT/fuzz.log"
step bench-driver-flags
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python tools/bench_brief.py "$OUT/bench.json" || true
step bench-rocprof-stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
    python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sweeps 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -20 "$OUT/prof_bench.err"; exit 1; }
step newton-512
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 > "$OUT/newton_r$r.json" 2> "$OUT/newton_r$r.err" || { tail "$OUT/newton_r$r.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/newton_r$r.json')); print('newton r$r', d['newton']['ms_per_iteration'])"
done
step ranks8
PROF=1 bash tools/bench_ranks.sh ${1:-r04j}/ranks8 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
python tools/rccl_grid.py gpurun_out/${1:-r04j}/ranks8 > "$OUT/rccl_grid.txt" || true
head -4 "$OUT/rccl_grid.txt" || true
python -c "import json; d=json.load(open('gpurun_out/${1:-r04j}/ranks8/rank0.json')); print({k: d['multi_gpu'][k] for k in ('rccl_ctas', 'rccl_channels_per_peer', 'rank_halo_host_us_max')})" || true
step done
