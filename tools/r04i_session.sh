#!/bin/bash
# r04i: NEWTON column-block pairs keep sweep 2's newtonV / f / E rows in LDS (RECOMP, as the prolongation pair
# does): the sweep-2 / column-block tests, then the 1023^3 level-0 kernels and Newton iteration, k_tb2 plain
# pairs (GS_NEWTON_XH=0) against column blocks (GS_NEWTON_XH=1).
set -o pipefail
OUT=gpurun_out/${1:-r04i}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests/test_gpu_sweep2.py tests/test_gpu_newton_pro.py tests/test_gpu_switches.py tests/test_gpu_newton_update.py \
  -m gpu -x -q -k "not switch_bit_identical or newton_rows700" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in 0 1; do
  step "kprobe 1023 GS_NEWTON_XH=$v"
  GS_NEWTON_XH=$v timeout -k 10 300 python tools/newton_kprobe.py 2 3 1023 > "$OUT/kp_xh$v.json" 2> "$OUT/kp_xh$v.err" || { tail -20 "$OUT/kp_xh$v.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/kp_xh$v.json'))['ms']; print('xh=$v', {k: min(x) for k, x in d.items() if k.startswith('newton') and isinstance(x, list)})"
done
nrun() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --size 1023 --steps 2 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail "$OUT/$tag.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['newton']['ms_per_iteration'], d['newton']['residuals'])"
}
step newton-1023
nrun xh0 GS_NEWTON_XH=0
nrun xh1 GS_NEWTON_XH=1
nrun xh0_r2 GS_NEWTON_XH=0
nrun xh1_r2 GS_NEWTON_XH=1
step ranks8-channels-per-peer
# does the p2p channel count per peer (not the CTA budget) set RCCL's send/recv grid? (socket rehearsal)
NCCL_NCHANNELS_PER_PEER=16 NCCL_NCHANNELS_PER_NET_PEER=16 PROF=1 bash tools/bench_ranks.sh r04i/ranks8_cpp16 8 256 \
  --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
python tools/rccl_grid.py gpurun_out/r04i/ranks8_cpp16 > "$OUT/rccl_grid.txt" || true
head -20 "$OUT/rccl_grid.txt" || true
step done
