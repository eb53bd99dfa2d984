#!/bin/bash
# r04t: longer parity campaigns at the round's final tree: 5000 seeded random solves against the oracle on a new
# seed, and 30 random multi-rank RCCL problems (2-5 rank processes, socket transport) against one GPU.
set -o pipefail
OUT=gpurun_out/${1:-r04t}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step fuzz
GS_FUZZ_N=5000 GS_FUZZ_SEED=20261019 timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q --timeout 900 --timeout-method thread > "$OUT/fuzz.log" 2>&1 || { tail -30 "$OUT/fuzz.log"; exit 1; }
tail -1 "$OUT/fuzz.log"
step rccl-fuzz
GS_RCCL_FUZZ_N=30 GS_RCCL_FUZZ_SEED=20261019 timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl_multirank.py -m gpu -x -v -k random_vs_single --timeout 900 --timeout-method thread > "$OUT/rccl_fuzz.log" 2>&1 || { tail -30 "$OUT/rccl_fuzz.log"; exit 1; }
tail -1 "$OUT/rccl_fuzz.log"
step done
