#!/bin/bash
# bench.py's N > 1 path (torch.distributed "nccl" process group, RCCL Z-slab grid, overlapped ghost
# exchange, cross-rank ramp agreement and timing) rehearsed on ONE GPU: N processes started the way
# torchrun starts them, each with its own NCCL_HOSTID so that RCCL accepts several ranks on one device
# (they connect over the socket transport on loopback, not xGMI: the times are not the 8-GPU node's).
#   tools/bench_ranks.sh <tag> [N] [per-rank edge] [extra bench args]
# PROF=1: every rank under rocprofv3 --kernel-trace (gpurun_out/<tag>/prof_r<rank>/): the workgroup grid of
# RCCL's send/recv kernels (tools/rccl_grid.py) against the communicator's CTA budget (GS_RCCL_CTAS)
set -o pipefail
TAG=${1:-bench_ranks}; N=${2:-2}; SIZE=${3:-256}; shift 3 2>/dev/null
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
PORT=$((29500 + RANDOM % 1000))
pids=()
for r in $(seq 0 $((N - 1))); do
  NCCL_HOSTID=gs-bench-rank-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 GS_COMM_INIT_TIMEOUT_S=90 GS_COMM_TIMEOUT_S=60 \
  WORLD_SIZE=$N RANK=$r LOCAL_RANK=0 LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
    timeout -k 10 300 ${PROF:+rocprofv3 --kernel-trace -d "$OUT/prof_r$r" -o run --output-format csv --} \
    python bench.py --gpus "$N" --size "$SIZE" --steps 10 --warmup 2 "$@" \
    > "$OUT/rank$r.json" 2> "$OUT/rank$r.err" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
for r in $(seq 0 $((N - 1))); do echo "rank $r stderr tail:"; tail -5 "$OUT/rank$r.err"; done
cat "$OUT/rank0.json"
exit $rc
