#!/bin/bash
# r06ac: the round's evidence on the tree with the FX pairs and the load orders (tools/sessions/r06_full.sh), then the
# N = 8 bench path rehearsed on this one GPU (8 rank processes, RCCL socket transport; cpu_baseline and per-GPU
# %-of-peak in the N > 1 line).
set -o pipefail
bash tools/sessions/r06_full.sh ${TAG:-r06ac} ${SEED:-20261028} || exit 1
echo "[$(date +%T)] 8-rank rehearsal"
bash tools/bench_ranks.sh ${TAG:-r06ac}/ranks8 8 256 --cpu-sweeps 2 > gpurun_out/${TAG:-r06ac}/ranks8.log 2>&1 || { tail -30 gpurun_out/${TAG:-r06ac}/ranks8.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/${TAG:-r06ac}/ranks8/rank0.json')); m=d.get('multi_gpu') or {}
print('N=8 rehearsal', d['value'], d['unit'], 'cpu_baseline' in d, {k: v for k, v in m.items() if 'frac' in k or 'peak' in k})"
