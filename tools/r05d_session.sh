#!/bin/bash
# r05d: one 1023^3 Newton iteration's kernel trace (config #5's grid in mode 2: the GS_NEWTON_B column-block
# prolongation pair, verdict item 6), the NEWTON fused-prolongation threshold under GS_NEWTON_B (GS_NEWTON_PRO_POINTS
# 2^20: level 2 of 512^3 too), config #5's per-rank slab pair alone (tools/pair_shape.py), and the 8-rank one-GPU
# rehearsal of the N > 1 line (RCCL transports, CTA A/B; verdict item 4).
set -o pipefail
OUT=gpurun_out/${1:-r05d}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step newton1023
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_n" -o run --output-format csv -- \
    python bench.py --size 1023 --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --vcycles 0 --config5 0 --newton-iters 1 > "$OUT/n1023.json" 2> "$OUT/n1023.err" || { tail -20 "$OUT/n1023.err"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_n -name '*kernel_trace.csv' -print -quit)" -4 --agg > "$OUT/n1023_seq.txt" && head -32 "$OUT/n1023_seq.txt"
python -c "import json; d=json.load(open('$OUT/n1023.json')); print('1023^3 newton', d['newton'])"
step pro-threshold
for r in 1 2; do
  for v in def p20; do
    if [ $v = p20 ]; then E="GS_NEWTON_PRO_POINTS=1048576"; else E="GS_NONE=1"; fi
    env $E timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/pro_${v}_r$r.json" 2> "$OUT/pro_${v}_r$r.err" || { tail "$OUT/pro_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/pro_${v}_r$r.json')); print('$v r$r', d['newton']['ms_per_iteration'])"
  done
done
step slab-pair
timeout -k 10 300 python tools/pair_shape.py 1024 1024 128 > "$OUT/slab_pair.txt" 2>&1 || { tail "$OUT/slab_pair.txt"; exit 1; }
cat "$OUT/slab_pair.txt"
timeout -k 10 300 python tools/pair_shape.py 512 512 512 > "$OUT/pair512.txt" 2>&1 || { tail "$OUT/pair512.txt"; exit 1; }
cat "$OUT/pair512.txt"
step ranks8
bash tools/bench_ranks.sh r05d/ranks8 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/ranks8/rank0.json'))
print(json.dumps({k: d.get(k) for k in ('value','scaling','rccl_cta_ab','rccl_transports')})[:3000])" || true
step done
