#!/bin/bash
# r04o: GS_SPEC_CACHED (the speculative pre-smoothing pair stores through the caches, so that k_rr2, which reads
# its last planes first, finds them in the Infinity Cache) on the linear V-cycle and the Newton iteration,
# interleaved, one process per run.
set -o pipefail
OUT=gpurun_out/${1:-r04o}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/knob_ab.sh ${1:-r04o}/vc GS_SPEC_CACHED 3 0 1 || exit 1
for r in 1 2 3; do
  for v in 0 1; do
    GS_SPEC_CACHED=$v timeout -k 10 300 python bench.py --steps 4 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 2 \
      > "$OUT/n_${v}_r$r.json" 2> "$OUT/n_${v}_r$r.err" || { tail "$OUT/n_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/n_${v}_r$r.json')); print('GS_SPEC_CACHED=$v r$r newton', d['newton']['ms_per_iteration'])"
  done
done
