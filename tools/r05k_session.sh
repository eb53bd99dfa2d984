#!/bin/bash
# r05k: GS_NEWTON_G (the first Newton iteration's inner solve takes gamma for its factor in the pairs and k_rr2). The
# NEWTON tests (kernels, switches, Z-slab, solver anchors), then bench.py with the driver's flags, default and
# GS_NO_NEWTON_G=1 interleaved (the bench line now times the first iteration alone as well).
set -o pipefail
OUT=gpurun_out/${1:-r05k}; mkdir -p $OUT; export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest-newton
timeout -k 10 900 python -u -m pytest tests/test_gpu_newton_b.py tests/test_gpu_switches.py tests/test_gpu_zslab.py tests/test_gpu_newton_update.py -m gpu -q --timeout 300 --timeout-method thread -k "newton or Newton or NEWTON or zslab or slab" > "$OUT/pytest.log" 2>&1; rc=$?
tail -5 "$OUT/pytest.log"; [ $rc -ge 124 ] && exit 1
step bench
for r in 1 2; do
  for v in g nog; do
    if [ $v = nog ]; then export GS_NO_NEWTON_G=1; else unset GS_NO_NEWTON_G; fi
    timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sweeps 0 > "$OUT/bench_${v}_r$r.json" 2> "$OUT/bench_${v}_r$r.err" || { tail -20 "$OUT/bench_${v}_r$r.err"; exit 1; }
    echo -n "$v r$r "; python tools/bench_brief.py "$OUT/bench_${v}_r$r.json" || true
  done
done
unset GS_NO_NEWTON_G
step done
