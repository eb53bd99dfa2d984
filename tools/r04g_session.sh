#!/bin/bash
# r04g: E = exp(newtonV) as a field (timing-only build lib_alt/efield, -DGS_EXP_EFIELD) against the product on
# the NEWTON level-0 kernels (tools/newton_kprobe.py, interleaved), and one 1024^3 Newton iteration (config #5's
# grid in mode 2: 1024-point rows, the column-block NEWTON prolongation pair) through bench.py, after the
# prolongation-pair tests.
set -o pipefail
OUT=gpurun_out/${1:-r04g}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest-pro
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep2.py tests/test_gpu_newton_pro.py -m gpu -x -q -k "prolong or newton" \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2 3; do
  step "kprobe round $r"
  timeout -k 10 200 python tools/newton_kprobe.py 2 10 > "$OUT/kp_product_r$r.json" 2> "$OUT/kp_product_r$r.err" || { tail -20 "$OUT/kp_product_r$r.err"; exit 1; }
  GS_KPROBE_LIB=$PWD/gpu-solve_amd/lib_alt/efield/libgpusolve_hip.so GS_KPROBE_EFIELD=1 \
    timeout -k 10 200 python tools/newton_kprobe.py 2 10 > "$OUT/kp_efield_r$r.json" 2> "$OUT/kp_efield_r$r.err" || { tail -20 "$OUT/kp_efield_r$r.err"; exit 1; }
  for v in product efield; do
    python -c "import json; d=json.load(open('$OUT/kp_${v}_r$r.json'))['ms']; print('$v r$r', {k: min(x) for k, x in d.items() if k.startswith('newton') and isinstance(x, list)})"
  done
done
step newton-1024
timeout -k 10 400 python bench.py --size 1024 --steps 2 --warmup 2 --vcycles 2 --cpu-sweeps 0 --config5 0 --newton-iters 1 \
  > "$OUT/newton1024.json" 2> "$OUT/newton1024.err" || { tail -20 "$OUT/newton1024.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/newton1024.json')); print('1024^3 newton', d['newton']); print('vcycle', d['vcycle']['ms'])"
step newton-1024-trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_n1024" -o run --output-format csv -- \
  python bench.py --size 1024 --steps 2 --warmup 2 --vcycles 0 --cpu-sweeps 0 --config5 0 --newton-iters 1 > "$OUT/prof_n1024.json" 2> "$OUT/prof_n1024.err" || { tail -20 "$OUT/prof_n1024.err"; exit 1; }
python tools/kernel_agg.py "$(find $OUT/prof_n1024 -name '*kernel_trace.csv' -print -quit)" > "$OUT/n1024_agg.txt" || true
head -25 "$OUT/n1024_agg.txt" || true
step done
