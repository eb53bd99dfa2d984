#!/bin/bash
# r04u: NEWTON k_rr2 with newtonV loaded where the residual uses it (165 VGPRs, three waves per SIMD instead of
# two; lib_alt/wlate) against the product: the level-0 kernel probe and bench.py's V-cycle + Newton, interleaved
# (tools/lib_ab_session.sh), then the NEWTON tests with the alternative library in place.
set -o pipefail
OUT=gpurun_out/${1:-r04u}
mkdir -p "$OUT"
export TMPDIR=/tmp
ALT=$PWD/gpu-solve_amd/lib_alt/wlate/libgpusolve_hip.so
for r in 1 2; do
  for v in product wlate; do
    lib=$PWD/gpu-solve_amd/lib/libgpusolve_hip.so; [ $v = wlate ] && lib=$ALT
    GS_KPROBE_LIB=$lib timeout -k 10 200 python tools/newton_kprobe.py 2 10 > "$OUT/kp_${v}_r$r.json" 2> "$OUT/kp_${v}_r$r.err" || { tail -20 "$OUT/kp_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/kp_${v}_r$r.json'))['ms']; print('$v r$r', {k: min(x) for k, x in d.items() if k.startswith('newton_rr') and isinstance(x, list)})"
  done
done
bash tools/lib_ab_session.sh ${1:-r04u}/ab 3 2 $ALT || exit 1
L=gpu-solve_amd/lib
cp $L/libgpusolve_hip.so "$OUT/product.so"
trap 'cp "$OUT/product.so" $L/libgpusolve_hip.so' EXIT INT TERM
cp $ALT $L/libgpusolve_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_newton_update.py tests/test_gpu_newton_pro.py tests/test_gpu_solver.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest_wlate.log" 2>&1 || { tail -30 "$OUT/pytest_wlate.log"; exit 1; }
tail -1 "$OUT/pytest_wlate.log"
