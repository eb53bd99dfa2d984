#!/bin/bash
# r04b: Z-slab / Newton-update GPU tests after the exchange and fused-update changes, the NEWTON level-0
# kernels under timing-only builds (barrier / exp / division removed), and the exchange probe per stand-in
# workgroup count.
set -o pipefail
OUT=gpurun_out/${1:-r04b}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests/test_gpu_zslab.py tests/test_gpu_newton_update.py tests/test_gpu_switches.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for lib in product nobar noexp nodiv all3; do
  step "kprobe $lib"
  if [ $lib = product ]; then
    timeout -k 10 300 python tools/newton_kprobe.py 3 10 > "$OUT/kprobe_$lib.json" 2> "$OUT/kprobe_$lib.err" || { tail -20 "$OUT/kprobe_$lib.err"; exit 1; }
  else
    GS_KPROBE_LIB=gpu-solve_amd/lib_alt/$lib/libgpusolve_hip.so timeout -k 10 300 python tools/newton_kprobe.py 3 10 > "$OUT/kprobe_$lib.json" 2> "$OUT/kprobe_$lib.err" || { tail -20 "$OUT/kprobe_$lib.err"; exit 1; }
  fi
  cat "$OUT/kprobe_$lib.json"
done
step exchange-probe
PROBE_WGS=0,8,16,32,64,128 PROBE_ROUNDS=2 timeout -k 10 300 python tools/exchange_probe.py 20 > "$OUT/exchange_wgs.json" 2> "$OUT/exchange_wgs.err" || { tail -20 "$OUT/exchange_wgs.err"; exit 1; }
cat "$OUT/exchange_wgs.json"
step done
