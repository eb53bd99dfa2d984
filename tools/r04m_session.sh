#!/bin/bash
# r04m: the NEWTON column-block edge-value schemes on one box, 1023^3 level-0 kernels interleaved (tools/newton_kprobe.py
# through GS_KPROBE_LIB): product (packed slots in the plain pairs, per-step loads in the prolongation pairs),
# lib_alt/elate (per-step loads in both), lib_alt/packed (packed slots in both).
set -o pipefail
OUT=gpurun_out/${1:-r04m}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for v in product elate packed; do
    lib=$PWD/gpu-solve_amd/lib/libgpusolve_hip.so
    [ "$v" != product ] && lib=$PWD/gpu-solve_amd/lib_alt/$v/libgpusolve_hip.so
    GS_KPROBE_LIB=$lib timeout -k 10 300 python tools/newton_kprobe.py 2 3 1023 > "$OUT/kp_${v}_r$r.json" 2> "$OUT/kp_${v}_r$r.err" || { tail -20 "$OUT/kp_${v}_r$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/kp_${v}_r$r.json'))['ms']; print('$v r$r', {k: min(x) for k, x in d.items() if k.startswith('newton') and isinstance(x, list)})"
  done
done
