#!/bin/bash
# r05c: GS_NEWTON_B pairs with the shared refined reciprocal of the Jacobi denominator (div_by_recip; bit-identical
# to the division: tests/test_gpu_fastdiv.py). The whole GPU suite, an interleaved A/B against the build without it
# (gpu-solve_amd/lib_exp/norcp, -DGS_NO_NEWTON_RCP), the level-0 kernels alone in both builds, one 1023^3 Newton
# iteration's kernel trace (config #5's grid in mode 2: the column-block NEWTON prolongation pair, verdict item 6),
# and the 8-rank one-GPU rehearsal (RCCL transports in the N > 1 line, verdict item 4).
set -o pipefail
OUT=gpurun_out/${1:-r05c}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1"; exit 1; }; return 0; }
step pytest-gpu-full
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 20 > "$OUT/pytest.log" 2>&1; rc=$?
tail -15 "$OUT/pytest.log"; fatal $rc
step kprobe
for lib in product norcp; do
  L=gpu-solve_amd/lib/libgpusolve_hip.so; [ $lib = norcp ] && L=gpu-solve_amd/lib_exp/norcp/libgpusolve_hip.so
  GS_KPROBE_LIB=$PWD/$L timeout -k 10 300 python tools/newton_kprobe.py 3 10 512 > "$OUT/kprobe_$lib.json" 2> "$OUT/kprobe_$lib.err" || { tail "$OUT/kprobe_$lib.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/kprobe_$lib.json'))['ms']; print('$lib', {k: min(v) for k, v in d.items() if k.startswith('newtonb') and not k.endswith('GBps')})"
done
step lib-ab
timeout -k 10 900 bash tools/lib_ab_session.sh r05c/libab 3 2 gpu-solve_amd/lib_exp/norcp/libgpusolve_hip.so || exit 1
step newton1023
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_n" -o run --output-format csv -- \
    python bench.py --size 1023 --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --vcycles 0 --config5 0 --newton-iters 1 > "$OUT/n1023.json" 2> "$OUT/n1023.err" || { tail -20 "$OUT/n1023.err"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_n -name '*kernel_trace.csv' -print -quit)" -4 --agg > "$OUT/n1023_seq.txt" && head -32 "$OUT/n1023_seq.txt"
python -c "import json; d=json.load(open('$OUT/n1023.json')); print('1023^3 newton', d['newton'])"
step ranks8
bash tools/bench_ranks.sh r05c/ranks8 8 256 --vcycles 2 --cpu-sweeps 0 --newton-iters 0 --config5 0 > "$OUT/ranks8.log" 2>&1 || { tail -30 "$OUT/ranks8.log"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/ranks8/rank0.json'))
print(json.dumps({k: d.get(k) for k in ('value','scaling','rccl_cta_ab','rccl_transports')})[:3000])" || true
step done
