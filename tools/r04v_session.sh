#!/bin/bash
# r04v: config #5's grid on one GPU at the round's final tree: a kernel trace of 1024^3 linear V-cycles as a
# norm-to-norm launch sequence (tools/trace_seq.py), and the same for one 1023^3 Newton iteration's inner cycle.
set -o pipefail
OUT=gpurun_out/${1:-r04v}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vc" -o run --output-format csv -- \
    python bench.py --size 1024 --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --newton-iters 0 --config5 0 --vcycles 4 > "$OUT/vc.json" 2> "$OUT/vc.err" || { tail -20 "$OUT/vc.err"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_vc -name '*kernel_trace.csv' -print -quit)" -3 > "$OUT/vc1024_seq.txt" && cat "$OUT/vc1024_seq.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_n" -o run --output-format csv -- \
    python bench.py --size 1023 --steps 2 --warmup 2 --ramp-ms 0 --cpu-sweeps 0 --vcycles 0 --config5 0 --newton-iters 1 > "$OUT/n.json" 2> "$OUT/n.err" || { tail -20 "$OUT/n.err"; exit 1; }
python tools/trace_seq.py "$(find $OUT/prof_n -name '*kernel_trace.csv' -print -quit)" -4 --agg > "$OUT/n1023_seq.txt" && head -40 "$OUT/n1023_seq.txt"
