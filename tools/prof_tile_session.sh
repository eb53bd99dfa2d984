set -o pipefail
O=gpurun_out/r03e; mkdir -p $O; export TMPDIR=/tmp
for t in 0 262144; do
GS_TILE_POINTS=$t timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_t$t -o run --output-format csv -- python bench.py --steps 2 --warmup 2 --ramp-ms 50 --vcycles 6 --cpu-sweeps 0 --newton-iters 0 --config5 0 > $O/b_t$t.json 2> $O/b_t$t.err || { tail $O/b_t$t.err; exit 1; }
python tools/vc_breakdown.py $(find $O/prof_t$t -name "*kernel_trace.csv" | head -1) 40 --seq > $O/vc_t$t.txt && cat $O/vc_t$t.txt
done
