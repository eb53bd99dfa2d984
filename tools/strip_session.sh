#!/bin/bash
# The column-block prolongation path after a change to k_pro_strip: its parity tests, then a kernel trace
# of config #5's grid on one GPU (strip and PRO pair times):   tools/strip_session.sh <tag>
set -o pipefail
O=gpurun_out/${1:-strip}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep2.py tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread -k "prolong or fields_bit" > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
tail -1 $O/p.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_zslab.py tests/test_gpu_config5.py -x -q --timeout 300 --timeout-method thread > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
tail -1 $O/p2.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --size 1024 --steps 4 --warmup 2 --ramp-ms 100 --vcycles 4 --cpu-sweeps 0 --newton-iters 0 --config5 0 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
python tools/vc_breakdown.py $(find $O/prof -name "*kernel_trace.csv" | head -1) 12 | tee $O/vc.txt
python -c "import json; d=json.load(open('$O/b.json')); print('vcycle_ms', d['vcycle']['ms'])"
# one 512^3 Newton iteration (config #4), kernel totals (SKIP_NEWTON=1: not)
[ -n "$SKIP_NEWTON" ] || timeout -k 10 300 rocprofv3 --kernel-trace -d $O/nprof -o run --output-format csv -- python tools/newton_prof.py 512 > $O/n.log 2>&1 || { tail $O/n.log; exit 1; }
[ -n "$SKIP_NEWTON" ] || python tools/kernel_agg.py $(find $O/nprof -name "*kernel_trace.csv" | head -1) 30 | tee $O/newton_kernels.txt
# the pipelined Z-slab exchange probe (boundary launches serial vs on two streams)
PROBE_ONLY_PIPE=1 timeout -k 10 300 python -u tools/exchange_probe.py > $O/probe.json 2> $O/probe.err || { tail $O/probe.err; exit 1; }
cat $O/probe.json
