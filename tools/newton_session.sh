set -o pipefail
# Newton session on the MI355X box: fused-prolongation parity tests, a kernel trace of one 512^3
# Newton iteration (tools/newton_prof.py) and a bench run with 3 Newton iterations.
export TMPDIR=/tmp
O=gpurun_out/${1:-newton}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_newton_pro.py tests/test_gpu_sweep2.py tests/test_gpu_solver.py -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -2 $O/pt.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/np2 -o run --output-format csv -- python tools/newton_prof.py > $O/np2.log 2>&1 || { tail -20 $O/np2.log; exit 1; }
python tools/kernel_agg.py $O/np2/run_kernel_trace.csv > $O/np2.txt && head -14 $O/np2.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 20 --cpu-sweeps 0 --newton-iters 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d.get('vcycle'), d.get('newton'))"
