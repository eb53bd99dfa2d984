set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmb; mkdir -p $O
for val in 512 128 32; do
  GS_PAIR_MIN_BLOCKS=$val timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$val.log 2>&1 || { tail -30 $O/pytest_$val.log; exit 1; }
  tail -1 $O/pytest_$val.log
done
for rep in 1 2; do for val in 512 128 32; do
  GS_PAIR_MIN_BLOCKS=$val timeout -k 10 300 python bench.py --steps 20 --vcycles 100 --cpu-sweeps 0 --newton-iters 0 > $O/b_${val}_$rep.json 2>$O/b_${val}_$rep.err || exit 1
  echo "$val $(python tools/bench_brief.py $O/b_${val}_$rep.json)"
done; done
for val in 512 32; do
  GS_PAIR_MIN_BLOCKS=$val timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$val -o run -- python bench.py --steps 20 --vcycles 5 --cpu-sweeps 0 --newton-iters 0 > $O/prof_$val.log 2>&1 || exit 1
  echo "== $val"; python tools/vc_breakdown.py $(find $O/prof_$val -name '*kernel_trace.csv' -print -quit) 30
done
