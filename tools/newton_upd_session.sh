set -o pipefail
mkdir -p gpurun_out/r03aa
timeout -k 10 300 python -u -m pytest tests/test_gpu_newton_update.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r03aa/pytest.log 2>&1 || { tail -20 gpurun_out/r03aa/pytest.log; exit 1; }
tail -1 gpurun_out/r03aa/pytest.log
for r in 1 2; do for x in 0 1; do GS_NEWTON_UPD_XCD=$x timeout -k 10 120 python tools/newton_upd_probe.py || exit 1; done; done
for x in 0 1; do
  GS_NEWTON_UPD_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03aa/pmc_$x -o run --output-format csv -- python tools/newton_upd_probe.py 512 3 > gpurun_out/r03aa/pmc_$x.log 2>&1 || { tail gpurun_out/r03aa/pmc_$x.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/r03aa/pmc_$x | grep -A2 "k_newton_upd\|k_rb" | grep -v "^--"
done
