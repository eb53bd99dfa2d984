#!/bin/bash
# r06al: config #5's column-block pair at one plane step of prefetch with its x-edge values in VGPRs (GS_TBX_PFD=1) against
# the default two steps: the 1024^3 pair leg and the per-rank slab pair, interleaved, plus the pair tests on the build.
set -o pipefail
O=gpurun_out/r06al; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep2.py tests/test_gpu_config5.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GS_TBX_PFD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep2.py tests/test_gpu_config5.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_pfd1.log 2>&1 || { tail -30 $O/pytest_pfd1.log; exit 1; }
tail -1 $O/pytest_pfd1.log
for r in 1 2 3; do
  for v in 2 1; do
    GS_TBX_PFD=$v timeout -k 10 200 python tools/c5_pair_zc.py 20 > $O/c5_$v_r$r.json 2>/dev/null || exit 1
    GS_TBX_PFD=$v timeout -k 10 200 python tools/pair_shape.py 1024 1024 128 > $O/slab_$v_r$r.txt 2>/dev/null || exit 1
    python -c "
import json; c=json.load(open('$O/c5_$v_r$r.json')); print('GS_TBX_PFD=$v r$r c5 pair', c['pair_kernel_ms'], c['pair_frac'], 'slab', open('$O/slab_$v_r$r.txt').read().split(':')[1].split(',')[0])"
  done
done
