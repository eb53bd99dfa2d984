#!/bin/bash
# r05l: r05k's GS_NEWTON_G validation (NEWTON tests, bench default vs GS_NO_NEWTON_G=1), then an interleaved A/B of the
# LINEAR prolongation pair at two plane steps of prefetch with its coarse X-pass rows in LDS (lib_exp/lpro2,
# -DGS_EXP_LPRO2: 250 VGPRs, no spill, 84 KB LDS) against the product.
set -o pipefail
OUT=gpurun_out/${1:-r05l}; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/r05k_session.sh ${1:-r05l}/k || exit 1
echo "[$(date +%T)] lpro2 A/B"
timeout -k 10 900 bash tools/multi_lib_ab.sh $OUT/ab 3 0 product lpro2 || exit 1
