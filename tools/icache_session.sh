#!/bin/bash
# Instruction-cache counters (SQC block, one pass of their own) over the linear V-cycle and one Newton
# iteration: do the larger fused kernels (21-42 KB of code, mirrored / unrolled step bodies) miss in the
# instruction cache?   tools/icache_session.sh <tag>          (through gpurun, from the repo root)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-icache}; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*" $O/avail.txt | sort -u > $O/sqc_counters.txt || true
cat $O/sqc_counters.txt
SET="SQC_ICACHE_HITS SQC_ICACHE_MISSES"
for prog in vc_pmc newton_prof; do
  timeout -s KILL 180 rocprofv3 --pmc $SET -d $O/$prog -o run --output-format csv -- python tools/$prog.py > $O/$prog.log 2>&1 \
    || { tail -20 $O/$prog.log; exit 1; }
  python tools/pmc_summary.py $O/$prog --md $O/${prog}_icache.md > /dev/null && grep -E "^###|ICACHE" $O/${prog}_icache.md
done
