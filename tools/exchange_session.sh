#!/bin/bash
# The Z-slab exchange probe on the MI355X box (through gpurun, from the repo root):
#   tools/exchange_session.sh <tag>      [PROBE_MASK=1: also the CU-masked interior stream]
# step times per ordering variant (tools/exchange_probe.py), then one kernel trace of a short run.
set -o pipefail
O=gpurun_out/${1:-exch}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/exchange_probe.py 20 > $O/probe.json 2> $O/probe.err || { tail $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python tools/exchange_probe.py 3 > $O/probe_prof.log 2>&1 || tail -3 $O/probe_prof.log
