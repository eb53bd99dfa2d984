#!/bin/bash
# The pipelined Z-slab step (tools/exchange_probe.py, PROBE_ONLY_PIPE) under several interior chunk
# lengths, one process each (GS_SLAB_ZC is read once when the library loads):
#   tools/zc_probe_session.sh <tag> [zc ...]
set -o pipefail
O=gpurun_out/${1:-zcp}; shift; mkdir -p $O; export TMPDIR=/tmp
for zc in ${@:-0 64 42 32}; do
  GS_SLAB_ZC=$zc PROBE_ONLY_PIPE=1 timeout -k 10 120 python tools/exchange_probe.py 20 > $O/probe_zc$zc.json 2> $O/probe_zc$zc.err || { tail $O/probe_zc$zc.err; exit 1; }
  grep pipelined $O/probe_zc$zc.json
done
