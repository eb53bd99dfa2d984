#!/bin/bash
# r05af: the GS_NEWTON_B zero-iterate pairs (level 1 every inner V-cycle, level 0 once per findError) at two plane
# steps of prefetch (zvpfd2, -DGS_EXP_ZVPFD2: 205 VGPRs, no spill) against the product (one step, 177), 3 rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05af}; mkdir -p $OUT
timeout -k 10 1000 bash tools/multi_lib_ab.sh $OUT 3 2 product zvpfd2
