#!/bin/bash
# r05g: interleaved A/B of the product library against two experiment builds: norecomp (-DGS_EXP_B_NORECOMP: NEWTON_B
# prolongation pairs keep sweep 2's B / f rows in registers) and touch (-DGS_EXP_TOUCH: NEWTON-mode pairs and k_rr2
# prefetch the next plane's operand lines into L2 / MALL with one-dword loads consumed two steps later).
set -o pipefail
OUT=gpurun_out/${1:-r05g}
mkdir -p "$OUT"
timeout -k 10 1100 bash tools/multi_lib_ab.sh $OUT 4 2 product norecomp touch
