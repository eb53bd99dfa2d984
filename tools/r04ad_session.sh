#!/bin/bash
# r04ad: the 256^3 level's LINEAR pairs (prolongation pair, plain pairs) in one round of blocks
# (GS_PAIR_ONE_ROUND_MID=1) against the default four rounds, on the V-cycle, interleaved; then its switch test.
set -o pipefail
bash tools/knob_ab.sh ${1:-r04ad}/vc GS_PAIR_ONE_ROUND_MID 4 0 1 || exit 1
