#!/bin/bash
# r04ac: with 64-plane k_rr2 chunks, re-check k_rr2's non-temporal loads (GS_RR_NTU=0: cached) and its reversed
# chunk order (GS_RR_REVERSE=0) on the V-cycle, interleaved.
set -o pipefail
bash tools/knob_ab.sh ${1:-r04ac}/ntu GS_RR_NTU 3 1 0 || exit 1
bash tools/knob_ab.sh ${1:-r04ac}/rev GS_RR_REVERSE 3 1 0 || exit 1
