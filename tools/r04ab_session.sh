#!/bin/bash
# r04ab: pair chunks on levels below 2^26 points for the LINEAR V-cycle (GS_MID_ZC: 256^3's prolongation pair runs
# 1024 blocks = four rounds by default; 64-plane chunks = one round), interleaved.
set -o pipefail
bash tools/knob_ab.sh ${1:-r04ab}/vc GS_MID_ZC 3 0 32 64 || exit 1
