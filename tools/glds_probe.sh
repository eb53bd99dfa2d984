#!/bin/bash
# Compile tools/glds_probe.hip for gfx950 and list the loop's LDS-DMA issues, LDS reads and waits
# (CPU only, no GPU needed). Output: the instruction sequence of the loop body.
set -euo pipefail
d=$(mktemp -d)
here=$(cd "$(dirname "$0")" && pwd)
(cd "$d" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -c "$here/glds_probe.hip" --save-temps -o p.o 2>/dev/null)
s=$(ls "$d"/*gfx950*.s)
awk '/Inner Loop Header/{on=1} on && /global_load_lds|ds_read|s_waitcnt vmcnt|s_cbranch/{print} /s_cbranch_scc0/{if(on) exit}' "$s"
rm -rf "$d"
