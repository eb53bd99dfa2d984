set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pf1; mkdir -p $O
timeout -k 10 300 python tools/kbench.py --pairs --zc 64,32 --variants 0 --rounds 7 --out $O/kb512.json > $O/kb512.log 2>&1 || { tail -20 $O/kb512.log; exit 1; }
timeout -k 10 300 python tools/kbench.py --n 301 --ny 77 --nz 131 --pairs --zc 64,6 --variants 0 --rounds 2 --out $O/kbodd.json > $O/kbodd.log 2>&1 || { tail -20 $O/kbodd.log; exit 1; }
python - <<'P'
import json
for fn in ("gpurun_out/pf1/kb512.json","gpurun_out/pf1/kbodd.json"):
    d=json.load(open(fn))
    pv=d.get("pairs") or d.get("pair_variants") or {}
    print(fn)
    for k,v in pv.items(): print(f"  {k:50s} {v.get('median_ms_per_pair')} eq={v.get('bitwise_equal_to_two_sweeps')}")
P
