set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
for c in 0 1; do
  GS_CC_LDS=$c timeout -k 10 120 python tools/cfg2_probe.py || exit 1
done
for c in 0 1; do
  GS_CC_LDS=$c timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/cc$c -o run --output-format csv -- python tools/cfg2_probe.py > $O/cc$c.log 2>&1 || exit 1
done
python - <<'PY'
import csv, glob
for c in (0, 1):
    f = glob.glob(f"gpurun_out/r06j/cc{c}/**/*kernel_stats.csv", recursive=True)[0]
    print("GS_CC_LDS", c)
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.2f} tot% {float(r['Percentage']):5.1f}")
PY
