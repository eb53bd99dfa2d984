"""One line per bench.py JSON file: headline, pair kernel ms, roofline frac, V-cycle ms, Newton ms."""
import json
import sys

for fn in sys.argv[1:]:
    d = json.load(open(fn))
    r = d["roofline"]
    v = d.get("vcycle") or {}
    n = d.get("newton") or {}
    print(f"{fn.split('/')[-1]:34s} value {d['value']:10.1f} kernel_ms {r['kernel_ms']:.4f} frac {r['frac']:.4f} "
          f"vcycle_ms {v.get('ms')} newton_ms {n.get('ms_per_iteration')} (first {n.get('ms_first_iteration')} later {n.get('ms_per_later_iteration')}) {r['kernel'][:24]}")
