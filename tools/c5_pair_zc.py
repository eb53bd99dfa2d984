#!/usr/bin/env python3
"""Config #5's 1024^3 pair (column blocks) under one z-chunk setting: bench.py's config5_single_gpu leg alone (no
V-cycles), one JSON line. Run one process per setting, since the library reads GS_PAIR_ZC once at load:
    GS_PAIR_ZC=1024 python tools/c5_pair_zc.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
r = bench.config5_single_gpu(steps, 0)
r.pop("note", None)
r["GS_PAIR_ZC"] = os.environ.get("GS_PAIR_ZC", "default")
print(json.dumps(r))
