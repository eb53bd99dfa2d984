#!/usr/bin/env python3
"""BASELINE config #2 (128^3 linear 2+2) V-cycles for a kernel trace: one warm-up solve, then --cycles V-cycles
through gs_grid_time_vcycles; prints ms per cycle.   python tools/cfg2_probe.py [--n 128] [--cycles 50]"""
import argparse
import ctypes as C
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=128)
ap.add_argument("--cycles", type=int, default=50)
ap.add_argument("--mode", type=int, default=0)
a = ap.parse_args()
p = gsv.GridParams(maxiter=10, tol=0.0, gridDim=(a.n, a.n, a.n), mode=a.mode, preSmoothing=2, postSmoothing=2)
with gsv.HipGridData(p) as g:
    gsv.NewtonSolver.solve(g) if a.mode == gsv.GS_NEWTON else gsv.HipSolver.solve(g)
    ms, last = C.c_double(), C.c_double()
    assert gsv.driver().gs_grid_time_vcycles(g.handle, a.cycles, C.byref(ms), C.byref(last)) == 0
    print(f"{a.n}^3 mode {a.mode}: {ms.value / a.cycles:.4f} ms per V-cycle ({os.environ.get('GS_CC_LDS', 'default')})")
