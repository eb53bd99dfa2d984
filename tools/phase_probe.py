#!/usr/bin/env python3
"""Per-phase cost of one workgroup's [work -> store -> barrier] rounds (gs_debug_phase_probe), the floor under the
one-launch coarse cycle (k_coarse_cycle: ~25 phases, ~26 us on config #2).   python tools/phase_probe.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402

kd = gsv.diag()
st = torch.cuda.current_stream()
g = torch.rand(16384, dtype=torch.float64, device="cuda")
sink = torch.zeros(1, dtype=torch.float64, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for work in (0, 1, 2):
    for threads in (512, 1024):
        res = {}
        for phases in (1, 101):
            for _ in range(3):
                assert kd.gs_debug_phase_probe(work, threads, phases, g.data_ptr(), sink.data_ptr(), st.cuda_stream) == 0
            e0.record(st)
            for _ in range(20):
                kd.gs_debug_phase_probe(work, threads, phases, g.data_ptr(), sink.data_ptr(), st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            res[phases] = e0.elapsed_time(e1) / 20 * 1e3
        print(f"work {work} threads {threads}: launch {res[1]:.2f} us, per phase {(res[101] - res[1]) / 100 * 1e3:.0f} ns")
