"""When does a small kernel on another stream get CUs while a level-0 pair holds the GPU? (the Z-slab
exchange path: RCCL's transport kernels run beside the interior pair). 512^3 pair on a normal-priority
stream, then — while it runs — a 16-block copy kernel (gs_debug_bw, 8 MB, standing in for one ghost
exchange) on a high- or normal-priority stream; the pair over the whole level (z0 = 0: one round of
blocks) or as an interior range (z0 = 2: two rounds, tb2_plan).
    rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python tools/overlap_probe.py
    python tools/overlap_probe.py --analyze <dir>/run_kernel_trace.csv"""
import csv
import ctypes as C
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def analyze(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    pair = None
    out = {}
    for r in rows:
        name, t0, t1 = r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "k_tb2y" in name:
            pair = (t0, t1, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) * int(r["Grid_Size_Y"]) // int(r["Workgroup_Size_Y"]))
        elif "k_bw" in name and pair and int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) == 16:
            p0, p1, blocks = pair
            key = blocks
            out.setdefault(key, []).append(((t0 - p0) / 1e3, (t1 - p1) / 1e3, (p1 - p0) / 1e3, (t1 - t0) / 1e3))
    for blocks, v in out.items():
        print(f"pair of {blocks} blocks: small kernel start - pair start / end - pair end / pair length / own length (us)")
        for a in v:
            print("   " + "  ".join(f"{x:8.1f}" for x in a))


def main():
    sys.path.insert(0, os.path.join(HERE, "..", "gpu-solve_amd"))
    import torch
    import gpusolve as gsv
    from gpusolve.devfield import DevField
    k = gsv.kernels()
    kd = gsv.diag()
    n = 512
    v, o, f = DevField(n, n, n, fill=0.5), DevField(n, n, n), DevField(n, n, n, fill=1.0)
    S = gsv.Stencil().to_abi()
    main_s = torch.cuda.Stream()
    least, greatest = torch.cuda.Stream.priority_range()
    hi_s, lo_s = torch.cuda.Stream(priority=greatest), torch.cuda.Stream(priority=least)
    m = 1 << 20
    A = torch.rand(m, dtype=torch.float64, device="cuda")
    B = torch.rand(m, dtype=torch.float64, device="cuda")
    O = torch.empty(m, dtype=torch.float64, device="cuda")
    sink = torch.zeros(1, dtype=torch.float64, device="cuda")
    for z0 in (0, 2, 0, 2, 0, 2):
        L = v.level(1.0 / (n + 1), z0)
        for side in (hi_s, lo_s):
            assert k.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, o.ptr, f.ptr, None, 0, 0,
                                      main_s.cuda_stream) == 0
            time.sleep(50e-6)
            assert kd.gs_debug_bw(2, 1, 1, 16, O.data_ptr(), A.data_ptr(), B.data_ptr(), m, sink.data_ptr(),
                                 side.cuda_stream) == 0
            torch.cuda.synchronize()
    print("priority range", least, greatest)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        main()
