"""Timing model of a deeper-ghost Z-slab schedule on config #5's per-rank slab (1024 x 1024 x 128), one
GPU, stand-in exchange (k_fatcopy at RCCL's kernel footprint, as tools/exchange_probe.py):

  d2 (the driver, r03): every pair step exchanges two ghost planes per side; boundary planes 1-2 / 127-128
     on a high-priority stream, the exchange after them beside the next interior (HipSolver::jacobi).
  d4: ghosts four planes deep, exchanged every OTHER step. Step A (after an exchange) sweeps planes
     -1..130 in one launch (two ghost planes per side recomputed redundantly from the depth-4 ghosts), so
     step B needs no exchange: its output planes 1..128 are split into boundary planes 1-4 / 125-128
     (high-priority stream) and the interior 5..124; the depth-4 exchange of B's boundary planes runs
     beside B's interior, and the next A waits for it.

Timing only (the field values are whatever the launches leave): per step ms over K steps on the compute
stream, for stand-in workgroup counts 0 (no exchange), 8 and 32.
    python tools/exchange_probe_d4.py [K]"""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
NX, NY, NZ = 1024, 1024, 128
G = 2  # extra planes each side held by the probe's field (local plane p <-> field plane p + G)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    K += K & 1
    sys.path.insert(0, os.path.join(HERE, "..", "gpu-solve_amd"))
    import torch
    import gpusolve as gsv
    from gpusolve.devfield import DevField
    k = gsv.kernels()
    kd = gsv.diag()
    v, o, f = (DevField(NX, NY, NZ + 2 * G, fill=x) for x in (0.5, 0.0, 1.0))
    S = gsv.Stencil().to_abi()
    h = 1.0 / (NY + 1)
    least, greatest = torch.cuda.Stream.priority_range()
    main_s = torch.cuda.Stream()
    bnd_s, comm_s = torch.cuda.Stream(priority=greatest), torch.cuda.Stream(priority=greatest)
    m4 = 4 * v.ldz  # two ghost planes per side, both sides
    A = torch.rand(2 * m4, dtype=torch.float64, device="cuda")
    O = torch.empty(2 * m4, dtype=torch.float64, device="cuda")
    sink = torch.zeros(1, dtype=torch.float64, device="cuda")

    def pair(z1, z2, st):
        """the fused pair over local planes z1..z2 (internal slab sides: ghosts current)"""
        L = v.level(h)
        L.nz = z2 - z1 + 1
        L.z0 = z1 - 1
        off = 8 * (z1 - 1 + G) * v.ldz
        assert k.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr + off, o.ptr + off, f.ptr + off, None,
                                  1, 1, st.cuda_stream) == 0

    def exchange(blocks, elems):
        if blocks:
            assert kd.gs_debug_bw(4, 1, 1, blocks, O.data_ptr(), A.data_ptr(), None, elems, sink.data_ptr(),
                                  comm_s.cuda_stream) == 0

    def d2(blocks, n):
        evb = [None, None]
        ev_x = None
        for s in range(n):
            ev_a = torch.cuda.Event()
            ev_a.record(main_s)
            bnd_s.wait_event(ev_a)
            if ev_x is not None:
                bnd_s.wait_event(ev_x)
            pair(1, 2, bnd_s)
            pair(NZ - 1, NZ, bnd_s)
            evb[s & 1] = torch.cuda.Event()
            evb[s & 1].record(bnd_s)
            comm_s.wait_event(evb[s & 1])
            if s > 0:
                main_s.wait_event(evb[(s - 1) & 1])
            pair(3, NZ - 2, main_s)
            exchange(blocks, m4)
            ev_x = torch.cuda.Event()
            ev_x.record(comm_s)
        main_s.wait_event(ev_x)
        main_s.wait_event(evb[(n - 1) & 1])

    def d4(blocks, n, bw=4):
        ev_x = None
        for s in range(0, n, 2):
            if ev_x is not None:
                main_s.wait_event(ev_x)
            pair(1 - G, NZ + G, main_s)  # A: one launch over the owned planes and two ghost planes per side
            ev_a = torch.cuda.Event()
            ev_a.record(main_s)
            bnd_s.wait_event(ev_a)
            pair(1, bw, bnd_s)  # B: boundary planes first
            pair(NZ - bw + 1, NZ, bnd_s)
            ev_b = torch.cuda.Event()
            ev_b.record(bnd_s)
            comm_s.wait_event(ev_b)
            pair(bw + 1, NZ - bw, main_s)  # B's interior beside the exchange
            exchange(blocks, 2 * m4)
            ev_x = torch.cuda.Event()
            ev_x.record(comm_s)
            main_s.wait_event(ev_b)
        main_s.wait_event(ev_x)

    def timed(fn, *args):
        for _ in range(2):
            fn(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        fn(*args)
        e1.record(main_s)
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / K, 4)

    res = {}
    for _ in range(2):  # interleaved repeats
        for b in (0, 8, 32):
            res.setdefault(f"d2 exchange x{b}", []).append(timed(d2, b, K))
            res.setdefault(f"d4 exchange x{b}", []).append(timed(d4, b, K))
    for _ in range(2):
        pair(1, NZ, main_s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main_s)
    for _ in range(K):
        pair(1, NZ, main_s)
    e1.record(main_s)
    torch.cuda.synchronize()
    res["unsplit pair, no exchange"] = [round(e0.elapsed_time(e1) / K, 4)]
    print(json.dumps({"slab": [NX, NY, NZ], "steps": K, "step_ms": res}, indent=1))


if __name__ == "__main__":
    main()
