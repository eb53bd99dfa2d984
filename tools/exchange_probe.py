"""One overlapped Z-slab pair step of config #5's per-rank slab (1024 x 1024 x 128) on one GPU, with a
stand-in for the RCCL exchange: the boundary planes (two per side) on a high-priority stream, then a
copy at the footprint of RCCL's gfx950 transport kernels (gs_debug_bw kind 4: 256 VGPRs, 37 KB LDS
per workgroup; 17 MB = one neighbour's two ghost planes each way) on a second high-priority stream,
and the interior planes 3..126 on the compute stream — unmasked, or on a stream whose CU mask leaves
R CUs per XCD free (the driver's GS_EXCHANGE_CUS, gs_grid.cpp MaskedStream). Reports, per setting,
the step time on the compute stream (fork to join, HIP events) and, from a kernel trace, when the
stand-in exchange started and ended relative to the interior launch.
    python tools/exchange_probe.py [reps]                    (step times)
    rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python tools/exchange_probe.py 3
    python tools/exchange_probe.py --analyze <dir>/run_kernel_trace.csv
r03: 'pipelined xK' times K consecutive steps under the driver's pipelined schedule (HipSolver::jacobi),
per step: exchange k overlaps interior k+1, the compute stream never waits for an exchange."""
import csv
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
NX, NY, NZ = 1024, 1024, 128


def mask_words(cus, per_xcd):
    """gs_grid.cpp MaskedStream::mask: bits 33x + 8r cleared (one per XCD under either bit mapping)."""
    m = [0] * ((cus + 31) // 32)
    for b in range(cus):
        m[b // 32] |= 1 << (b % 32)
    if cus == 256:
        for r in range(min(per_xcd, 3)):
            for x in range(8):
                b = 33 * x + 8 * r
                m[b // 32] &= ~(1 << (b % 32))
    return m


def analyze(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    interior, steps = None, []
    for r in rows:
        name, t0, t1 = r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "k_tb2y" in name and t1 - t0 > 200000:
            interior = (t0, t1)  # the interior launch (boundary launches: 2 planes, < 100 us)
        elif "k_fatcopy" in name and interior:
            i0, i1 = interior
            steps.append(((t0 - i0) / 1e3, (t1 - i1) / 1e3, (i1 - i0) / 1e3, (t1 - t0) / 1e3))
    print("stand-in exchange start - interior start / end - interior end / interior length / own length (us)")
    for a in steps:
        print("   " + "  ".join(f"{x:8.1f}" for x in a))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sys.path.insert(0, os.path.join(HERE, "..", "gpu-solve_amd"))
    import torch
    import gpusolve as gsv
    from gpusolve.devfield import DevField
    k = gsv.kernels()
    kd = gsv.diag()
    hip = C.CDLL("libamdhip64.so")
    v, o, f = DevField(NX, NY, NZ, fill=0.5), DevField(NX, NY, NZ), DevField(NX, NY, NZ, fill=1.0)
    S = gsv.Stencil().to_abi()
    h = 1.0 / (NY + 1)
    least, greatest = torch.cuda.Stream.priority_range()
    main_s = torch.cuda.Stream()
    bnd_s, comm_s = torch.cuda.Stream(priority=greatest), torch.cuda.Stream(priority=greatest)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    streams = {0: main_s}
    for r in ((1,) if os.environ.get("PROBE_MASK") else ()):
        words = mask_words(cus, r)
        raw = C.c_void_p()
        arr = (C.c_uint32 * len(words))(*words)
        assert hip.hipExtStreamCreateWithCUMask(C.byref(raw), len(words), arr) == 0
        streams[r] = torch.cuda.ExternalStream(raw.value)
    m = 2 * 2 * v.ldz  # two ghost planes each way
    A = torch.rand(m, dtype=torch.float64, device="cuda")
    O = torch.empty(m, dtype=torch.float64, device="cuda")
    sink = torch.zeros(1, dtype=torch.float64, device="cuda")

    def sub(z1, z2):
        L = v.level(h)
        L.nz = z2 - z1 + 1
        L.z0 = z1 - 1
        off = 8 * (z1 - 1) * v.ldz
        return L, off

    def pair(z1, z2, st):
        L, off = sub(z1, z2)
        assert k.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr + off, o.ptr + off, f.ptr + off, None,
                                  1, 1, st.cuda_stream) == 0

    bnd2_s = torch.cuda.Stream(priority=greatest)

    def step2(variant, blocks):
        """variant: 'cur' boundary planes in sequence on one stream, interior concurrent (r02 driver);
        'two' both boundary launches on their own streams, interior concurrent; 'first' both on their own
        streams and the interior waits for them (the exchange and the interior become ready together);
        'first-mask' the same with the interior on the 1-CU-per-XCD masked stream; 'delay-n' as 'first',
        with the interior also waiting for a one-wave kernel of n x s_sleep(127) (~3.4 us each) started
        after the boundary planes, so that the exchange kernel is dispatched onto an idle GPU first."""
        ist = streams[1] if variant == "first-mask" else main_s
        delay = int(variant.split("-")[1]) if variant.startswith("delay-") else 0
        ev = torch.cuda.Event()
        ev.record(main_s)
        bnd_s.wait_event(ev)
        pair(1, 2, bnd_s)
        if variant == "cur":
            pair(NZ - 1, NZ, bnd_s)
        else:
            bnd2_s.wait_event(ev)
            pair(NZ - 1, NZ, bnd2_s)
            bnd_s.wait_stream(bnd2_s)
        if blocks:
            comm_s.wait_stream(bnd_s)
            assert kd.gs_debug_bw(4, 1, 1, blocks, O.data_ptr(), A.data_ptr(), None, m, sink.data_ptr(),
                                 comm_s.cuda_stream) == 0
        if ist is not main_s:
            ist.wait_event(ev)
        if variant in ("first", "first-mask"):
            ist.wait_stream(bnd_s)
        if delay:  # the interior waits for the boundary planes, then a sleeping wave on its own stream
            ist.wait_stream(bnd_s)
            assert kd.gs_debug_bw(5, 1, 1, 1, None, None, None, delay, None, ist.cuda_stream) == 0
        pair(3, NZ - 2, ist)
        if ist is not main_s:
            main_s.wait_stream(ist)
        main_s.wait_stream(comm_s if blocks else bnd_s)

    def pipe_steps2(blocks, nsteps):
        """pipe_steps with the two boundary launches on two high-priority streams (concurrent)."""
        evb = [None, None]
        ev_x = None
        for k_ in range(nsteps):
            ev_a = torch.cuda.Event()
            ev_a.record(main_s)
            for st_ in (bnd_s, bnd2_s):
                st_.wait_event(ev_a)
                if ev_x is not None:
                    st_.wait_event(ev_x)
            pair(1, 2, bnd_s)
            pair(NZ - 1, NZ, bnd2_s)
            bnd_s.wait_stream(bnd2_s)
            evb[k_ & 1] = torch.cuda.Event()
            evb[k_ & 1].record(bnd_s)
            comm_s.wait_event(evb[k_ & 1])
            if k_ > 0:
                main_s.wait_event(evb[(k_ - 1) & 1])
            pair(3, NZ - 2, main_s)
            if blocks:
                assert kd.gs_debug_bw(4, 1, 1, blocks, O.data_ptr(), A.data_ptr(), None, m, sink.data_ptr(),
                                      comm_s.cuda_stream) == 0
            ev_x = torch.cuda.Event()
            ev_x.record(comm_s)
        main_s.wait_event(ev_x)
        main_s.wait_event(evb[(nsteps - 1) & 1])

    def pipe_steps_b(blocks, nsteps, B, serial=False):
        """pipe_steps with B-plane boundary ranges (planes 1..B, NZ-B+1..NZ; interior B+1..NZ-B); serial: the
        boundary launches on the compute stream ahead of the interior (no concurrency between the two)."""
        evb = [None, None]
        ev_x = None
        bs = main_s if serial else bnd_s
        for k_ in range(nsteps):
            if not serial:
                ev_a = torch.cuda.Event()
                ev_a.record(main_s)
                bs.wait_event(ev_a)
            if ev_x is not None:
                bs.wait_event(ev_x)
            pair(1, B, bs)
            pair(NZ - B + 1, NZ, bs)
            evb[k_ & 1] = torch.cuda.Event()
            evb[k_ & 1].record(bs)
            comm_s.wait_event(evb[k_ & 1])
            if k_ > 0 and not serial:
                main_s.wait_event(evb[(k_ - 1) & 1])
            pair(B + 1, NZ - B, main_s)
            if blocks:
                assert kd.gs_debug_bw(4, 1, 1, blocks, O.data_ptr(), A.data_ptr(), None, m, sink.data_ptr(),
                                      comm_s.cuda_stream) == 0
            ev_x = torch.cuda.Event()
            ev_x.record(comm_s)
        main_s.wait_event(ev_x)
        main_s.wait_event(evb[(nsteps - 1) & 1])

    def pipe_steps(blocks, nsteps):
        """r03 driver (HipSolver::jacobi): a sequence of overlapped steps in which the compute stream never
        waits for an exchange. Boundary k waits for interior k-1 and exchange k-1; the interior k waits for
        boundary k-1 only; exchange k follows boundary k on the comm stream; the last exchange is joined."""
        evb = [None, None]
        ev_x = None
        for k_ in range(nsteps):
            ev_a = torch.cuda.Event()
            ev_a.record(main_s)
            bnd_s.wait_event(ev_a)
            if ev_x is not None:
                bnd_s.wait_event(ev_x)
            pair(1, 2, bnd_s)
            pair(NZ - 1, NZ, bnd_s)
            evb[k_ & 1] = torch.cuda.Event()
            evb[k_ & 1].record(bnd_s)
            comm_s.wait_event(evb[k_ & 1])
            if k_ > 0:
                main_s.wait_event(evb[(k_ - 1) & 1])
            pair(3, NZ - 2, main_s)
            if blocks:
                assert kd.gs_debug_bw(4, 1, 1, blocks, O.data_ptr(), A.data_ptr(), None, m, sink.data_ptr(),
                                     comm_s.cuda_stream) == 0
            ev_x = torch.cuda.Event()
            ev_x.record(comm_s)
        main_s.wait_event(ev_x)
        main_s.wait_event(evb[(nsteps - 1) & 1])

    def pipe_steps_defer(blocks, nsteps):
        """r04 driver order when exchange k-1 has not settled on the host yet (HipSolver::jacobi): interior k
        is enqueued BEFORE boundary k (it needs boundary k-1 only), then boundary k (after interior k-1 and
        exchange k-1), then exchange k. The GPU-side cost of that dispatch order."""
        evb = [None, None]
        ev_x = None
        for k_ in range(nsteps):
            ev_a = torch.cuda.Event()
            ev_a.record(main_s)
            if k_ > 0:
                main_s.wait_event(evb[(k_ - 1) & 1])
            pair(3, NZ - 2, main_s)
            bnd_s.wait_event(ev_a)
            if ev_x is not None:
                bnd_s.wait_event(ev_x)
            pair(1, 2, bnd_s)
            pair(NZ - 1, NZ, bnd_s)
            evb[k_ & 1] = torch.cuda.Event()
            evb[k_ & 1].record(bnd_s)
            comm_s.wait_event(evb[k_ & 1])
            if blocks:
                assert kd.gs_debug_bw(4, 1, 1, blocks, O.data_ptr(), A.data_ptr(), None, m, sink.data_ptr(),
                                      comm_s.cuda_stream) == 0
            ev_x = torch.cuda.Event()
            ev_x.record(comm_s)
        main_s.wait_event(ev_x)
        main_s.wait_event(evb[(nsteps - 1) & 1])

    def timed(fn, *args):
        for _ in range(2):
            fn(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        fn(*args)
        e1.record(main_s)
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps, 4)

    if os.environ.get("PROBE_WGS"):
        # r04: the driver's pipelined step against the stand-in exchange's workgroup count (the RCCL CTA
        # budget GS_RCCL_CTAS sets), in both dispatch orders; interleaved, PROBE_ROUNDS rounds
        wgs = [int(x) for x in os.environ["PROBE_WGS"].split(",")]
        res = {}
        for rnd in range(int(os.environ.get("PROBE_ROUNDS", "2"))):
            for b in wgs:
                for name, fn in (("pipelined", pipe_steps), ("pipelined-interior-first", pipe_steps_defer)):
                    key = f"{name} x{reps} exchange={'fat x%d' % b if b else 'none'}"
                    res.setdefault(key, []).append(timed(fn, b, reps))
        print(json.dumps({"slab": [NX, NY, NZ], "cus": cus, "step_ms": res,
                          "note": "pipelined overlapped pair steps of config #5's slab per stand-in exchange workgroup "
                                  "count (k_fatcopy at RCCL's kernel footprint, 34 MB); one value per round"}, indent=1))
        return

    res = {}
    # the boundary launches alone (B planes each side)
    for B in (2, 4):
        for _ in range(2):
            pair(1, B, main_s)
            pair(NZ - B + 1, NZ, main_s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        for _ in range(reps):
            pair(1, B, main_s)
            pair(NZ - B + 1, NZ, main_s)
        e1.record(main_s)
        torch.cuda.synchronize()
        res[f"boundary alone B={B}"] = round(e0.elapsed_time(e1) / reps, 4)
    for B, serial in ((2, True), (4, False), (4, True), (6, False)):
        for b in (0, 32):
            for _ in range(2):
                pipe_steps_b(b, reps, B, serial)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            pipe_steps_b(b, reps, B, serial)
            e1.record(main_s)
            torch.cuda.synchronize()
            res[f"pipelined B={B}{' serial' if serial else ''} exchange={'fat x%d' % b if b else 'none'}"] = \
                round(e0.elapsed_time(e1) / reps, 4)
    for b in (0, 32):
        for _ in range(2):
            pipe_steps2(b, reps)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        pipe_steps2(b, reps)
        e1.record(main_s)
        torch.cuda.synchronize()
        res[f"pipelined-2bnd x{reps} exchange={'fat x%d' % b if b else 'none'}"] = round(e0.elapsed_time(e1) / reps, 4)
    for b in (0, 8, 32):
        for _ in range(2):
            pipe_steps(b, reps)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        pipe_steps(b, reps)
        e1.record(main_s)
        torch.cuda.synchronize()
        res[f"pipelined x{reps} interior_zc={os.environ.get('GS_SLAB_ZC', '0')} exchange={'fat x%d' % b if b else 'none'}"] = round(e0.elapsed_time(e1) / reps, 4)
    settings = [(v_, b, "0") for v_ in ("cur", "first", "delay-1", "delay-3", "delay-6", "delay-12")
                for b in (0, 8, 32)]
    if os.environ.get("PROBE_ONLY_PIPE"):  # the r03 driver's schedule only (A/B of GS_SLAB_ZC per process)
        settings = []
    if os.environ.get("PROBE_MASK"):
        settings += [("first-mask", b, "0") for b in (0, 8, 32)]
    for _ in range(2):
        for v_, b, zc in settings:
            step2(v_, b)
    torch.cuda.synchronize()
    for v_, b, zc in settings:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        for _ in range(reps):
            step2(v_, b)
        e1.record(main_s)
        torch.cuda.synchronize()
        res[f"{v_} interior_zc={os.environ.get('GS_SLAB_ZC', '0')} exchange={'fat x%d' % b if b else 'none'}"] = round(e0.elapsed_time(e1) / reps, 4)
    # interior alone (unmasked / masked). The chunk length of the launches past a slab's first plane is
    # GS_SLAB_ZC, read once when the library loads: run the probe under different values for an A/B
    for r in streams:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st = streams[r]
        st.wait_stream(main_s)
        e0.record(st)
        for _ in range(reps):
            pair(3, NZ - 2, st)
        e1.record(st)
        torch.cuda.synchronize()
        res[f"interior alone, mask_free_per_xcd={r}"] = round(e0.elapsed_time(e1) / reps, 4)
    out = {"slab": [NX, NY, NZ], "cus": cus, "step_ms": res,
           "note": "one overlapped pair step: boundary pairs (planes 1-2, 127-128, high priority) -> stand-in "
                   "exchange (k_fatcopy, 34 MB copy at RCCL's kernel footprint) || interior pair planes 3..126"}
    print(json.dumps(out, indent=1))
    torch.cuda.synchronize()
    for r in [r for r in streams if r]:
        hip.hipStreamDestroy(C.c_void_p(streams[r].cuda_stream))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        main()
