#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on MI355X:
   "MLUPS (Jacobi smoother) + V-cycle wall-time, 512^3 fp64; achieved HBM GB/s %peak".

A step = one damped-Jacobi sweep (residual + update, 7-point stencil, fp64, LINEAR mode) over level 0
of the 512^3 grid of BASELINE config #3 (512^3 lattice updates). The K timed sweeps run exactly as
the solver runs its 2+2 smoothing: in fused pairs (gs_jacobi_sweep2, temporal blocking: one read of
v and f and one write per pair), an odd last sweep alone. value = lattice updates of all ranks /
max-over-ranks wall time (MLUPS). Inputs are resident in HBM before the timed region. The one-sweep
kernel is also timed on its own ("single_sweep_kernel"), and the V-cycle wall time (512^3, 2+2,
including the 8-byte norm readback) is measured after the timed region ("vcycle").

Multi-GPU (torchrun, one process per GPU): the grid is Z-slab partitioned over RCCL (xGMI), ghost
planes exchanged every sweep on a second stream while the interior planes are swept; weak scaling
with 512^3 lattice points per rank: N=2 -> 512x512x1024, N=4 -> 512x1024x1024 (every rank's slab has
the single-GPU run's 512-point rows, so the per-rank kernels are the N=1 ones), N=8 -> 1024^3
(BASELINE config #5: 1024-point rows, the column-block pair); other N -> 512x512x(512N). Every
rank runs the same number of sweeps (the untimed ramp's length is agreed across ranks), since each
sweep's ghost exchange pairs with the neighbours'.

Roofline: the smoother is HBM-bound (0.5 flop/B per sweep); algorithmic bytes per launch = 24 B
per lattice point (read v, read f, write the result) x 512^3, for a single sweep
and for a fused pair alike / the average launch duration measured with HIP events on the solver's
stream; peak = 8000 GB/s (MI355X HBM3E, MI355X_MICROARCH.md).
cpu_baseline: the reference's own CpuSolver::jacobi (oracle/_ref/ref_probe, compiled from
/root/reference/src/cpu) on this host's cores, a bounded sample of the same workload.
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gpu-solve_amd"))

import gpusolve as gsv  # noqa: E402

PEAK_GBPS = 8000.0
BYTES_PER_LUP = 24.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=200, help="untimed sweeps first (also brings the GPU clocks up)")
    ap.add_argument("--ramp-ms", type=float, default=400.0,
                    help="after --warmup, keep running untimed sweeps until this much wall time has passed")
    ap.add_argument("--size", type=int, default=512, help="per-rank cube edge (BASELINE config #3: 512)")
    ap.add_argument("--vcycles", type=int, default=20, help="timed V-cycles after one warm-up cycle (0: skip)")
    ap.add_argument("--cpu-sweeps", type=int, default=10, help="cpu_baseline sample size (0: skip)")
    ap.add_argument("--cpu-vcycles", type=int, default=2, help="cpu_baseline V-cycles after one warm-up cycle (0: skip)")
    ap.add_argument("--config5", type=int, default=1,
                    help="N=1: also time config #5's 1024^3 grid on this GPU (the strong-scaling denominator)")
    ap.add_argument("--config2", type=int, default=1,
                    help="N=1: also time BASELINE config #2 (128^3 linear 2+2, 10 V-cycles)")
    ap.add_argument("--newton-iters", type=int, default=2,
                    help="timed Newton iterations of BASELINE config #4 (512^3 Newton 2+2) at N=1 (0: skip)")
    ap.add_argument("--cta-ab", default="16,64",
                    help="N > 1: after the headline, time the same sweeps on fresh RCCL communicators with these "
                         "CTA budgets (ncclConfig_t::minCTAs = maxCTAs), interleaved twice ('' skips)")
    return ap.parse_args()


def pmc_traffic(n):
    """HBM bytes per launch of the smoother from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(REPO, "profiles", "pmc_smoother.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if int(d.get("n", -1)) == n:
            return float(d["hbm_bytes_per_launch"]), d
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def _cpu_run(exe, args, threads, timeout):
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = str(threads)
    env.setdefault("OMP_PROC_BIND", "close")
    r = subprocess.run([exe, *args], capture_output=True, text=True, env=env, timeout=timeout)
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(n, sweeps, vcycles):
    """CPU baseline on this host's cores, a bounded sample of the same workload.

    kind "reference": oracle/_ref/ref_probe, the reference's own src/cpu (CpuSolver::jacobi / vcycle)
    compiled from /root/reference by oracle/Makefile in the build container and shipped to the GPU box
    as a built binary (no reference source travels). Without it, kind "port": the oracle restatement
    (oracle/build/gso_cli). Legs: all host threads (OMP_NUM_THREADS = the box's CPU share), one thread,
    and the port timed on the same sample (calibration: port / reference speed ratio)."""
    ref = os.path.join(REPO, "oracle", "_ref", "ref_probe")
    port = os.path.join(REPO, "oracle", "build", "gso_cli")
    exe, kind = (ref, "reference") if os.path.exists(ref) else (port, "port")
    if not os.path.exists(exe):
        return None
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    out = {"unit": "MLUPS", "cores": threads, "kind": kind,
           "binary": os.path.relpath(exe, REPO) + (" (reference src/cpu compiled by oracle/Makefile)"
                                                    if kind == "reference" else " (oracle restatement)")}
    j = _cpu_run(exe, ["time_jacobi", str(n), str(n), str(n), "0", str(sweeps)], threads, 600)
    out["value"] = round(float(j["mlups"]), 3)
    out["sample"] = (f"{sweeps} level-0 Jacobi sweeps (CpuSolver::jacobi, residual+update) of the {n}^3 linear "
                     f"grid after 1 warm-up sweep, {threads} OpenMP threads")
    if vcycles > 0:
        j = _cpu_run(exe, ["time_vcycle", str(n), str(n), str(n), "0", str(vcycles)], threads, 900)
        out["vcycle_ms"] = round(float(j["ms_per_cycle"]), 1)
        out["sample"] += f"; {vcycles} 2+2 V-cycle(s) after 1 warm-up cycle"
    # one-thread leg (OMP_NUM_THREADS=1), 1 timed sweep of the same grid
    try:
        j = _cpu_run(exe, ["time_jacobi", str(n), str(n), str(n), "0", "1"], 1, 600)
        out["one_thread"] = {"value": round(float(j["mlups"]), 3), "cores": 1,
                             "sample": f"1 level-0 Jacobi sweep of the {n}^3 linear grid after 1 warm-up sweep"}
    except Exception as e:  # reported, never required
        out["one_thread"] = {"error": str(e)}
    if kind == "reference" and os.path.exists(port):
        try:
            j = _cpu_run(port, ["time_jacobi", str(n), str(n), str(n), "0", str(sweeps)], threads, 600)
            out["port_calibration"] = {"port_value": round(float(j["mlups"]), 3),
                                       "port_over_reference": round(float(j["mlups"]) / out["value"], 3),
                                       "sample": f"same {sweeps} sweeps, {threads} threads, oracle/build/gso_cli"}
        except Exception as e:
            out["port_calibration"] = {"error": str(e)}
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
        out["cpu_model"] = model
    except (OSError, IndexError):
        pass
    return out


def global_dims(n, world):
    table = {1: (n, n, n), 2: (n, n, 2 * n), 4: (n, 2 * n, 2 * n), 8: (2 * n, 2 * n, 2 * n)}
    return table.get(world, (n, n, n * world))


def make_grid(params, rank, world, ctas=-1):
    """Single-GPU grid, or this rank's Z-slab of an RCCL-partitioned grid (its own communicator, CTA budget
    `ctas`; -1: the library's default)."""
    import ctypes as C
    if world == 1:
        return gsv.HipGridData(params)
    drv = gsv.driver()
    uid = (C.c_ubyte * 128)()
    if rank == 0 and drv.gs_rccl_unique_id(uid) != 0:
        raise gsv.GpuSolveError(drv.gs_last_error().decode())
    t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device="cuda")
    dist.broadcast(t, 0)
    uid = (C.c_ubyte * 128)(*t.cpu().tolist())
    grid = gsv.HipGridData.__new__(gsv.HipGridData)
    grid.params = params
    grid._abi_params = params.to_abi()
    grid.handle = drv.gs_grid_create_rccl_ctas(C.byref(grid._abi_params), rank, world, uid, ctas)
    if not grid.handle:
        raise gsv.GpuSolveError(drv.gs_last_error().decode())
    return grid


def single_sweep_timing(grid, dims, k):
    """The one-sweep kernel alone (gs_jacobi_sweep on the grid's level-0 fields), for reference."""
    import ctypes as C
    from gpusolve.devfield import DevField
    kl, drv = gsv.kernels(), gsv.driver()
    L = grid.getLevel(0).geom
    S = grid.params.stencil.to_abi()
    v = drv.gs_grid_field(grid.handle, 0, 0)
    f = drv.gs_grid_field(grid.handle, 0, 3)
    tmp = DevField(L.nx, L.ny, L.nz)
    st = grid.stream()
    stream = torch.cuda.ExternalStream(st)
    a_, b_ = v, tmp.ptr
    for _ in range(2):
        kl.gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, a_, b_, f, None, st)
        a_, b_ = b_, a_
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        kl.gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, a_, b_, f, None, st)
        a_, b_ = b_, a_
    e1.record(stream)
    torch.cuda.synchronize()
    if k % 2:  # leave the iterate in the grid's own buffer
        kl.gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, a_, b_, f, None, st)
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / k
    pts = float(L.nx) * L.ny * L.nz
    gbps = BYTES_PER_LUP * pts / (ms * 1e-3) / 1e9
    return {"kernel": "k_rb (one sweep per launch)", "ms": round(ms, 4), "mlups": round(pts / ms / 1e3, 1),
            "achieved_GBps": round(gbps, 1), "frac": round(gbps / PEAK_GBPS, 4)}


def vcycle_level0_kernels(grid, k):
    """The V-cycle's two other level-0 passes timed alone with HIP events on the grid's own fields
    (after the V-cycles: level 1's f is scratch, the prolongation pair writes a spare buffer): the
    fused residual + restriction (16 B/point read + 1 B coarse write) and the prolongation pair (24 B
    + 1 B coarse read). Algorithmic bytes per point / average launch time, as `roofline`."""
    import ctypes as C
    from gpusolve.devfield import DevField
    kl, drv = gsv.kernels(), gsv.driver()
    L0, L1 = grid.getLevel(0).geom, grid.getLevel(1).geom
    S = grid.params.stencil.to_abi()
    p = grid.params
    v, f = drv.gs_grid_field(grid.handle, 0, 0), drv.gs_grid_field(grid.handle, 0, 3)
    cv, cf = drv.gs_grid_field(grid.handle, 1, 0), drv.gs_grid_field(grid.handle, 1, 3)
    out = DevField(L0.nx, L0.ny, L0.nz)
    st = grid.stream()
    stream = torch.cuda.ExternalStream(st)
    pts = float(L0.nx) * L0.ny * L0.nz

    def rr():
        assert kl.gs_residual_restrict(C.byref(S), C.byref(L0), 0, p.gamma, v, f, None, cf, None, C.byref(L1), st) == 0

    wsn = kl.gs_jacobi_sweep2_prolong_ws_elems(C.byref(S), C.byref(L0), 0)  # rows > 512: edge-column strip
    ws = torch.empty(max(1, wsn), dtype=torch.float64, device="cuda")

    def pro():
        assert kl.gs_jacobi_sweep2_prolong_ws(C.byref(S), C.byref(L0), 0, p.omega, p.gamma, v, cv, None, C.byref(L1),
                                              out.ptr, f, None, 0, 0, ws.data_ptr(), wsn, st) == 0

    res = {}
    for name, fn, bpp in (("residual_restrict", rr, 17.0), ("prolong_pair", pro, 25.0)):
        try:
            fn()
        except AssertionError:
            res[name] = {"error": "no fused kernel for this level shape"}
            continue
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / k
        gbps = bpp * pts / (ms * 1e-3) / 1e9
        res[name] = {"ms": round(ms, 4), "bytes_per_point": bpp, "achieved_GBps": round(gbps, 1),
                     "frac": round(gbps / PEAK_GBPS, 4)}
    res["kernels"] = "k_rr2 (residual + full weighting), k_tb2y PRO (prolongation + correction + 2 sweeps)"
    del out
    return res


def slab_local_pair_ms(grid, rank, world, k):
    """N > 1: the level-0 pair on this rank's slab with no exchange (gs_jacobi_sweep2 on the grid's own
    v and f into a spare field, the slab's internal sides flagged as ghost planes), averaged over k
    launches: set beside kernel_ms (the overlapped sweep with its RCCL exchange) it shows what the
    exchange costs per pair on this rank."""
    import ctypes as C
    from gpusolve.devfield import DevField
    kl, drv = gsv.kernels(), gsv.driver()
    L = grid.getLevel(0).geom
    S = grid.params.stencil.to_abi()
    v, f = drv.gs_grid_field(grid.handle, 0, 0), drv.gs_grid_field(grid.handle, 0, 3)
    out = DevField(L.nx, L.ny, L.nz)
    st = grid.stream()
    stream = torch.cuda.ExternalStream(st)
    zlo, zhi = int(rank > 0), int(rank + 1 < world)

    def run():
        assert kl.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v, out.ptr, f, None, zlo, zhi, st) == 0

    for _ in range(2):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    del out
    return e0.elapsed_time(e1) / k


# gs_debug_bw kind, bytes per element
CEILING_KINDS = {"read": (0, 8.0), "copy": (2, 16.0), "triad": (3, 24.0), "write": (1, 8.0)}
# (blocks, unroll) shapes: grid-stride loops over 1024 / 2048 / 4096 blocks with 1 or 4 dwordx4 in flight per lane,
# and (r06) blocks = 0: the guide's float4-copy shape, a grid covering the array once (no loop), 1 / 2 / 4 dwordx4
# per thread
CEILING_SHAPES = [(b, u) for b in (1024, 2048, 4096) for u in (1, 4)] + [(0, u) for u in (1, 2, 4)]


def stream_ceilings(n):
    """This GPU's streaming ceilings on arrays of the level's size, measured in this run beside the kernels
    they bound: the triad (2 streamed reads + 1 streamed write, 24 B per element: the smoother's byte mix),
    a copy (1 read + 1 write), a read-only and a store-only stream, each 16 B per lane (dwordx4), the best
    over CEILING_SHAPES x default / non-temporal policy (gs_debug_bw); per kind also the best of each shape
    family (grid-stride / flat). Boxes differ by up to ~25 %, so the kernel's fraction of these is reported next
    to the fraction of the 8 TB/s datasheet peak."""
    kl = gsv.diag()  # the streaming probes live in the diagnostics library
    A = torch.rand(n, dtype=torch.float64, device="cuda")
    B = torch.rand(n, dtype=torch.float64, device="cuda")
    O = torch.empty(n, dtype=torch.float64, device="cuda")
    sink = torch.zeros(1, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}
    def shape_name(blocks, unroll, nt):
        s = (f"{blocks} blocks, grid-stride, {unroll} dwordx4 in flight per lane" if blocks > 0 else
             f"flat grid covering the array, {unroll} dwordx4 per thread, no loop")
        return s + (", nt" if nt else ", default policy")

    for name, (kind, bpe) in CEILING_KINDS.items():
        best, fam = None, {}
        for blocks, unroll in CEILING_SHAPES:
            for nt in (1, 0):
                def run():
                    rc = kl.gs_debug_bw(kind, unroll, nt, blocks, O.data_ptr(), A.data_ptr(), B.data_ptr(), n,
                                        sink.data_ptr(), st.cuda_stream)
                    assert rc == 0, rc
                for _ in range(2):
                    run()
                e0.record(st)
                for _ in range(8):
                    run()
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 8
                if best is None or ms < best[0]:
                    best = (ms, blocks, unroll, nt)
                f = "flat" if blocks <= 0 else "grid_stride"
                if f not in fam or ms < fam[f][0]:
                    fam[f] = (ms, blocks, unroll, nt)
        ms, blocks, unroll, nt = best
        out[name] = {"kernel": f"streaming {name}, {int(bpe)} B per element, 16 B per lane, " +
                               shape_name(blocks, unroll, nt),
                     "elements": n, "ms": round(ms, 4), "gbps": round(bpe * n / (ms * 1e-3) / 1e9, 1),
                     "by_shape": {f: {"gbps": round(bpe * n / (v[0] * 1e-3) / 1e9, 1), "shape": shape_name(*v[1:])}
                                  for f, v in fam.items()}}
    del A, B, O
    return out


def newton_timing(n, iters):
    """BASELINE config #4: the n^3 Newton solve (mode 2, 2+2, omega 0.8, gamma 1, tol 0), `iters` outer
    iterations through the driver (NewtonSolver::solve: per iteration restrict newtonV, an inner solve
    of 10 V-cycles, newtonV += v, compF + norm), on its own grid after one untimed iteration."""
    p = gsv.GridParams(maxiter=1, tol=0.0, gridDim=(n, n, n), mode=gsv.GS_NEWTON, preSmoothing=2, postSmoothing=2)

    def timed(maxiter):
        p.maxiter = maxiter
        with gsv.HipGridData(p) as g:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hist = gsv.NewtonSolver.solve(g)
            return (time.perf_counter() - t0) * 1e3, hist

    timed(1)  # warm-up: first touch of every level
    # the first iteration starts from newtonV = 0 (every linearisation factor is gamma: GS_NEWTON_G inner solve,
    # DESIGN.md §4.6), so it is cheaper than the later ones: a one-iteration solve times it alone
    ms1, _ = timed(1)
    ms, hist = timed(iters)
    out = {"ms_per_iteration": round(ms / iters, 2), "iterations": iters,
           "config": f"{n}^3 Newton 2+2 (BASELINE config #4), 10 inner V-cycles per iteration, norm readbacks included",
           "ms_first_iteration": round(ms1, 2), "residuals": hist}
    if iters > 1:
        out["ms_per_later_iteration"] = round((ms - ms1) / (iters - 1), 2)
    return out


KERNEL_OPS = {"pair", "sweep", "pro", "residual", "resrestrict", "restrict", "prolongadd", "applyadd", "coarse",
              "tiledpre", "tiledpro", "norm", "copy", "newtonF", "axpy", "bfac", "newtonFupdate"}


def launches_per_cycle(p):
    """Kernel launches one more V-cycle adds to the solve's schedule, counted on the driver's own schedule trace
    (gs_zslab_schedule, one rank: no device touched): solves of maxiter 2 and 3 differ by one steady-state cycle."""
    import ctypes as C
    d = gsv.driver()

    def count(maxiter):
        q = gsv.GridParams(maxiter=maxiter, tol=0.0, gridDim=p.gridDim, mode=p.mode, preSmoothing=p.preSmoothing,
                           postSmoothing=p.postSmoothing).to_abi()
        n = C.c_int64()
        assert d.gs_zslab_schedule(C.byref(q), 1, 0, 0, None, 0, C.byref(n)) == 0
        buf = C.create_string_buffer(n.value + 1)
        assert d.gs_zslab_schedule(C.byref(q), 1, 0, 0, buf, n.value + 1, C.byref(n)) == 0
        ops = [l.split()[0] for l in buf.value.decode().splitlines() if l.strip()]
        return sum(op in KERNEL_OPS for op in ops), ops

    a, _ = count(2)
    b, ops = count(3)
    return b - a


def config2_timing(n=128, cycles=10):
    """BASELINE config #2: 128^3 linear 7-point, 2+2 smoothing, 10 V-cycles, fp64 (CpuSolver::solve,
    src/cpu/CpuSolver.cpp:12-43 with vcycle :85-139). The whole 10-cycle solve as the reference runs it (initial
    residual, ten V-cycles, every norm read back; host wall clock), after one untimed solve on the same grid; the
    steady-state cycle (gs_grid_time_vcycles); the launches one cycle takes (the driver's schedule trace); and the
    device ms per level of one cycle (a second grid with the per-level HIP-event clock, GS_METRICS: that clock turns
    the norm-wait overlap off, so its cycle is the unpipelined one)."""
    import ctypes as C
    drv = gsv.driver()
    p = gsv.GridParams(maxiter=cycles, tol=0.0, gridDim=(n, n, n), mode=gsv.GS_LINEAR, preSmoothing=2,
                       postSmoothing=2)
    out = {"config": f"{n}^3 linear 7-point, 2+2, {cycles} V-cycles, fp64 (BASELINE config #2)"}
    with gsv.HipGridData(p) as g:
        gsv.HipSolver.solve(g)  # warm-up: first touch of every level
        walls = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hist = gsv.HipSolver.solve(g)
            walls.append((time.perf_counter() - t0) * 1e3)
        out["solve_ms"] = round(min(walls), 3)
        out["solve_ms_runs"] = [round(w, 3) for w in walls]
        out["ms_per_cycle"] = round(min(walls) / cycles, 4)
        out["residuals_last_run"] = [hist[0], hist[-1]]
        ms, last = C.c_double(), C.c_double()
        if drv.gs_grid_time_vcycles(g.handle, 50, C.byref(ms), C.byref(last)):
            raise gsv.GpuSolveError(drv.gs_last_error().decode())
        out["steady_cycle_ms"] = round(ms.value / 50, 4)
    try:
        out["launches_per_cycle"] = launches_per_cycle(p)
    except Exception as e:  # noqa: BLE001 (reported, never required)
        out["launches_per_cycle"] = {"error": str(e)}
    out.update(level_split(p))
    return out


def level_split(p):
    """Device ms per V-cycle by level: a grid of the same params created with the per-level HIP-event clock
    (GS_METRICS=1, read at grid creation), one solve of p.maxiter cycles. That clock records events around each
    level's down- and up-leg work and turns the norm-wait overlap off, so its cycle is the unpipelined one."""
    import ctypes as C
    drv = gsv.driver()
    old = os.environ.get("GS_METRICS")
    os.environ["GS_METRICS"] = "1"
    try:
        with gsv.HipGridData(p) as g:
            gsv.HipSolver.solve(g)
            nl = g.numLevels()
            lv = (C.c_double * nl)()
            line = C.create_string_buffer(4096)
            if drv.gs_grid_metrics(g.handle, line, 4096, lv, nl):
                raise gsv.GpuSolveError(drv.gs_last_error().decode())
            ms = [float(x) for x in lv]
            return {"level_ms_per_cycle": [round(x, 4) for x in ms],
                    "levels_ge1_ms_per_cycle": round(sum(ms[1:]), 4),
                    "level_ms_note": ("device ms per V-cycle by level (HIP events around each level's down- and up-leg "
                                      "work, unpipelined cycle, GS_METRICS grid; levels of the one-launch coarse end "
                                      "are booked to the level it starts from)")}
    except Exception as e:  # noqa: BLE001 (reported, never required)
        return {"level_ms_per_cycle": {"error": f"{type(e).__name__}: {e}"}}
    finally:
        if old is None:
            os.environ.pop("GS_METRICS", None)
        else:
            os.environ["GS_METRICS"] = old


CONFIG5_FILE = os.path.join(REPO, "profiles", "config5_single_gpu.json")


def config5_single_gpu(steps, vcycles, n=1024):
    """BASELINE config #5's grid (1024^3 linear 2+2) on this ONE GPU, after the headline and outside its
    timed region: the same-grid denominator of the strong-scaling ratio north_star names (8 GPUs vs 1 on
    1024^3). The level-0 smoother as the solver runs it (fused pairs, 1024-point rows: column blocks),
    timed like the headline (untimed ramp, then `steps` sweeps bracketed by HIP events on the grid's
    stream), and the 2+2 V-cycle wall time (norm readback included)."""
    import ctypes as C
    drv = gsv.driver()
    p = gsv.GridParams(maxiter=1, tol=0.0, gridDim=(n, n, n), mode=gsv.GS_LINEAR, preSmoothing=2, postSmoothing=2)
    with gsv.HipGridData(p) as g:
        stream = torch.cuda.ExternalStream(g.stream())

        def sweeps(k):
            if drv.gs_grid_jacobi(g.handle, 0, k):
                raise gsv.GpuSolveError(drv.gs_last_error().decode())

        tw = time.perf_counter()
        while (time.perf_counter() - tw) < 0.3:
            sweeps(20)
            g.sync()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        sweeps(steps)
        ev1.record(stream)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        fused = drv.gs_grid_level_fused(g.handle, 0) == 1
        passes = (steps // 2 + steps % 2) if fused else steps
        kernel_ms = ev0.elapsed_time(ev1) / passes
        pts = float(n) ** 3
        kname = gsv.kernels().gs_jacobi_sweep2_kernel(C.byref(p.stencil.to_abi()), C.byref(g.getLevel(0).geom),
                                                      0).decode()
        out = {"grid": [n, n, n], "steps": steps, "mlups": round(pts * steps / elapsed / 1e6, 1),
               "ms_per_step": round(elapsed / steps * 1e3, 4), "pair_kernel_ms": round(kernel_ms, 4),
               "pair_kernel": kname.split(":")[0],
               "pair_frac": round(BYTES_PER_LUP * pts / (kernel_ms * 1e-3) / 1e9 / PEAK_GBPS, 4)}
        if vcycles > 0:
            gsv.HipSolver.vcycle(g)  # warm-up
            ms, last = C.c_double(), C.c_double()
            if drv.gs_grid_time_vcycles(g.handle, vcycles, C.byref(ms), C.byref(last)):
                raise gsv.GpuSolveError(drv.gs_last_error().decode())
            out["vcycle_ms"] = round(ms.value / vcycles, 3)
            out["vcycles"] = vcycles
    out["note"] = ("1024^3 linear 2+2 on one GPU (BASELINE config #5's grid): the N=8 line's strong-scaling "
                   "denominator (speedup_vs_1gpu_same_grid: rank 0 measures it again in that job; the driver's copy "
                   "of this object, profiles/config5_single_gpu.json, is its secondary denominator)")
    return out


RCCL_LINK = None


def rccl_debug_setup():
    """N > 1, before any communicator exists: RCCL's INFO log (connection set-up lines only: subsystems INIT,
    P2P, NET) goes to a per-process file, so that the line can report the transport every peer connection
    actually took (P2P/IPC over xGMI, P2P/direct pointer, SHM, NET/Socket ...). An explicit NCCL_DEBUG /
    NCCL_DEBUG_FILE in the environment wins. Returns this process's log path or None."""
    if os.environ.get("NCCL_DEBUG_FILE"):  # the launcher's own log file: parsed if it logs at INFO
        if os.environ.get("NCCL_DEBUG", "").upper() not in ("INFO", "TRACE"):
            return None
    else:  # (a preset NCCL_DEBUG level without a file would print to stdout / stderr: the file takes over)
        os.environ["NCCL_DEBUG"] = "INFO"
        os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,P2P,NET"
        os.environ["NCCL_DEBUG_FILE"] = os.path.join(
            "/tmp", f"gs-rccl-{os.environ.get('MASTER_PORT', '0')}-{os.environ.get('RANK', '0')}-%h-%p.log")
    return os.environ["NCCL_DEBUG_FILE"].replace("%h", os.uname().nodename).replace("%p", str(os.getpid()))


def rccl_transports(path):
    """The peer connections in one process's RCCL INFO log: {communicator: {"nranks": n, "peers":
    {peer: [transport, ...]}}}, e.g. {"0x5f..": {"nranks": 8, "peers": {"1": ["P2P/IPC/read"]}}}."""
    import re
    pat = re.compile(r"Channel \d+(?:/\d+)? : (\d+)\[[0-9a-fx]+\] -> (\d+)\[[0-9a-fx]+\] "
                     r"(?:\[(send|receive)\] )?via (.+?) comm (\S+) nRanks (\d+)")
    out = {}
    try:
        with open(path, errors="replace") as f:
            for line in f:
                m = pat.search(line)
                if not m:
                    continue
                src, dst, _, via, comm, nr = m.groups()
                c = out.setdefault(comm, {"nranks": int(nr), "peers": {}})
                me = int(os.environ.get("RANK", "0"))
                peer = dst if int(src) == me else src
                t = c["peers"].setdefault(peer, [])
                via = via.strip()
                if via not in t:
                    t.append(via)
    except OSError as e:
        return {"error": str(e)}
    return out


def ramp_sweeps(run, ramp_ms, any_rank, chunk=40):
    """Untimed ramp: `run(chunk)` (launch + wait) until `ramp_ms` of wall time has passed on EVERY rank.
    `any_rank(flag)` is the OR of flag over all ranks, so all ranks run the same number of chunks — a
    rank that ran one chunk more than its neighbour would post a ghost exchange nobody answers.
    Returns (sweeps run, wall ms)."""
    tw = time.perf_counter()
    done = 0
    while any_rank((time.perf_counter() - tw) * 1e3 < ramp_ms):
        run(chunk)
        done += chunk
    return done, (time.perf_counter() - tw) * 1e3


def main():
    a = parse()
    # stdout carries exactly the one JSON line: anything the libraries print there (RCCL writes a version
    # banner at communicator creation) goes to stderr instead
    sys.stdout.flush()
    json_out = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    rccl_log = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # RCCL's p2p channels per peer fill the halo communicator's CTA budget (gs_rccl_channels_per_peer_hint:
        # GS_RCCL_CTAS, default 64, over the four send/recv of a rank's grouped exchange). RCCL reads the variable
        # once per process, so the launcher sets it before torch's communicator; an explicit value wins.
        cpp = gsv.driver().gs_rccl_channels_per_peer_hint(-1)
        if cpp > 0:
            os.environ.setdefault("NCCL_NCHANNELS_PER_PEER", str(cpp))
        rccl_log = rccl_debug_setup()
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local % max(1, torch.cuda.device_count())))

    def barrier():
        if world > 1:
            dist.barrier()

    n = a.size
    dims = global_dims(n, world)
    # N=8 on config #5's grid: rank 0 first times the same 1024^3 grid on its own GPU, in this job and on
    # this node, before any rank builds its slab (the other ranks wait): the same-job denominator of
    # speedup_vs_1gpu_same_grid, beside the committed driver record's
    c5_same_job = None
    if world > 1 and tuple(dims) == (1024, 1024, 1024) and a.config5:
        if rank == 0:
            try:
                c5_same_job = config5_single_gpu(a.steps, 0)
            except Exception as e:  # noqa: BLE001 (reported, never required)
                c5_same_job = {"error": f"{type(e).__name__}: {e}"}
            torch.cuda.synchronize()
        barrier()
    params = gsv.GridParams(maxiter=1, tol=0.0, gridDim=dims, mode=gsv.GS_LINEAR, preSmoothing=2,
                            postSmoothing=2)
    grid = make_grid(params, rank, world)
    drv = gsv.driver()
    fused = drv.gs_grid_level_fused(grid.handle, 0) == 1
    # untimed ramp: the requested warm-up sweeps, then more until at least --ramp-ms of smoother launches
    # have run (cold launches run ~25 % slower: BENCH_r01 timed them inside a 7.8 ms window)
    def any_rank(flag):
        if world == 1:
            return flag
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item() > 0

    def timed_window(g, warmup, ramp_ms, steps):
        """Untimed warm-up + agreed ramp, then exactly `steps` sweeps bracketed by a barrier and a device
        synchronisation on both sides, HIP events on the grid's own stream. Returns (max-over-ranks wall s,
        this rank's wall s, this rank's average pass ms, ramp sweeps, warm-up ms)."""
        gstream = torch.cuda.ExternalStream(g.stream())

        def gsweeps(k):
            if drv.gs_grid_jacobi(g.handle, 0, k):
                raise gsv.GpuSolveError(drv.gs_last_error().decode())

        def grun(k):
            gsweeps(k)
            g.sync()

        tw = time.perf_counter()
        grun(warmup)
        rmp, _ = ramp_sweeps(grun, max(0.0, ramp_ms - (time.perf_counter() - tw) * 1e3), any_rank)
        wms = (time.perf_counter() - tw) * 1e3
        barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(gstream)
        gsweeps(steps)
        ev1.record(gstream)
        torch.cuda.synchronize()
        barrier()
        own = time.perf_counter() - t0
        # passes over the level: a fused pair reads v and f once and writes once, like a single sweep
        npass = (steps // 2 + steps % 2) if drv.gs_grid_level_fused(g.handle, 0) == 1 else steps
        kms = ev0.elapsed_time(ev1) / npass  # average pass duration on the solver's stream
        t = torch.tensor([own], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item(), own, kms, rmp, wms

    elapsed, own_elapsed, kernel_ms, ramp, warmup_ms = timed_window(grid, a.warmup, a.ramp_ms, a.steps)
    passes = (a.steps // 2 + a.steps % 2) if fused else a.steps

    multi = None
    if world > 1:  # per-rank view of the timed window, and the pair's cost without its exchange
        try:
            local = slab_local_pair_ms(grid, rank, world, max(4, passes))
        except Exception:  # noqa: BLE001 (diagnostic only)
            local = float("nan")
        import ctypes as C
        hms, hcalls, hmax = C.c_double(), C.c_int64(), C.c_double()
        drv.gs_grid_comm_stats(grid.handle, C.byref(hms), C.byref(hcalls))
        drv.gs_grid_comm_stats_max(grid.handle, C.byref(hmax))
        halo_us = hms.value / max(1, hcalls.value) * 1e3
        per = torch.tensor([own_elapsed / a.steps * 1e3, kernel_ms, local, halo_us, hmax.value * 1e3],
                           dtype=torch.float64, device="cuda")
        allp = [torch.zeros_like(per) for _ in range(world)]
        dist.all_gather(allp, per)
        rows = [x.tolist() for x in allp]
        fin = lambda x: round(x, 4) if math.isfinite(x) else None  # noqa: E731 (JSON has no NaN)
        gaps = [r[1] - r[2] for r in rows if math.isfinite(r[2])]
        slab_bytes = BYTES_PER_LUP * float(dims[0]) * dims[1] * dims[2] / world
        multi = {"rank_ms_per_step": [fin(r[0]) for r in rows],
                 "rank_pair_ms": [fin(r[1]) for r in rows],
                 # per GPU: 24 B x the rank's slab points / its overlapped pair's average launch time, over 8 TB/s
                 "rank_pair_frac_of_peak": [fin(slab_bytes / (r[1] * 1e-3) / 1e9 / PEAK_GBPS) if r[1] > 0 else None
                                            for r in rows],
                 "rank_pair_frac_of_peak_no_exchange": [
                     fin(slab_bytes / (r[2] * 1e-3) / 1e9 / PEAK_GBPS) if math.isfinite(r[2]) and r[2] > 0 else None
                     for r in rows],
                 "rank_pair_ms_no_exchange": [fin(r[2]) for r in rows],
                 "exchange_ms_per_pair_max": fin(max(gaps)) if gaps else None,
                 "rank_halo_host_us_per_call": [fin(r[3]) for r in rows],
                 "rank_halo_host_us_max": [fin(r[4]) for r in rows],
                 "rccl_ctas": drv.gs_grid_comm_ctas(grid.handle),
                 "rccl_channels_per_peer": os.environ.get("NCCL_NCHANNELS_PER_PEER"),
                 "note": "rank_pair_ms: the overlapped pair (boundary planes, RCCL ghost exchange, interior) "
                         "per launch on each rank's compute stream; _no_exchange: the same pair on the same "
                         "slab run locally, no exchange; rank_halo_host_us_per_call / _max: host wall time of "
                         "one ghost exchange (RCCL group issue, polls and settle), mean and maximum over every "
                         "exchange so far; in a sequence of sweeps an exchange is settled only before the next "
                         "boundary planes, after the next interior is already enqueued when it is still in "
                         "flight"}

    single = ceilings = ceiling = None
    if world == 1:
        single = single_sweep_timing(grid, dims, a.steps)
        ceilings = stream_ceilings((int(dims[0]) * dims[1] * dims[2]) & ~1)  # (the probe streams element pairs)
        ceiling = ceilings["triad"]

    lups_per_rank = float(dims[0]) * dims[1] * dims[2] / world
    total_lups = lups_per_rank * a.steps * world
    value = total_lups / elapsed / 1e6
    achieved = BYTES_PER_LUP * lups_per_rank / (kernel_ms * 1e-3) / 1e9
    # the committed PMC summary is of the N=1 grid's pair (512^3, k_tb2y); a rank's slab at N > 1 is another
    # launch shape (config #5: 1024x1024x128, column blocks; its counters: profiles/r02h_pmc_level0.md)
    traffic, pmc = pmc_traffic(n) if world == 1 else (None, None)
    import ctypes as C
    pair_kernel = gsv.kernels().gs_jacobi_sweep2_kernel(C.byref(grid.params.stencil.to_abi()),
                                                        C.byref(grid.getLevel(0).geom), 0).decode()

    vc = None
    if a.vcycles > 0:
        # after the headline: a failure here (e.g. the RCCL communicator timing out and aborting, which
        # raises instead of hanging) is reported in the line rather than losing it; the ranks agree on
        # the outcome before the cross-rank maximum
        err = None
        try:
            res = gsv.HipSolver.vcycle(grid)  # warm-up (first touch of every level)
            barrier()
            import ctypes as C
            ms, last = C.c_double(), C.c_double()
            rc = drv.gs_grid_time_vcycles(grid.handle, a.vcycles, C.byref(ms), C.byref(last))
            if rc:
                raise gsv.GpuSolveError(drv.gs_last_error().decode())
        except Exception as e:  # noqa: BLE001 (reported, never required)
            err = f"{type(e).__name__}: {e}"
        if any_rank(err is not None):
            vc = {"error": err or "failed on another rank"}
        else:
            vt = torch.tensor([ms.value / a.vcycles], dtype=torch.float64, device="cuda")
            if world > 1:
                dist.all_reduce(vt, op=dist.ReduceOp.MAX)
            vc = {"ms": round(vt.item(), 3), "cycles": a.vcycles,
                  "config": f"{dims[0]}x{dims[1]}x{dims[2]} linear 2+2, norm readback included",
                  "first_residual": res}
            if world == 1:  # the other two level-0 passes of the V-cycle, each alone
                vc["level0_kernels"] = vcycle_level0_kernels(grid, max(4, min(a.steps, 20)))
                vc.update(level_split(gsv.GridParams(maxiter=5, tol=0.0, gridDim=dims, mode=gsv.GS_LINEAR,
                                                     preSmoothing=2, postSmoothing=2)))

    cta_ab = None
    if world > 1 and a.cta_ab:
        # the RCCL CTA budget (ncclConfig_t::minCTAs = maxCTAs) on this node's transport: the same timed window
        # on a fresh grid + communicator per value, interleaved twice; the headline above ran the default
        cta_ab = {"note": "per value: max-over-ranks ms per sweep of the same timed window on a fresh grid whose "
                          "RCCL communicator has this CTA budget (two interleaved rounds), and the slowest rank's "
                          "overlapped pair ms; NCCL_NCHANNELS_PER_PEER is per process: " +
                          str(os.environ.get("NCCL_NCHANNELS_PER_PEER"))}
        for rnd in range(2):
            for c in [int(x) for x in a.cta_ab.split(",") if x.strip()]:
                err, res = None, None
                g2 = None
                try:
                    g2 = make_grid(params, rank, world, ctas=c)
                except Exception as e:  # noqa: BLE001 (reported, never required)
                    err = f"{type(e).__name__}: {e}"
                # every rank has its grid (or none has) before any rank enters the timed window's collectives
                if not any_rank(err is not None):
                    try:
                        el, _, kms, _, _ = timed_window(g2, a.warmup, min(a.ramp_ms, 200.0), a.steps)
                        res = (el, kms)
                    except Exception as e:  # noqa: BLE001 (reported, never required)
                        err = f"{type(e).__name__}: {e}"
                elif err is None:
                    err = "grid creation failed on another rank"
                if g2 is not None:
                    g2.close()
                if any_rank(err is not None):
                    cta_ab.setdefault(str(c), []).append({"error": err or "failed on another rank"})
                    continue
                km = torch.tensor([res[1]], dtype=torch.float64, device="cuda")
                dist.all_reduce(km, op=dist.ReduceOp.MAX)
                cta_ab.setdefault(str(c), []).append({"ms_per_step": round(res[0] / a.steps * 1e3, 4),
                                                      "pair_ms_max_rank": round(km.item(), 4)})

    transports = None
    if world > 1 and not rccl_log:
        transports = {"error": "NCCL_DEBUG_FILE preset without NCCL_DEBUG=INFO: no connection log to parse"}
    if world > 1 and rccl_log:
        mine = rccl_transports(rccl_log)
        allt = [None] * world
        dist.all_gather_object(allt, mine)
        # per rank: {peer: [transports]} merged over its communicators (torch's process group and the grids')
        transports = {"per_rank": [], "log": "NCCL_DEBUG=INFO (subsystems INIT,P2P,NET) to NCCL_DEBUG_FILE, "
                                             "connection set-up lines 'Channel .. -> .. via <transport>'"}
        for r, t in enumerate(allt):
            if not isinstance(t, dict) or "error" in t:
                transports["per_rank"].append(t)
                continue
            peers = {}
            for c in t.values():
                for peer, vias in c["peers"].items():
                    for v in vias:
                        if v not in peers.setdefault(peer, []):
                            peers[peer].append(v)
            transports["per_rank"].append({"rank": r, "communicators": len(t), "peers": peers})
        kinds = sorted({v.split("/")[0] for t in transports["per_rank"] if isinstance(t, dict) and "peers" in t
                        for vs in t["peers"].values() for v in vs})
        transports["kinds"] = kinds

    newton = None
    if world == 1 and a.newton_iters > 0:
        newton = newton_timing(n, a.newton_iters)

    c5 = None
    if world == 1 and a.config5:
        grid.close()  # the 512^3 hierarchy is not needed any more
        try:
            c5 = config5_single_gpu(a.steps, 5 if a.vcycles > 0 else 0)
        except Exception as e:  # noqa: BLE001 (reported, never required)
            c5 = {"error": f"{type(e).__name__}: {e}"}
    speedup = None
    if world > 1 and tuple(dims) == (1024, 1024, 1024):
        # strong scaling on 1024^3 (north_star's >= 6x): this line's MLUPS over one GPU's on the same grid.
        # "value" always divides by rank 0's same-job measurement (same node, same run, same software), so the
        # ratio means the same in every round; the driver's committed N=1 record is a secondary field only
        speedup = {"scaling": "strong", "value": None,
                   "note": "value: this line's MLUPS / rank 0's one-GPU MLUPS on the same 1024^3 grid measured in "
                           "this job before the slabs were built (bench.py config5_single_gpu); vs_driver_record: "
                           "the same over the driver's committed N=1 record (secondary)"}
        try:
            with open(CONFIG5_FILE) as f:
                ref1 = json.load(f)
            speedup["vs_driver_record"] = round(value / float(ref1["mlups"]), 3)
            speedup["driver_record_mlups"] = ref1["mlups"]
            speedup["driver_record_source"] = (os.path.relpath(CONFIG5_FILE, REPO) + " (" + ref1.get("source", "?")
                                               + ")")
        except (OSError, ValueError, KeyError) as e:
            speedup["driver_record_error"] = str(e)
        if c5_same_job and "mlups" in c5_same_job:
            speedup["value"] = round(value / float(c5_same_job["mlups"]), 3)
            speedup["one_gpu_mlups"] = c5_same_job["mlups"]
            speedup["one_gpu_pair_kernel_ms"] = c5_same_job.get("pair_kernel_ms")
        else:
            speedup["same_job_error"] = (c5_same_job or {}).get("error", "not measured (--config5 0)")

    c2 = None
    if world == 1 and a.config2:
        try:
            c2 = config2_timing()
        except Exception as e:  # noqa: BLE001 (reported, never required)
            c2 = {"error": f"{type(e).__name__}: {e}"}

    cpu = None
    if rank == 0 and a.cpu_sweeps > 0:
        # north_star: the CPU reference "timed on the same box's host cores ... in the same run" at every N: rank 0
        # runs it after every GPU leg of this job (the other ranks are done); N > 1 takes a reduced sample
        try:
            if world == 1:
                cpu = cpu_baseline(n, a.cpu_sweeps, a.cpu_vcycles)
            else:
                cpu = cpu_baseline(n, max(2, a.cpu_sweeps // 3), 0)
                cpu["note"] = (f"rank 0 of {world}, after every GPU leg of this job, reduced sample; the GPU line's value "
                               f"is the whole job's ({world} GPUs)")
        except Exception as e:  # the baseline is reported, never required
            cpu = {"error": str(e)}

    # weak scaling: every N runs n^3 lattice points per rank (512^3 by default); only N = 8's grid is a
    # BASELINE config (#5: 1024^3); N = 2 / 4 are weak-scaling shapes that keep the N = 1 run's row length
    scaling = "weak" if int(lups_per_rank) == n ** 3 else "strong"
    if world == 1:
        workload = f"{n}^3 linear 7-point fused Jacobi sweep (level 0), BASELINE config #3"
    elif tuple(dims) == (1024, 1024, 1024):
        workload = (f"1024^3 linear 7-point fused Jacobi sweep (level 0) = BASELINE config #5's grid, Z-slab over "
                    f"{world} GPUs ({dims[2] // world} planes per rank)")
    else:
        workload = (f"{dims[0]}x{dims[1]}x{dims[2]} linear 7-point fused Jacobi sweep (level 0), Z-slab over {world} "
                    f"GPUs: a weak-scaling shape with {n}^3 points per rank (not a BASELINE config)")
    if rank == 0:
        line = {
            "metric": "MLUPS (Jacobi smoother) + V-cycle wall-time, 512³ fp64; achieved HBM GB/s %peak",
            "value": round(value, 1),
            "unit": "MLUPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_ms": round(warmup_ms, 1),
            "warmup_sweeps_total": a.warmup + ramp,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (analytic RHS of the reference, v0 = 0)",
            "config": {"workload": workload,
                       "grid": list(dims), "points_per_rank": int(lups_per_rank),
                       "per_rank_slab": [int(dims[0]), int(dims[1]), int(dims[2]) // world],
                       "per_rank_pair_kernel": pair_kernel.split(":")[0],
                       "mode": "linear", "omega": 0.8,
                       "parallelism": f"zslab{world}-rccl" if world > 1 else "single"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_GBPS, 4),
                         "frac_of_measured_ceiling": round(achieved / ceiling["gbps"], 4) if ceiling else None,
                         "frac_of_best_ceiling": (round(achieved / max(c["gbps"] for c in ceilings.values()), 4)
                                                  if ceilings else None),
                         "frac_of_best_store_ceiling": (
                             round(achieved / max(ceilings[k]["gbps"] for k in ("copy", "triad", "write")), 4)
                             if ceilings else None),
                         "ceiling_note": ("frac_of_measured_ceiling: of the streaming triad (the smoother's 2 reads + "
                                          "1 write), frac_of_best_store_ceiling: of the fastest stream that stores "
                                          "(triad, copy, store-only), frac_of_best_ceiling: of the fastest of those "
                                          "and the read-only stream, all measured in this run in two shapes "
                                          "(measured_ceilings)"),
                         "traffic": traffic, "kernel_ms": round(kernel_ms, 4),
                         "kernel": (pair_kernel + ": two fused sweeps per launch (24 B per point per launch)"
                                    if fused else "k_rb: one sweep per launch (24 B per point per launch)"),
                         "lups_per_launch": 2 if fused else 1,
                         "points_per_launch": int(lups_per_rank),
                         "compulsory_bytes_per_lup": BYTES_PER_LUP / (2 if fused else 1),
                         "algorithmic_bytes_per_launch": BYTES_PER_LUP * lups_per_rank,
                         "effective_GBps": round(value / world * BYTES_PER_LUP / 1e3, 1),
                         "effective_GBps_note": ("MLUPS x 24 B per lattice update per GPU, the BASELINE.md "
                                                 "definition; with temporal blocking (2 updates per pass) this is "
                                                 "NOT HBM traffic: the HBM-side figure is `achieved` "
                                                 "(24 B per point per launch / kernel_ms)")},
            "multi_gpu": multi,
            "rccl_cta_ab": cta_ab,
            "rccl_transports": transports,
            "single_sweep_kernel": single,
            "measured_ceiling": ceiling,
            "measured_ceilings": ceilings,
            "vcycle": vc,
            "newton": newton,
            "config5_single_gpu": c5,
            "config2": c2,
            "speedup_vs_1gpu_same_grid": speedup,
            "cpu_baseline": cpu,
            "kernel_build": gsv.build_info(),
        }
        if pmc:
            line["roofline"]["traffic_source"] = pmc.get("source")
        os.write(json_out, (json.dumps(line) + "\n").encode())
    grid.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
