"""The three level-0 passes of a NEWTON V-cycle timed alone on a 512^3 grid through the kernel C ABI
(and their LINEAR counterparts), HIP events around K launches each, interleaved over rounds:
    python tools/newton_kprobe.py [rounds] [K] [n]
  (each in mode 3 = GS_NEWTON_B with the factor field from gs_newton_bfac, mode 2 = GS_NEWTON, mode 0)
  spec pair    gs_jacobi_sweep2_norm  (two sweeps + the norm partials of the input's residual), 32 B/point
  rr           gs_residual_restrict   (residual + full weighting), 25 B/point (LINEAR 17)
  pro pair     gs_jacobi_sweep2_prolong_ws (prolongation + correction + two sweeps), 33 B/point (LINEAR 25)
Inputs: smooth fields (v = 0.25 sin, f = 1, newtonV = 0.1 sin, coarse v = 0.05), so every launch runs the
arithmetic of a sane iterate. Prints one JSON line: ms per launch (min over rounds) and GB/s algorithmic.
GS_KPROBE_LIB=<path to an alternative libgpusolve_hip.so> loads that build instead (A/B of kernel
variants: the same script against two builds). GS_KPROBE_EFIELD=1 (with a -DGS_EXP_EFIELD build) gives
the pairs a second field E = exp(newtonV) of newtonV's shape and passes its distance (gs_exp_set_efoff)."""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "gpu-solve_amd"))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    import numpy as np
    import torch
    import gpusolve as gsv
    from gpusolve import _abi
    if os.environ.get("GS_KPROBE_LIB"):
        _abi.KERNEL_LIB = os.environ["GS_KPROBE_LIB"]
    from gpusolve.devfield import DevField
    kl = gsv.kernels()
    S = gsv.Stencil().to_abi()
    dims = (n, n, n)
    cd = tuple(d // 2 for d in dims)
    h, hc = 1.0 / (n + 1), 1.0 / (cd[1] + 1)

    def smooth(a, amp):
        x = torch.linspace(0, 3.0, a.zyx.shape[2], dtype=torch.float64, device="cuda")
        a.zyx[1:-1, 1:-1, 1:-1] = amp * torch.sin(x[1:-1]).view(1, 1, -1)
        a.zyx[:, :, a.nx + 1:] = 0.0
        return a

    v = smooth(DevField(*dims), 0.25)
    w = smooth(DevField(*dims), 0.1)
    if os.environ.get("GS_KPROBE_EFIELD"):
        e = DevField(*dims)
        e.zyx_ext.copy_(torch.exp(w.zyx_ext))
        assert (e.ptr - w.ptr) % 8 == 0
        fn = getattr(kl, "gs_exp_set_efoff")  # only a -DGS_EXP_EFIELD build exports it
        fn.argtypes, fn.restype = [C.c_int64], None
        fn((e.ptr - w.ptr) // 8)
    f = DevField(*dims, fill=1.0)
    out = DevField(*dims)
    cv = DevField(*cd, fill=0.05)
    cf = DevField(*cd)
    L, Lc = v.level(h), cv.level(hc)
    st = torch.cuda.current_stream()
    s = st.cuda_stream
    parts = torch.zeros(max(1, kl.gs_jacobi_sweep2_num_partials(C.byref(S), C.byref(L), 2)) + 4096,
                        dtype=torch.float64, device="cuda")
    res = {}
    # mode 3 (GS_NEWTON_B): the same kernels with the precomputed factor as their w operand
    b = DevField(*dims)
    assert kl.gs_newton_bfac(C.byref(w.level(h)), 1.0, w.ptr, b.ptr, None) == 0
    for mode, name in ((3, "newtonb"), (2, "newton"), (0, "linear")):
        wp = (w.ptr if mode == 2 else b.ptr) if mode >= 2 else None
        wsn = kl.gs_jacobi_sweep2_prolong_ws_elems(C.byref(S), C.byref(L), mode)
        ws = torch.empty(max(1, wsn), dtype=torch.float64, device="cuda")

        def pair():
            assert kl.gs_jacobi_sweep2_norm(C.byref(S), C.byref(L), mode, 0.8, 1.0, v.ptr, out.ptr, f.ptr, wp, 0, 0,
                                            parts.data_ptr(), s) == 0

        def rr():
            assert kl.gs_residual_restrict(C.byref(S), C.byref(L), mode, 1.0, v.ptr, f.ptr, wp, cf.ptr, None,
                                           C.byref(Lc), s) == 0

        def pro():
            assert kl.gs_jacobi_sweep2_prolong_ws(C.byref(S), C.byref(L), mode, 0.8, 1.0, v.ptr, cv.ptr, None,
                                                  C.byref(Lc), out.ptr, f.ptr, wp, 0, 0, ws.data_ptr(), wsn, s) == 0

        def padd():
            assert kl.gs_prolong_add(cv.ptr, None, C.byref(Lc), out.ptr, C.byref(L), s) == 0

        nw = mode >= 2
        bpp = {"pair": 32.0 if nw else 24.0, "rr": 25.0 if nw else 17.0,
               "pro": 33.0 if nw else 25.0, "prolong_add": 16.0}
        for _ in range(rounds):
            for kname, fn in (("pair", pair), ("rr", rr), ("pro", pro), ("prolong_add", padd)):
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(K):
                    fn()
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / K
                key = f"{name}_{kname}"
                res.setdefault(key, []).append(round(ms, 4))
        for kname in ("pair", "rr", "pro", "prolong_add"):
            key = f"{name}_{kname}"
            m = min(res[key])
            res[key + "_GBps"] = round(bpp[kname] * n ** 3 / (m * 1e-3) / 1e9, 1)
    a = out.to_xyz() if n <= 128 else None
    print(json.dumps({"lib": _abi.KERNEL_LIB, "n": n, "K": K, "ms": res,
                      "checksum": None if a is None else float(np.nansum(a))}))


if __name__ == "__main__":
    main()
