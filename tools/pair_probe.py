"""Why does the fused pair run slower inside the driver than in kbench? Times the same kernel on
(a) the driver's level-0 fields through gs_grid_jacobi, (b) the same fields through the kernel ABI,
(c) DevFields with random data, (d) DevFields holding copies of the driver's fields."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def timeit(fn, stream, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = 512
    kl, drv = gsv.kernels(), gsv.driver()
    p = gsv.GridParams(maxiter=1, gridDim=(n, n, n), printProgress=False)
    grid = gsv.HipGridData(p)
    S = p.stencil.to_abi()
    L = grid.getLevel(0).geom
    st = grid.stream()
    gstream = torch.cuda.ExternalStream(st)
    print("fused level 0:", drv.gs_grid_level_fused(grid.handle, 0))
    for it in range(3):
        ms = timeit(lambda: drv.gs_grid_jacobi(grid.handle, 0, 2), gstream)
        print(f"(a) driver pair: {ms:.4f} ms")
    v = drv.gs_grid_field(grid.handle, 0, 0)
    f = drv.gs_grid_field(grid.handle, 0, 3)
    tmp = DevField(n, n, n)
    ms = timeit(lambda: kl.gs_jacobi_sweep2(C.byref(S), C.byref(L), 0, 0.8, 1.0, v, tmp.ptr, f, None, 0, 0, st), gstream)
    print(f"(b) ABI pair on driver fields: {ms:.4f} ms")
    cur = torch.cuda.current_stream()
    vr, fr, out = DevField(n, n, n), DevField(n, n, n), DevField(n, n, n)
    g = torch.Generator(device="cuda").manual_seed(3)
    inner = vr.zyx[1:-1, 1:-1, 1:n + 1]
    inner.copy_(torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) * 1e-3)
    assert kl.gs_rhs_init(C.byref(vr.level(1.0 / (n + 1))), fr.ptr, 0, 1.0 / (n + 1), 1.0, cur.cuda_stream) == 0
    Lr = vr.level(1.0 / (n + 1))
    ms = timeit(lambda: kl.gs_jacobi_sweep2(C.byref(S), C.byref(Lr), 0, 0.8, 1.0, vr.ptr, out.ptr, fr.ptr, None, 0, 0,
                                            cur.cuda_stream), cur)
    print(f"(c) random v, rhs f: {ms:.4f} ms")
    # copy the driver's v into vr
    host = grid.field(0, "v")
    vr.from_xyz(host)
    ms = timeit(lambda: kl.gs_jacobi_sweep2(C.byref(S), C.byref(Lr), 0, 0.8, 1.0, vr.ptr, out.ptr, fr.ptr, None, 0, 0,
                                            cur.cuda_stream), cur)
    print(f"(d) driver's v copied, rhs f: {ms:.4f} ms")
    import numpy as np
    inner = host[1:-1, 1:-1, 1:-1]
    print("v stats: zeros", int((inner == 0).sum()), "min|v|", float(np.abs(inner[inner != 0]).min()) if (inner != 0).any() else 0)
    fh = grid.field(0, "f")[1:-1, 1:-1, 1:-1]
    print("f stats: zeros", int((fh == 0).sum()), "max", float(np.abs(fh).max()))
    vr.zero()
    ms = timeit(lambda: kl.gs_jacobi_sweep2(C.byref(S), C.byref(Lr), 0, 0.8, 1.0, vr.ptr, out.ptr, fr.ptr, None, 0, 0,
                                            cur.cuda_stream), cur)
    print(f"(e) v = 0: {ms:.4f} ms")


if __name__ == "__main__":
    main()
