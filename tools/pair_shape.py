"""Time the level-0 fused pair (gs_grid_jacobi, 2 sweeps per launch) on an arbitrary grid shape, e.g. the
per-rank slab of BASELINE config #5 at N=8:   python tools/pair_shape.py 1024 1024 128"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402


def main():
    dims = tuple(int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (1024, 1024, 128)
    p = gsv.GridParams(maxiter=1, gridDim=dims, mode=gsv.GS_LINEAR)
    drv, kl = gsv.driver(), gsv.kernels()
    with gsv.HipGridData(p) as g:
        L = g.getLevel(0).geom
        name = kl.gs_jacobi_sweep2_kernel(C.byref(p.stencil.to_abi()), C.byref(L), 0).decode()
        ms = C.c_float()
        assert drv.gs_grid_time_jacobi(g.handle, 0, 400, 200, C.byref(ms)) == 0, drv.gs_last_error()
        per_pair = ms.value / 100
        pts = dims[0] * dims[1] * dims[2]
        print(f"{dims}: {per_pair:.4f} ms per pair, {2 * pts / per_pair / 1e6:.1f} GLUPS, "
              f"{24.0 * pts / (per_pair * 1e-3) / 1e9:.1f} GB/s algorithmic; {name}")


if __name__ == "__main__":
    main()
