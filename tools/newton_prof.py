"""One 512^3 Newton iteration (BASELINE config #4) for a kernel trace:
    rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python tools/newton_prof.py
then `python tools/kernel_agg.py <dir>/run_kernel_trace.csv`."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-solve_amd"))
import gpusolve as gsv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
p = gsv.GridParams(maxiter=1, tol=0.0, gridDim=(n, n, n), mode=gsv.GS_NEWTON)
with gsv.HipGridData(p) as g:
    print(gsv.NewtonSolver.solve(g))
