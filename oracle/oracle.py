"""ctypes wrapper of the CPU ORACLE (oracle/build/libgs_oracle.so) — TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; the product
(gpu-solve_amd/) never imports it. Arrays are numpy float64 in the reference layout: shape
(nx+2, ny+2, nz+2), C-contiguous (z unit-stride, src/cpu/Vector3.cpp:16).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libgs_oracle.so")
CLI = os.path.join(HERE, "build", "gso_cli")
REF_PROBE = os.path.join(HERE, "_ref", "ref_probe")
REF_EXE = os.path.join(HERE, "_ref", "GpuSolve-cpu")

LINEAR, NONLINEAR, NEWTON = 0, 1, 2
CANONICAL = [(0, 0, 0), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]


class Stencil(C.Structure):
    _fields_ = [("s", C.c_double * 7), ("ox", C.c_int * 7), ("oy", C.c_int * 7), ("oz", C.c_int * 7)]

    @classmethod
    def make(cls, values=(6, -1, -1, -1, -1, -1, -1), offsets=CANONICAL):
        s = cls()
        for i in range(7):
            s.s[i] = float(values[i])
            s.ox[i], s.oy[i], s.oz[i] = offsets[i]
        return s


_lib = None
D = C.POINTER(C.c_double)
I3 = C.c_int64 * 3


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError(f"{LIB} missing: run `make -C oracle`")
        L = C.CDLL(LIB)
        sig = {
            "gso_residual": (C.c_double, [C.POINTER(Stencil), I3, C.c_double, C.c_int, C.c_double, D, D, D, D]),
            "gso_jacobi": (None, [C.POINTER(Stencil), I3, C.c_double, C.c_int, C.c_double, C.c_double, C.c_int,
                                  D, D, D, D]),
            "gso_apply_op": (None, [C.POINTER(Stencil), I3, C.c_double, C.c_double, D, D]),
            "gso_restrict": (None, [D, I3, D, I3]),
            "gso_interpolate": (None, [D, I3, D, I3]),
            "gso_newton_F": (C.c_double, [C.POINTER(Stencil), I3, C.c_double, C.c_double, D, D, D]),
            "gso_rhs": (None, [I3, C.c_double, C.c_int, C.c_double, D]),
            "gso_grid_create": (C.c_void_p, [C.POINTER(Stencil), I3, C.c_int, C.c_int64, C.c_double, C.c_double,
                                             C.c_double, C.c_int64, C.c_int64]),
            "gso_grid_destroy": (None, [C.c_void_p]),
            "gso_grid_levels": (C.c_int, [C.c_void_p]),
            "gso_grid_level_info": (None, [C.c_void_p, C.c_int, I3, D]),
            "gso_grid_field": (D, [C.c_void_p, C.c_int, C.c_int]),
            "gso_grid_vcycle": (C.c_double, [C.c_void_p]),
            "gso_grid_solve": (C.c_int, [C.c_void_p, C.c_int, D, C.c_int]),
            "gso_num_threads": (C.c_int, []),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(D)


def _dims(a):
    return I3(*(s - 2 for s in a.shape))


def zeros(nx, ny, nz):
    return np.zeros((nx + 2, ny + 2, nz + 2))


def residual(v, f, h, mode=LINEAR, gamma=1.0, w=None, stencil=None, want_r=True):
    S = stencil or Stencil.make()
    r = np.zeros_like(v) if want_r else None
    n = lib().gso_residual(C.byref(S), _dims(v), h, mode, gamma, _p(v), _p(f), _p(w if w is not None else v), _p(r))
    return r, n


def jacobi(v, f, h, mode=LINEAR, omega=0.8, gamma=1.0, sweeps=1, w=None, stencil=None):
    S = stencil or Stencil.make()
    out = v.copy()
    scratch = np.zeros_like(v)
    lib().gso_jacobi(C.byref(S), _dims(v), h, mode, omega, gamma, sweeps, _p(out), _p(f),
                     _p(w if w is not None else v), _p(scratch))
    return out


def apply_op(u, h, gamma=1.0, stencil=None):
    S = stencil or Stencil.make()
    out = np.zeros_like(u)
    lib().gso_apply_op(C.byref(S), _dims(u), h, gamma, _p(u), _p(out))
    return out


def restrict(fine, coarse_shape_interior):
    c = zeros(*coarse_shape_interior)
    lib().gso_restrict(_p(fine), _dims(fine), _p(c), _dims(c))
    return c


def interpolate(coarse, fine_shape_interior):
    e = zeros(*fine_shape_interior)
    lib().gso_interpolate(_p(coarse), _dims(coarse), _p(e), _dims(e))
    return e


def newton_F(w, F, h, gamma=1.0, stencil=None):
    S = stencil or Stencil.make()
    f = np.zeros_like(w)
    n = lib().gso_newton_F(C.byref(S), _dims(w), h, gamma, _p(w), _p(F), _p(f))
    return f, n


def rhs(nx, ny, nz, mode, gamma=1.0, h=None):
    f = zeros(nx, ny, nz)
    lib().gso_rhs(I3(nx, ny, nz), h if h is not None else 1.0 / (ny + 1), mode, gamma, _p(f))
    return f


FIELD = {"v": 0, "restV": 1, "newtonV": 2, "f": 3, "r": 4, "e": 5}


class Grid:
    """Oracle level hierarchy + drivers (CpuGridData + CpuSolver / NewtonSolver restated)."""

    def __init__(self, dims, mode=LINEAR, maxiter=10, tol=0.0, omega=0.8, gamma=1.0, pre=2, post=2,
                 stencil=None):
        self.S = stencil or Stencil.make()
        self.dims = tuple(dims)
        self.maxiter = maxiter
        self.h = lib().gso_grid_create(C.byref(self.S), I3(*dims), mode, maxiter, tol, omega, gamma, pre, post)

    def __del__(self):
        if getattr(self, "h", None):
            lib().gso_grid_destroy(self.h)
            self.h = None

    def levels(self):
        return lib().gso_grid_levels(self.h)

    def level_info(self, l):
        d = I3()
        h = C.c_double()
        lib().gso_grid_level_info(self.h, l, d, C.byref(h))
        return tuple(d), h.value

    def field(self, l, name):
        (nx, ny, nz), _ = self.level_info(l)
        p = lib().gso_grid_field(self.h, l, FIELD[name])
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(nx + 2, ny + 2, nz + 2))

    def vcycle(self):
        return lib().gso_grid_vcycle(self.h)

    def solve(self, print_mode=0):
        cap = 4 * (self.maxiter + 2)
        hist = (C.c_double * cap)()
        n = lib().gso_grid_solve(self.h, print_mode, hist, cap)
        return list(hist[: min(n, cap)])
