"""gpusolve — Python mirror of the GpuSolve-hip backend interface (MI355X, HIP, fp64).

Same names, argument meaning and error behaviour as the reference's C++ backend contract
(Bricktricker/gpu-solve):

    GridParams / Stencil          src/gridParams.h:7-47
    read_config                   src/main.cpp:32-85 (14-line config file)
    HipGridData(params)           CpuGridData(const GridParams&)      src/cpu/CpuGridData.cpp:15-79
    HipSolver.solve(grid)         CpuSolver::solve                    src/cpu/CpuSolver.cpp:12-43
    HipSolver.vcycle / jacobi / compResidual                          src/cpu/CpuSolver.cpp:45-180
    NewtonSolver.solve(grid)      NewtonSolver::solve                 src/cpu/NewtonSolver.cpp:10-44

Everything runs through libgpusolve_driver.so -> libgpusolve_hip.so (hand-written gfx950 kernels).
There is no CPU fallback: without the built libraries or a GPU the calls raise.
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

from . import _abi
from ._abi import GS_LINEAR, GS_NEWTON, GS_NEWTON_B, GS_NEWTON_G, GS_NONLINEAR, gs_level, gs_params, gs_stencil, kernels, driver, diag  # noqa: F401

CANONICAL_OFFSETS = [(0, 0, 0), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]


class GpuSolveError(RuntimeError):
    """A backend failure; str() is what GpuSolve-hip prints after "Exception: "."""


@dataclass
class Stencil:
    values: List[float] = field(default_factory=lambda: [6.0, -1, -1, -1, -1, -1, -1])
    offsets: List[Tuple[int, int, int]] = field(default_factory=lambda: list(CANONICAL_OFFSETS))

    def to_abi(self) -> gs_stencil:
        s = gs_stencil()
        for i in range(7):
            s.s[i] = float(self.values[i])
            s.ox[i], s.oy[i], s.oz[i] = (int(o) for o in self.offsets[i])
        return s


@dataclass
class GridParams:
    LINEAR = GS_LINEAR
    NONLINEAR = GS_NONLINEAR
    NEWTON = GS_NEWTON

    maxiter: int = 10
    tol: float = 0.0
    gridDim: Tuple[int, int, int] = (31, 31, 31)
    mode: int = GS_LINEAR
    preSmoothing: int = 2
    postSmoothing: int = 2
    omega: float = 0.8
    gamma: float = 1.0
    stencil: Stencil = field(default_factory=Stencil)
    printProgress: bool = True

    @property
    def h(self) -> float:  # src/main.cpp:84
        return 1.0 / (self.gridDim[1] + 1)

    def to_abi(self) -> gs_params:
        p = gs_params()
        p.maxiter, p.tol = int(self.maxiter), float(self.tol)
        for i in range(3):
            p.dims[i] = int(self.gridDim[i])
        p.mode, p.pre, p.post = int(self.mode), int(self.preSmoothing), int(self.postSmoothing)
        p.omega, p.gamma = float(self.omega), float(self.gamma)
        p.stencil = self.stencil.to_abi()
        return p

    def config_text(self) -> str:
        st = self.stencil
        return "\n".join([str(self.maxiter), repr(float(self.tol)), *(str(d) for d in self.gridDim), str(self.mode),
                          str(self.preSmoothing), str(self.postSmoothing), repr(float(self.omega)),
                          repr(float(self.gamma)), " ".join(repr(float(v)) for v in st.values),
                          *(" ".join(str(o[a]) for o in st.offsets) for a in range(3))]) + "\n"


def parse_config(text: str) -> GridParams:
    """Parses the reference's 14-line config text (README.md:17-33) with the library's parser."""
    p = gs_params()
    rc = driver().gs_parse_config(text.encode(), C.byref(p))
    if rc == 1:
        raise ValueError("Invalid mode")
    if rc == 2:
        raise ValueError("Invalid stencil offset (must be -1, 0 or 1)")
    st = Stencil([p.stencil.s[i] for i in range(7)],
                 [(p.stencil.ox[i], p.stencil.oy[i], p.stencil.oz[i]) for i in range(7)])
    return GridParams(maxiter=p.maxiter, tol=p.tol, gridDim=tuple(p.dims), mode=p.mode, preSmoothing=p.pre,
                      postSmoothing=p.post, omega=p.omega, gamma=p.gamma, stencil=st)


def read_config(path: str) -> GridParams:
    with open(path) as f:
        return parse_config(f.read())


def _check(rc: int):
    if rc != 0:
        raise GpuSolveError(driver().gs_last_error().decode())


FIELDS = {"v": 0, "restV": 1, "newtonV": 2, "f": 3, "r": 4, "newtonF": 5}


@dataclass
class LevelInfo:
    levelDim: Tuple[int, int, int]
    h: float
    geom: gs_level


class HipGridData:
    """Device-resident level hierarchy (fields in HBM for the object's lifetime)."""

    def __init__(self, params: GridParams):
        self.params = params
        self._abi_params = params.to_abi()
        self.handle = driver().gs_grid_create(C.byref(self._abi_params))
        if not self.handle:
            raise GpuSolveError(driver().gs_last_error().decode())

    def close(self):
        if getattr(self, "handle", None):
            driver().gs_grid_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def mode(self):
        return self.params.mode

    def numLevels(self) -> int:
        return driver().gs_grid_num_levels(self.handle)

    def getLevel(self, l: int) -> LevelInfo:
        g = gs_level()
        if driver().gs_grid_level(self.handle, l, C.byref(g)) != 0:
            raise IndexError(l)
        return LevelInfo((g.nx, g.ny, g.nz), g.h, g)

    def stream(self) -> int:
        return driver().gs_grid_stream(self.handle)

    def field(self, level: int, name: str) -> np.ndarray:
        """Copy of a padded field as a dense array indexed [x][y][z] (the reference's axis order)."""
        g = self.getLevel(level).geom
        host = np.empty((g.nz + 2, g.ny + 2, g.nx + 2), dtype=np.float64)
        _check(driver().gs_grid_download(self.handle, level, FIELDS[name], host.ctypes.data_as(_abi.dptr)))
        return host.transpose(2, 1, 0)

    def set_field(self, level: int, name: str, arr_xyz: np.ndarray):
        g = self.getLevel(level).geom
        host = np.ascontiguousarray(np.asarray(arr_xyz, dtype=np.float64).transpose(2, 1, 0))
        assert host.shape == (g.nz + 2, g.ny + 2, g.nx + 2)
        _check(driver().gs_grid_upload(self.handle, level, FIELDS[name], host.ctypes.data_as(_abi.dptr)))

    def sync(self):
        _check(driver().gs_grid_sync(self.handle))

    def dump(self, path: str, level: int = 0, name: str = "v"):
        """Vector3::dump (src/cpu/Vector3.cpp:56-78) of a field: the plotter.py input format."""
        _check(driver().gs_grid_dump(self.handle, level, FIELDS[name], path.encode()))


def dump_write(arr_xyz: np.ndarray, path: str):
    """Vector3::dump text of a padded host array indexed [x][y][z] (the driver's writer)."""
    a = np.ascontiguousarray(np.asarray(arr_xyz, dtype=np.float64).transpose(2, 1, 0))
    px, py, pz = arr_xyz.shape
    _check(driver().gs_dump_write(a.ctypes.data_as(_abi.dptr), px, py, pz, path.encode()))


def read_dump(path: str) -> np.ndarray:
    """plotter.py's readFile (reference plotter.py:10-26): a dump back into an [x][y][z] array."""
    with open(path) as f:
        px, py, pz = (int(t) for t in f.readline().split())
        data = np.loadtxt(f, ndmin=2)
    out = np.zeros((px, py, pz))
    out[data[:, 0].astype(int), data[:, 1].astype(int), data[:, 2].astype(int)] = data[:, 3]
    return out


def analytic_error(mesh: np.ndarray) -> float:
    """Max |computed - u| over the mesh, u = (x-x^2)(y-y^2)(z-z^2) on linspace(0, 1, n) per axis
    (reference plotter.py:7-8, 28-31: the exact solution of the NONLINEAR / NEWTON problems)."""
    g = [np.linspace(0.0, 1.0, n) for n in mesh.shape]
    X, Y, Z = np.meshgrid(*g, indexing="ij")
    return float(np.abs(mesh - (X - X * X) * (Y - Y * Y) * (Z - Z * Z)).max())


class HipSolver:
    @staticmethod
    def solve(grid: HipGridData, print_progress: bool = False) -> List[float]:
        """Runs the solve for grid's mode (main.cpp:88-94 dispatch); returns the residual history."""
        cap = 4 * (int(grid.params.maxiter) + 2)
        hist = (C.c_double * cap)()
        n = C.c_int(0)
        _check(driver().gs_grid_solve(grid.handle, 1 if print_progress else 0, hist, cap, C.byref(n)))
        return list(hist[: min(n.value, cap)])

    @staticmethod
    def vcycle(grid: HipGridData) -> float:
        r = C.c_double()
        _check(driver().gs_grid_vcycle(grid.handle, C.byref(r)))
        return r.value

    @staticmethod
    def jacobi(grid: HipGridData, level: int, sweeps: int):
        _check(driver().gs_grid_jacobi(grid.handle, level, sweeps))

    @staticmethod
    def compResidual(grid: HipGridData, level: int) -> float:
        r = C.c_double()
        _check(driver().gs_grid_residual_norm(grid.handle, level, C.byref(r)))
        return r.value


class NewtonSolver:
    @staticmethod
    def solve(grid: HipGridData, print_progress: bool = False) -> List[float]:
        if grid.mode != GS_NEWTON:
            raise ValueError("NewtonSolver needs mode NEWTON")
        return HipSolver.solve(grid, print_progress)


def field_layout(nx: int, ny: int, nz: int):
    """(ldy, ldz, alloc_elems, origin_offset) of include/gpusolve_hip.h's pitched layout."""
    a, b, c, d = (C.c_int64() for _ in range(4))
    rc = kernels().gs_field_layout(nx, ny, nz, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
    if rc:
        raise ValueError(kernels().gs_strerror(rc).decode())
    return a.value, b.value, c.value, d.value


def build_info() -> str:
    return kernels().gs_build_info().decode()
