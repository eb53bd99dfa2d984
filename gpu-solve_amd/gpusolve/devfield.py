"""Device fields in the kernel ABI's pitched layout, backed by torch (device memory plumbing only).

Used by the kernel-level parity tests and bench.py to call libgpusolve_hip.so's launchers
directly. Host copies are returned as dense arrays indexed [x][y][z] — the reference's axis order —
so they compare element-wise with the oracle.
"""
import numpy as np
import torch

from . import field_layout, gs_level


class DevField:
    def __init__(self, nx: int, ny: int, nz: int, device="cuda", fill=0.0):
        self.nx, self.ny, self.nz = nx, ny, nz
        self.ldy, self.ldz, alloc, origin = field_layout(nx, ny, nz)
        self.buf = torch.full((alloc,), float(fill), dtype=torch.float64, device=device)
        self.origin = origin
        self.ptr = self.buf.data_ptr() + 8 * origin
        self.span = self.ldz * (nz + 2)
        # [z][y][x] view of the padded region (x extends to ldy; columns >= nx+2 are pitch padding)
        self.zyx = self.buf[origin: origin + self.span].view(nz + 2, ny + 2, self.ldy)
        # the same including the second ghost planes z = -1 and z = nz+2
        self.zyx_ext = self.buf[origin - self.ldz: origin + self.span + self.ldz].view(nz + 4, ny + 2, self.ldy)

    def level(self, h: float, z0: int = 0) -> gs_level:
        return gs_level(self.nx, self.ny, self.nz, self.ldy, self.ldz, z0, h)

    def to_xyz(self) -> np.ndarray:
        torch.cuda.synchronize()
        a = self.zyx[:, :, : self.nx + 2].cpu().numpy()
        return np.ascontiguousarray(a.transpose(2, 1, 0))

    def from_xyz(self, arr: np.ndarray):
        a = np.asarray(arr, dtype=np.float64)
        assert a.shape == (self.nx + 2, self.ny + 2, self.nz + 2), a.shape
        self.zyx[:, :, : self.nx + 2] = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 1, 0))).to(self.buf.device)
        return self

    def from_xyz_ext(self, arr: np.ndarray):
        """Set planes z = -1 .. nz+2 from an array shaped (nx+2, ny+2, nz+4)."""
        a = np.asarray(arr, dtype=np.float64)
        assert a.shape == (self.nx + 2, self.ny + 2, self.nz + 4), a.shape
        self.zyx_ext[:, :, : self.nx + 2] = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 1, 0))).to(
            self.buf.device)
        return self

    def zero(self):
        self.buf.zero_()
        return self
