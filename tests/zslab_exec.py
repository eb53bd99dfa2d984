"""Replays the driver's own Z-slab schedule (gs_zslab_schedule: HipGridData / HipSolver in trace mode,
gs_grid.cpp) on CPU ranks with the oracle's arithmetic — TEST INFRASTRUCTURE (tests/ only).

Every op of the traced schedule is executed here exactly as the HIP kernel it stands for would
execute it on this rank's slab (same planes, same ghost planes, same exchange partners), with the
reference's point expressions evaluated in the reference's order (src/cpu/CpuSolver.cpp:45-180,
:211-290) on numpy float64 — so a correct schedule reproduces the single-domain oracle bit for bit, and
a wrong one (a missing or misplaced exchange, a wrong plane range, a wrong ghost depth) does not.
Ghost planes hold NaN until an exchange fills them, so any read of a stale ghost plane poisons the
result. LINEAR mode (the schedule BASELINE config #5 runs) bit for bit; NEWTON mode (NewtonSolver.cpp:10-108:
newtonF, the fused newtonV update with its ghost planes, the per-level newtonV restriction, the inner solves)
with numpy's exp in place of libm's, so to ~1e-10 instead of bit for bit.

Arrays use the reference layout (x, y, z), z last; a level's array covers global planes
[base, base + NP) with base = lo - 2 on a Z-slab level (two ghost planes each side) and -1 on a
replicated level.
"""
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

import gpusolve as gsv
import oracle as O

STENCIL = (6.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0)
LINEAR, NEWTON = 0, 2


def schedule(params, nranks, rank, min_points):
    d = gsv.driver()
    p = params.to_abi()
    n = C.c_int64()
    assert d.gs_zslab_schedule(C.byref(p), nranks, rank, min_points, None, 0, C.byref(n)) == 0, d.gs_last_error()
    buf = C.create_string_buffer(n.value + 1)
    assert d.gs_zslab_schedule(C.byref(p), nranks, rank, min_points, buf, n.value + 1, C.byref(n)) == 0
    ops = []
    for line in buf.value.decode().splitlines():
        t = line.split()
        kv = {}
        for a in t[1:]:
            k, v = a.split("=", 1)
            kv[k] = v if k == "field" else int(v)
        ops.append((t[0], kv))
    return ops


def mutate(ops, kind):
    """A deliberately broken schedule (tests the replay's power to catch one): "halo" drops the first
    ghost exchange of a level-1 iterate, "depth" exchanges level-0 iterate ghosts one plane deep only,
    "range" shortens the first interior pair's plane range by one plane, "bfac" drops the second Newton
    iteration's GS_NEWTON_B factor of level 0 (its inner solve reads the first iteration's)."""
    out = [(op, dict(kv)) for op, kv in ops]
    if kind == "bfac":
        idx = [i for i, (op, kv) in enumerate(out) if op == "bfac" and kv["L"] == 0]
        del out[idx[1]]
        return out
    for i, (op, kv) in enumerate(out):
        if kind == "halo" and op == "halo" and kv.get("L") == 1 and kv["field"] == "vAlt":
            del out[i]
            break
        if kind == "depth" and op == "halo" and kv["field"] == "vAlt" and kv["L"] == 0:
            kv["depth"] = 1
        if kind == "range" and op == "pair" and kv["L"] == 0 and kv["z1"] == 3:
            kv["z2"] -= 1
            break
    return out


def plan(dims, nranks, min_points):
    d = gsv.driver()
    L = 16
    distributed = (C.c_int * L)()
    lo = (C.c_int64 * (L * nranks))()
    hi = (C.c_int64 * (L * nranks))()
    n = d.gs_zslab_plan((C.c_int64 * 3)(*dims), nranks, min_points, L, distributed, lo, hi)
    return [(bool(distributed[l]), [lo[l * nranks + r] for r in range(nranks)], [hi[l * nranks + r] for r in range(nranks)])
            for l in range(n)]


def level_dims(dims, n):
    out = [tuple(dims)]
    for _ in range(n - 1):
        out.append(tuple(x // 2 for x in out[-1]))
    return out


class Level:
    def __init__(self, dims, dist_, lo, hi, rank):
        self.nx, self.ny, self.nz = dims
        self.h = 1.0 / (self.ny + 1)
        self.dist = dist_
        self.lo_all, self.hi_all = lo, hi
        if dist_:
            self.lo, self.hi = lo[rank], hi[rank]
            self.base = self.lo - 2
            npl = self.hi - self.lo + 5
        else:
            self.lo, self.hi = 1, self.nz
            self.base = -1
            npl = self.nz + 4
        shape = (self.nx + 2, self.ny + 2, npl)
        nan = np.full(shape, np.nan)
        self.fields = {"v": np.zeros(shape), "vAlt": np.zeros(shape), "f": np.zeros(shape), "r": np.zeros(shape),
                       "newtonV": np.zeros(shape), "newtonF": np.zeros(shape)}
        # ghost planes of f / r are unknown until exchanged (NaN: any read before poisons the result);
        # v and vAlt start as the zero iterate everywhere, ghost planes included, as on the device
        if dist_:
            for name in ("f", "r"):
                a = self.fields[name]
                for g in (self.lo - 2, self.lo - 1, self.hi + 1, self.hi + 2):
                    if 1 <= g <= self.nz:
                        a[:, :, g - self.base] = nan[:, :, 0]
        self.zero_v = False

    def idx(self, g):
        return g - self.base

    def local_to_global(self, z):
        return z + self.lo - 1


def stencil_div(A, zi, hh):
    """(sum_i S_i A(p + o_i)) / hh at the interior x / y points of array planes zi (reference order)."""
    s0, s1, s2, s3, s4, s5, s6 = STENCIL
    c = A[1:-1, 1:-1, zi]
    s = 0.0 + s0 * c
    s = s + s1 * A[2:, 1:-1, zi]
    s = s + s2 * A[:-2, 1:-1, zi]
    s = s + s3 * A[1:-1, 2:, zi]
    s = s + s4 * A[1:-1, :-2, zi]
    s = s + s5 * A[1:-1, 1:-1, zi + 1]
    s = s + s6 * A[1:-1, 1:-1, zi - 1]
    return s / hh


def operator(V, zi, L, mode, W, gamma):
    """A(V) at the interior x / y points of array planes zi: the stencil over h^2, plus NEWTON's
    gamma (1 + w) v exp(w) with w = W (CpuSolver.cpp:56-66, reference order); also A = gamma (1 + w),
    E = exp(w) for the update's denominator."""
    s = stencil_div(V, zi, L.h * L.h)
    if mode == NEWTON:
        w = W[1:-1, 1:-1, zi]
        A, E = gamma * (1 + w), np.exp(w)
        return s + A * V[1:-1, 1:-1, zi] * E, A, E
    return s, None, None


def sweep_planes(V, F, gplanes, L, omega, keep=None, mode=LINEAR, W=None, gamma=1.0):
    """One Jacobi sweep (CpuSolver.cpp:144-171) of array V at global planes gplanes: returns the
    new values of those planes (whole padded cross-sections; boundary rows / columns keep V) and the
    residual r = f - A V there."""
    zi = np.array([L.idx(g) for g in gplanes])
    hh = L.h * L.h
    alpha = hh / STENCIL[0]
    a, A, E = operator(V, zi, L, mode, W, gamma)
    r = F[1:-1, 1:-1, zi] - a
    out = V[:, :, zi].copy()
    if mode == NEWTON:
        out[1:-1, 1:-1, :] = V[1:-1, 1:-1, zi] + omega * (r / (STENCIL[0] / hh + A * E))
    else:
        out[1:-1, 1:-1, :] = V[1:-1, 1:-1, zi] + omega * (alpha * r)
    if keep is not None:
        for j, g in enumerate(gplanes):
            if keep(g):
                out[:, :, j] = V[:, :, zi[j]]
    return out, r


def prolong_full(c, fine_dims):
    """Trilinear prolongation in closed form, X then Y then Z pass (CpuSolver.cpp:240-290, SURVEY.md
    Appendix A.7); c is a padded coarse array (any NaN planes propagate), result padded fine."""
    def axis(a, n_f, ax):
        P = n_f + 2
        i = np.arange(P)
        lo_ = i // 2
        hi_ = np.minimum(i // 2 + 1, a.shape[ax] - 1)
        A_lo = np.take(a, lo_, axis=ax)
        A_hi = np.take(a, hi_, axis=ax)
        odd = (i % 2 == 1)
        shape = [1, 1, 1]
        shape[ax] = P
        odd = odd.reshape(shape)
        out = np.where(odd, 0.5 * A_lo + 0.5 * A_hi, A_lo)
        last = [slice(None)] * 3
        last[ax] = P - 1
        out[tuple(last)] = 0.0  # index P-1 is never written by the reference
        return out
    nx, ny, nz = fine_dims
    x = axis(c, nx, 0)
    y = axis(x, ny, 1)
    return axis(y, nz, 2)


def restrict_planes(R, Lf, Lc, c1, c2):
    """27-point full weighting (CpuSolver.cpp:215-235, ii outermost) of fine array R onto global coarse
    planes c1..c2 (interior x / y): returns shape (ncx, ncy, c2-c1+1)."""
    ncx, ncy = Lc.nx, Lc.ny
    out = np.zeros((ncx, ncy, c2 - c1 + 1))
    X = 2 * np.arange(1, ncx + 1)
    Y = 2 * np.arange(1, ncy + 1)
    Z = np.array([Lf.idx(2 * cz) for cz in range(c1, c2 + 1)])
    for ii in (-1, 0, 1):
        for jj in (-1, 0, 1):
            for kk in (-1, 0, 1):
                w = 0.125 * ((2.0 - abs(ii)) / 2.0) * ((2.0 - abs(jj)) / 2.0) * ((2.0 - abs(kk)) / 2.0)
                out = out + w * R[np.ix_(X + ii, Y + jj, Z + kk)]
    return out


class Rank:
    def __init__(self, params, rank, world, min_points):
        self.p = params
        self.rank, self.world = rank, world
        pl = plan(params.gridDim, world, min_points)
        dims = level_dims(params.gridDim, len(pl))
        self.levels = [Level(dims[l], *pl[l], rank) for l in range(len(pl))]
        self.partial = 0.0
        self.history = []
        self.mode, self.gamma = params.mode, params.gamma
        self.newton_history, self._newton_norm = [], False
        self.bmode = False  # the schedule computes GS_NEWTON_B factors (bfac ops)

    # ---- communication (gloo) ----
    def halo(self, L, name, depth):
        a = self.fields(L, name)
        reqs, recv = [], {}
        if self.rank > 0:
            send = np.ascontiguousarray(a[:, :, L.idx(L.lo): L.idx(L.lo) + depth])
            reqs.append(dist.isend(torch.from_numpy(send), self.rank - 1))
            recv["lo"] = torch.empty(send.shape, dtype=torch.float64)
            reqs.append(dist.irecv(recv["lo"], self.rank - 1))
        if self.rank + 1 < self.world:
            send = np.ascontiguousarray(a[:, :, L.idx(L.hi) - depth + 1: L.idx(L.hi) + 1])
            reqs.append(dist.isend(torch.from_numpy(send), self.rank + 1))
            recv["hi"] = torch.empty(send.shape, dtype=torch.float64)
            reqs.append(dist.irecv(recv["hi"], self.rank + 1))
        for r in reqs:
            r.wait()
        if "lo" in recv:
            a[:, :, L.idx(L.lo) - depth: L.idx(L.lo)] = recv["lo"].numpy()
        if "hi" in recv:
            a[:, :, L.idx(L.hi) + 1: L.idx(L.hi) + 1 + depth] = recv["hi"].numpy()

    def gather(self, L, name):
        a = self.fields(L, name)
        for q in range(self.world):
            lo, hi = L.lo_all[q], L.hi_all[q]
            if hi < lo:
                continue
            t = torch.from_numpy(np.ascontiguousarray(a[:, :, L.idx(lo): L.idx(hi) + 1]))
            dist.broadcast(t, q)
            a[:, :, L.idx(lo): L.idx(hi) + 1] = t.numpy()

    def norm(self, allgather):
        if allgather:
            parts = [torch.zeros(1, dtype=torch.float64) for _ in range(self.world)]
            dist.all_gather(parts, torch.tensor([self.partial], dtype=torch.float64))
            total = 0.0
            for t in parts:  # rank order, as HipSolver::finishNorm
                total += t.item()
        else:
            total = self.partial
        self.partial = 0.0
        self.history.append(float(np.sqrt(total)))
        if self._newton_norm:  # the norm of a newtonF pass: NewtonSolver's own residual
            self.newton_history.append(self.history[-1])
            self._newton_norm = False

    def fields(self, L, name):
        return L.fields[name]

    # ---- ops ----
    def v_in(self, L, vzero):
        return np.zeros_like(L.fields["v"]) if vzero else L.fields["v"]

    def w_of(self, L):
        """The linearisation point the smoothing kernels read: newtonV, or — once the schedule computes the
        GS_NEWTON_B factors ("bfac") — the newtonV that level's factor was computed from (its snapshot at the
        bfac op; a schedule that lets newtonV change without recomputing the factor replays the stale point)."""
        if not self.bmode:
            return L.fields["newtonV"]
        return L.fields["bfacW"]

    def sw(self, L):
        return dict(mode=self.mode, W=self.w_of(L), gamma=self.gamma)

    def op_pair(self, L, z1, z2, zlo, zhi, vzero, norm, V=None):
        g1, g2 = L.local_to_global(z1), L.local_to_global(z2)
        V = self.v_in(L, vzero) if V is None else V
        F = L.fields["f"]
        om = self.p.omega
        # sweep 1 on g1-1 .. g2+1: planes outside the range are computed only on an internal side
        gp = list(range(g1 - 1, g2 + 2))
        keep = lambda g: (g == g1 - 1 and not zlo) or (g == g2 + 1 and not zhi)  # noqa: E731
        S1, r = sweep_planes(V, F, gp, L, om, keep, **self.sw(L))
        if norm:
            self.partial += float(np.sum(r[:, :, 1:-1] ** 2))
        W = V.copy()
        for j, g in enumerate(gp):
            W[:, :, L.idx(g)] = S1[:, :, j]
        S2, _ = sweep_planes(W, F, list(range(g1, g2 + 1)), L, om, **self.sw(L))
        out = L.fields["vAlt"]
        out[1:-1, 1:-1, L.idx(g1): L.idx(g2) + 1] = S2[1:-1, 1:-1, :]

    def op_sweep(self, L, z1, z2, vzero, norm):
        g1, g2 = L.local_to_global(z1), L.local_to_global(z2)
        S, r = sweep_planes(self.v_in(L, vzero), L.fields["f"], list(range(g1, g2 + 1)), L, self.p.omega,
                            **self.sw(L))
        if norm:
            self.partial += float(np.sum(r ** 2))
        L.fields["vAlt"][1:-1, 1:-1, L.idx(g1): L.idx(g2) + 1] = S[1:-1, 1:-1, :]

    def correction(self, Lf, Lc, garr):
        """e = P(v^2h) at fine global planes garr (padded cross-sections), from this rank's coarse array
        (planes it does not hold are NaN)."""
        c = np.full((Lc.nx + 2, Lc.ny + 2, Lc.nz + 2), np.nan)
        V = Lc.fields["v"]
        for g in range(0, Lc.nz + 2):
            k = Lc.idx(g)
            if 0 <= k < V.shape[2]:
                c[:, :, g] = V[:, :, k]
        c[:, :, 0] = 0.0
        c[:, :, Lc.nz + 1] = 0.0
        e = prolong_full(c, (Lf.nx, Lf.ny, Lf.nz))
        return e[:, :, garr]

    def op_pro(self, L, Lc, z1, z2, zlo, zhi):
        g1, g2 = L.local_to_global(z1), L.local_to_global(z2)
        V = L.fields["v"].copy()
        gs_ = [g for g in range(g1 - 2, g2 + 3) if 1 <= g <= L.nz]  # corrected: interior global planes
        e = self.correction(L, Lc, gs_)
        for j, g in enumerate(gs_):
            V[1:-1, 1:-1, L.idx(g)] = V[1:-1, 1:-1, L.idx(g)] + e[1:-1, 1:-1, j]
        self.op_pair(L, z1, z2, zlo, zhi, 0, 0, V=V)

    def op_prolongadd(self, L, Lc):
        gs_ = list(range(L.lo, L.hi + 1))
        e = self.correction(L, Lc, gs_)
        V = L.fields["v"]
        for j, g in enumerate(gs_):
            V[1:-1, 1:-1, L.idx(g)] = V[1:-1, 1:-1, L.idx(g)] + e[1:-1, 1:-1, j]

    def residual_planes(self, L, gplanes):
        """r = f - A v at global planes gplanes (0 outside the level's interior planes)."""
        hh = L.h * L.h
        R = np.zeros((L.nx + 2, L.ny + 2, len(gplanes)))
        inner = [j for j, g in enumerate(gplanes) if 1 <= g <= L.nz]
        if inner:
            zi = np.array([L.idx(gplanes[j]) for j in inner])
            a, _, _ = operator(L.fields["v"], zi, L, self.mode, self.w_of(L), self.gamma)
            R[1:-1, 1:-1, inner] = L.fields["f"][1:-1, 1:-1, zi] - a
        return R

    def op_resrestrict(self, L, Lc, c1, c2):
        gplanes = list(range(2 * c1 - 1, 2 * c2 + 2))
        R = np.zeros_like(L.fields["v"])
        Rp = self.residual_planes(L, gplanes)
        for j, g in enumerate(gplanes):
            R[:, :, L.idx(g)] = Rp[:, :, j]
        Lc.fields["f"][1:-1, 1:-1, Lc.idx(c1): Lc.idx(c2) + 1] = restrict_planes(R, L, Lc, c1, c2)

    def op_residual(self, L, store, norm):
        gplanes = list(range(L.lo, L.hi + 1))
        Rp = self.residual_planes(L, gplanes)
        if norm:
            self.partial += float(np.sum(Rp[1:-1, 1:-1, :] ** 2))
        if store:
            L.fields["r"][:, :, L.idx(L.lo): L.idx(L.hi) + 1] = Rp

    def op_restrict(self, L, Lc, src, dsts, c1, c2):
        out = restrict_planes(L.fields[src], L, Lc, c1, c2)
        for d in dsts:
            Lc.fields[d][1:-1, 1:-1, Lc.idx(c1): Lc.idx(c2) + 1] = out

    def op_coarse(self, frm, vzero):
        """gs_coarse_cycle: CpuSolver::vcycle's recursion below level `frm` on replicated levels, with
        the oracle's operators (bit-identical to the per-operator path, tests/test_gpu_coarse.py)."""
        p = self.p
        nl = len(self.levels)

        def arr(L, name):  # global planes 0 .. nz+1
            return np.ascontiguousarray(L.fields[name][:, :, 1: L.nz + 3])

        def put(L, name, a):
            L.fields[name][:, :, 1: L.nz + 3] = a

        vs = {}

        m, g = self.mode, self.gamma

        def vc(l, v):
            L = self.levels[l]
            f = arr(L, "f")
            w = (arr(L, "bfacW") if self.bmode else arr(L, "newtonV")) if m == NEWTON else None
            if l == nl - 1:
                return O.jacobi(v, f, L.h, m, p.omega, g, p.preSmoothing + p.postSmoothing, w=w)
            v = O.jacobi(v, f, L.h, m, p.omega, g, p.preSmoothing, w=w) if p.preSmoothing else v
            r, _ = O.residual(v, f, L.h, m, g, w=w)
            C_ = self.levels[l + 1]
            put(C_, "f", O.restrict(r, (C_.nx, C_.ny, C_.nz)))
            vc_ = vc(l + 1, O.zeros(C_.nx, C_.ny, C_.nz))
            vs[l + 1] = vc_
            v = v + O.interpolate(vc_, (L.nx, L.ny, L.nz))
            return O.jacobi(v, f, L.h, m, p.omega, g, p.postSmoothing, w=w) if p.postSmoothing else v

        L0 = self.levels[frm]
        v0 = np.zeros((L0.nx + 2, L0.ny + 2, L0.nz + 2)) if vzero else arr(L0, "v")
        vs[frm] = vc(frm, v0)
        odd = (p.preSmoothing + p.postSmoothing) % 2 == 1  # the kernel leaves odd counts in vAlt
        for l, v in vs.items():
            put(self.levels[l], "vAlt" if odd else "v", v)

    # ---- Newton (NewtonSolver.cpp:48-81, 105-107) ----
    def newton_f(self, L, W, gplanes):
        """f = newtonF - N(W) on planes gplanes (N: the NONLINEAR operator, reference order), + partials."""
        zi = np.array([L.idx(g) for g in gplanes])
        s = stencil_div(W, zi, L.h * L.h)
        w = W[1:-1, 1:-1, zi]
        s = s + self.gamma * w * np.exp(w)
        r = L.fields["newtonF"][1:-1, 1:-1, zi] - s
        L.fields["f"][1:-1, 1:-1, zi] = r
        self.partial += float(np.sum(r ** 2))
        self._newton_norm = True

    def op_newton_update(self, L):
        """gs_newton_F_update: w' = newtonV + v formed wherever compF reads it (owned planes and the ghost
        planes next to them), stored on the owned planes' interior into vAlt; f from w'."""
        g1, g2 = L.lo - 1, L.hi + 1
        W = np.full_like(L.fields["v"], np.nan)
        sl = slice(L.idx(g1), L.idx(g2) + 1)
        W[:, :, sl] = L.fields["newtonV"][:, :, sl] + L.fields["v"][:, :, sl]
        own = slice(L.idx(L.lo), L.idx(L.hi) + 1)
        L.fields["vAlt"][1:-1, 1:-1, own] = W[1:-1, 1:-1, own]
        self.newton_f(L, W, list(range(L.lo, L.hi + 1)))
        return W

    def op_newton_update_restrict(self, L, Lc, W):
        """gs_newton_F_update_restrict (single domain): level 1's newtonV = R(w') in the same pass."""
        Lc.fields["vAlt_newton"] = Lc.fields.get("vAlt_newton", np.zeros_like(Lc.fields["newtonV"]))
        Lc.fields["vAlt_newton"][1:-1, 1:-1, Lc.idx(1): Lc.idx(Lc.nz) + 1] = restrict_planes(W, L, Lc, 1, Lc.nz)

    def run(self, ops):
        Ls = self.levels
        for op, kv in ops:
            L = Ls[kv["L"]] if "L" in kv else None
            if op == "rhs":
                f = O.rhs(L.nx, L.ny, L.nz, self.mode, self.gamma)
                L.fields["f"][:, :, L.idx(L.lo): L.idx(L.hi) + 1] = f[:, :, L.lo: L.hi + 1]
            elif op == "copy":  # f > newtonF (NewtonSolver.cpp:12), the whole local array
                L.fields["newtonF"][:] = L.fields["f"]
            elif op == "newtonF":
                self.newton_f(L, L.fields["newtonV"], list(range(L.lo, L.hi + 1)))
            elif op == "newtonFupdate":
                W = self.op_newton_update(L)
                if kv.get("restrict"):
                    self.op_newton_update_restrict(L, Ls[kv["L"] + 1], W)
                if kv.get("bfac"):  # the next inner solve's factor of this level, from w'
                    self.bmode = True
                    L.fields["bfacW"] = W.copy()
            elif op == "ghostsum":  # a ghost plane of the new newtonV: newtonV + 1.0 v (the axpy's value)
                g = L.local_to_global(kv["plane"])
                L.fields["vAlt"][:, :, L.idx(g)] = L.fields["newtonV"][:, :, L.idx(g)] + 1.0 * L.fields["v"][:, :, L.idx(g)]
            elif op == "swapnewton" and kv["L"] > 0:  # findError takes the fused update's restriction
                L.fields["newtonV"], L.fields["vAlt_newton"] = L.fields["vAlt_newton"], L.fields["newtonV"]
            elif op == "swapnewton":
                L.fields["newtonV"], L.fields["vAlt"] = L.fields["vAlt"], L.fields["newtonV"]
                # the second ghost layer came over from the iterate's buffer: never read as newtonV
                for g in (L.lo - 2, L.hi + 2):
                    L.fields["newtonV"][:, :, L.idx(g)] = np.nan
            elif op == "axpy":  # newtonV += v over planes 0 .. nz+1 of the local array
                sl = slice(L.idx(L.lo - 1), L.idx(L.hi + 1) + 1)
                L.fields["newtonV"][:, :, sl] = L.fields["newtonV"][:, :, sl] + 1.0 * L.fields["v"][:, :, sl]
            elif op == "nonorm":  # the last inner cycle's unread closing norm, not computed
                pass
            elif op == "bfac":  # gs_newton_bfac: the level's GS_NEWTON_B factor from its current newtonV
                self.bmode = True
                L.fields["bfacW"] = L.fields["newtonV"].copy()
            elif op == "halo":
                self.halo(L, kv["field"], kv["depth"])
            elif op == "gather":
                self.gather(L, kv["field"])
            elif op == "norm":
                self.norm(kv["allgather"])
            elif op == "pair":
                self.op_pair(L, kv["z1"], kv["z2"], kv["zlo"], kv["zhi"], kv["vzero"], kv["norm"])
            elif op == "sweep":
                self.op_sweep(L, kv["z1"], kv["z2"], kv["vzero"], kv["norm"])
            elif op == "pro":
                self.op_pro(L, Ls[kv["L"] + 1], kv["z1"], kv["z2"], kv["zlo"], kv["zhi"])
            elif op == "prolongadd":
                assert not kv["sub"]
                self.op_prolongadd(L, Ls[kv["L"] + 1])
            elif op == "swap":
                L.fields["v"], L.fields["vAlt"] = L.fields["vAlt"], L.fields["v"]
            elif op == "zero":
                L.fields[kv["field"]][:] = 0.0
            elif op == "resrestrict":
                self.op_resrestrict(L, Ls[kv["L"] + 1], kv["c1"], kv["c2"])
            elif op == "residual":
                self.op_residual(L, kv["store"], kv["norm"])
            elif op == "restrict":
                src, dsts = kv["field"].split(">")
                self.op_restrict(L, Ls[kv["L"] + 1], src, dsts.split(","), kv["c1"], kv["c2"])
            elif op == "coarse":
                self.op_coarse(kv["from"], kv["vzero"])
            elif op == "tiledpre":
                # gs_smooth2_restrict_tiled on a replicated level: the pair into vAlt, then the residual of
                # that result restricted onto every coarse plane
                C_ = Ls[kv["L"] + 1]
                self.op_pair(L, 1, L.nz, 0, 0, kv["vzero"], 0)
                L.fields["v"], L.fields["vAlt"] = L.fields["vAlt"], L.fields["v"]
                self.op_resrestrict(L, C_, 1, C_.nz)
                L.fields["v"], L.fields["vAlt"] = L.fields["vAlt"], L.fields["v"]
            elif op == "tiledpro":
                # gs_prolong_smooth2_tiled: v + P v^2h and two sweeps into vAlt
                self.op_pro(L, Ls[kv["L"] + 1], 1, L.nz, 0, 0)
            else:
                raise NotImplementedError(op)

    def owned_v(self, name="v"):
        L = self.levels[0]
        return L.lo, L.hi, L.fields[name][:, :, L.idx(L.lo): L.idx(L.hi) + 1].copy()
