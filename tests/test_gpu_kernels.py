"""HIP kernels (libgpusolve_hip.so, called through the thin C ABI) vs the reference's own operator
outputs (tests/golden/ops.npz, produced by oracle/_ref/ref_probe) and vs the pinned CPU oracle on
seeded random fields.

Tolerances: LINEAR-mode fields must be bit-identical (the library is built with -ffp-contract=off
and keeps the reference's evaluation order). In NONLINEAR / NEWTON modes ocml's exp may differ
from glibc's by an ulp, so fields must agree to 1e-12 relative to the field's max magnitude.
l2 norms: 1e-12 relative (summation order differs)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402
import oracle as O  # noqa: E402
from conftest import rel  # noqa: E402

K = None


def k():
    global K
    if K is None:
        assert torch.cuda.is_available(), "GPU tests need a GPU (no CPU fallback exists)"
        K = gsv.kernels()
    return K


def stream():
    return torch.cuda.current_stream().cuda_stream


def ok(rc):
    assert rc == 0, k().gs_strerror(rc).decode()


def S_abi(values=(6, -1, -1, -1, -1, -1, -1), offsets=gsv.CANONICAL_OFFSETS):
    return gsv.Stencil(list(values), list(offsets)).to_abi()


def dev(arr):
    nx, ny, nz = (s - 2 for s in arr.shape)
    return DevField(nx, ny, nz).from_xyz(arr)


def assert_field(got, ref, mode, key=""):
    if mode == gsv.GS_LINEAR:
        np.testing.assert_array_equal(got, ref, err_msg=key)
    else:
        scale = max(np.abs(ref).max(), 1e-300)
        assert np.abs(got - ref).max() <= 1e-12 * scale, (key, np.abs(got - ref).max(), scale)


def residual_norm(S, L, mode, gamma, v, f, w, r=None):
    n = k().gs_residual_num_partials(C.byref(S), C.byref(L))
    parts = torch.zeros(max(n, 1), dtype=torch.float64, device="cuda")
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    ok(k().gs_residual(C.byref(S), C.byref(L), mode, gamma, v.ptr, f.ptr, w.ptr if w else None,
                       r.ptr if r else None, parts.data_ptr(), stream()))
    ok(k().gs_sumsq_finish(parts.data_ptr(), n, out.data_ptr(), 0, stream()))
    return out.item()


def lvl_dims(dims, lvl):
    d = list(dims)
    for _ in range(lvl):
        d = [x // 2 for x in d]
    return d


def _fixture(ops_arrays, key):
    return {kk.split("/", 1)[1]: v for kk, v in ops_arrays.items() if kk.split("/", 1)[0] == key}


def test_ops_vs_reference_fixtures(ops_meta, ops_arrays):
    S = S_abi()
    done = 0
    for key, info in ops_meta.items():
        a = _fixture(ops_arrays, key)
        name, mode, lvl = info["name"], info["mode"], info["level"]
        dims = lvl_dims(info["dims"], lvl)
        h = 1.0 / (dims[1] + 1)
        extra = info["extra"]
        omega, gamma, nsw = (float(extra[0]), float(extra[1]), int(extra[2])) if extra else (0.8, 1.0, 1)
        if name == "residual":
            v, f, w = dev(a["v"]), dev(a["f"]), dev(a["newtonV"])
            r = DevField(*dims)
            L = v.level(h)
            n = residual_norm(S, L, mode, gamma, v, f, w, r)
            assert_field(r.to_xyz(), a["r"], mode, key)
            assert rel(n, info["norm"]) < 1e-12, key
        elif name == "jacobi":
            v, f, w = dev(a["v"]), dev(a["f"]), dev(a["newtonV"])
            alt = DevField(*dims)
            L = v.level(h)
            for _ in range(nsw):
                ok(k().gs_jacobi_sweep(C.byref(S), C.byref(L), mode, omega, gamma, v.ptr, alt.ptr, f.ptr, w.ptr,
                                       stream()))
                v, alt = alt, v
            assert_field(v.to_xyz(), a["v_out"], mode, key)
        elif name == "restrict":
            fine = dev(a["fine"])
            cd = lvl_dims(info["dims"], lvl + 1)
            c = DevField(*cd)
            ok(k().gs_restrict(fine.ptr, C.byref(fine.level(h)), c.ptr, C.byref(c.level(1.0 / (cd[1] + 1))),
                               stream()))
            np.testing.assert_array_equal(c.to_xyz(), a["coarse"], err_msg=key)
        elif name == "interpolate":
            c = dev(a["coarse"])
            e = DevField(*dims, fill=np.nan)
            ok(k().gs_interpolate(c.ptr, C.byref(c.level(0.5)), e.ptr, C.byref(e.level(h)), stream()))
            np.testing.assert_array_equal(e.to_xyz(), a["e"], err_msg=key)
            # fused form: v += P(c) on the interior equals interpolate + whole-array +=
            base = np.random.default_rng(1).uniform(-1, 1, a["e"].shape)
            base[0, :, :] = base[-1, :, :] = base[:, 0, :] = base[:, -1, :] = base[:, :, 0] = base[:, :, -1] = 0
            v = dev(base)
            ok(k().gs_prolong_add(c.ptr, None, C.byref(c.level(0.5)), v.ptr, C.byref(v.level(h)), stream()))
            np.testing.assert_array_equal(v.to_xyz(), base + a["e"], err_msg=key)
        elif name == "applyStencil":
            u = dev(a["u"])
            out = DevField(*dims)
            ok(k().gs_apply_op(C.byref(S), C.byref(u.level(h)), gamma, u.ptr, out.ptr, stream()))
            assert_field(out.to_xyz(), a["r"], gsv.GS_NONLINEAR, key)
        elif name == "compF":
            w, F = dev(a["newtonV"]), dev(a["newtonF"])
            f = DevField(*dims)
            L = w.level(h)
            nparts = k().gs_residual_num_partials(C.byref(S), C.byref(L))
            parts = torch.zeros(nparts, dtype=torch.float64, device="cuda")
            out = torch.zeros(1, dtype=torch.float64, device="cuda")
            ok(k().gs_newton_F(C.byref(S), C.byref(L), gamma, w.ptr, F.ptr, f.ptr, parts.data_ptr(), stream()))
            ok(k().gs_sumsq_finish(parts.data_ptr(), nparts, out.data_ptr(), 0, stream()))
            assert_field(f.to_xyz()[1:-1, 1:-1, 1:-1], a["f"][1:-1, 1:-1, 1:-1], gsv.GS_NEWTON, key)
            assert rel(out.item(), info["norm"]) < 1e-12
        elif name == "vcycle":
            p = gsv.GridParams(maxiter=1, gridDim=tuple(info["dims"]), mode=mode)
            with gsv.HipGridData(p) as g:
                for l in range(g.numLevels()):
                    if mode == gsv.GS_NEWTON:
                        g.set_field(l, "newtonV", a[f"newtonV{l}"])
                g.set_field(0, "v", a["v"])
                assert_field(g.field(0, "f"), a["f"], mode, key + "/rhs")
                n = gsv.HipSolver.vcycle(g)
                assert_field(g.field(0, "v"), a["v_out"], mode, key)
                assert rel(n, info["norm"]) < 1e-11, key
        else:
            raise AssertionError(name)
        done += 1
    assert done == len(ops_meta)


def test_rhs_vs_reference(rhs_arrays):
    for key, ref in rhs_arrays.items():
        _, dims, m, gm = key.split("_")
        nx, ny, nz = (int(x) for x in dims.split("x"))
        f = DevField(nx, ny, nz)
        ok(k().gs_rhs_init(C.byref(f.level(1.0 / (ny + 1))), f.ptr, int(m[1:]), 1.0 / (ny + 1), float(gm[1:]),
                           stream()))
        assert_field(f.to_xyz(), ref, int(m[1:]), key)


# --- seeded random grids vs the oracle: shapes that exercise every tile edge of the kernels ----
SHAPES = [(1, 1, 1), (2, 3, 1), (5, 4, 33), (127, 5, 3), (128, 4, 32), (129, 9, 65), (130, 7, 31), (257, 3, 2),
          (64, 64, 64), (33, 100, 40)]


def rand_field(rng, nx, ny, nz, scale=1.0):
    a = np.zeros((nx + 2, ny + 2, nz + 2))
    a[1:-1, 1:-1, 1:-1] = rng.uniform(-scale, scale, (nx, ny, nz))
    return a


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_sweep_and_residual_random(shape, mode):
    rng = np.random.default_rng(hash((shape, mode)) & 0xFFFF)
    nx, ny, nz = shape
    h = 1.0 / (ny + 1)
    v0, f0, w0 = (rand_field(rng, *shape) for _ in range(3))
    f0 *= 100.0
    S = S_abi()
    # two fused sweeps
    v, f, w, alt = dev(v0), dev(f0), dev(w0), DevField(*shape)
    L = v.level(h)
    for _ in range(2):
        ok(k().gs_jacobi_sweep(C.byref(S), C.byref(L), mode, 0.8, 1.0, v.ptr, alt.ptr, f.ptr, w.ptr, stream()))
        v, alt = alt, v
    ref = O.jacobi(v0, f0, h, mode, 0.8, 1.0, 2, w=w0)
    assert_field(v.to_xyz(), ref, mode, f"sweep {shape} m{mode}")
    # residual + norm
    r = DevField(*shape)
    n = residual_norm(S, L, mode, 1.0, dev(v0), f, w, r)
    rr, nn = O.residual(v0, f0, h, mode, 1.0, w=w0)
    assert_field(r.to_xyz(), rr, mode, f"residual {shape}")
    assert rel(n, nn) < 1e-12


@pytest.mark.parametrize("stencil", [
    ((-1, -1, 6, -1, -1, -1, -1), [(0, 0, 1), (-1, 0, 0), (0, 0, 0), (0, 0, -1), (1, 0, 0), (0, 1, 0), (0, -1, 0)]),
    ((4, -1, -1, -0.5, -0.5, -0.5, -0.5), gsv.CANONICAL_OFFSETS),
    ((8, -1, -1, -1, -1, -2, -2), [(0, 0, 0), (1, 1, 0), (-1, -1, 0), (1, -1, 1), (-1, 1, -1), (0, 1, 1), (0, -1, -1)]),
])
@pytest.mark.parametrize("mode", [0, 1])
def test_generic_and_reordered_stencils(stencil, mode):
    rng = np.random.default_rng(7)
    shape = (37, 11, 9)
    h = 1.0 / (shape[1] + 1)
    vals, offs = stencil
    v0, f0 = rand_field(rng, *shape), rand_field(rng, *shape, 50.0)
    S = S_abi(vals, offs)
    So = O.Stencil.make(vals, offs)
    v, f, alt = dev(v0), dev(f0), DevField(*shape)
    L = v.level(h)
    ok(k().gs_jacobi_sweep(C.byref(S), C.byref(L), mode, 0.7, 0.5, v.ptr, alt.ptr, f.ptr, None, stream()))
    ref = O.jacobi(v0, f0, h, mode, 0.7, 0.5, 1, stencil=So)
    assert_field(alt.to_xyz(), ref, mode, "generic sweep")
    r = DevField(*shape)
    n = residual_norm(S, L, mode, 0.5, v, f, None, r)
    rr, nn = O.residual(v0, f0, h, mode, 0.5, stencil=So)
    assert_field(r.to_xyz(), rr, mode, "generic residual")
    assert rel(n, nn) < 1e-12


def test_restrict_prolong_random_shapes():
    rng = np.random.default_rng(3)
    for fd in [(2, 2, 2), (3, 5, 7), (16, 17, 18), (129, 33, 20), (130, 8, 9)]:
        cd = [x // 2 for x in fd]
        fine = rand_field(rng, *fd)
        ref = O.restrict(fine, cd)
        fdev, c = dev(fine), DevField(*cd)
        ok(k().gs_restrict(fdev.ptr, C.byref(fdev.level(0.1)), c.ptr, C.byref(c.level(0.2)), stream()))
        np.testing.assert_array_equal(c.to_xyz(), ref)
        # FAS pair + fused (v_c - restV_c) prolongation
        a2 = DevField(*cd)
        ok(k().gs_restrict2(fdev.ptr, C.byref(fdev.level(0.1)), c.ptr, a2.ptr, C.byref(c.level(0.2)), stream()))
        np.testing.assert_array_equal(a2.to_xyz(), ref)
        coarse = rand_field(rng, *cd)
        sub = rand_field(rng, *cd)
        e_ref = O.interpolate(coarse - sub, fd)
        base = rand_field(rng, *fd)
        v = dev(base)
        cdev, sdev = dev(coarse), dev(sub)
        ok(k().gs_prolong_add(cdev.ptr, sdev.ptr, C.byref(cdev.level(0.2)), v.ptr, C.byref(v.level(0.1)), stream()))
        np.testing.assert_array_equal(v.to_xyz(), base + e_ref)


def test_apply_op_add_and_axpy():
    rng = np.random.default_rng(11)
    shape = (65, 13, 34)
    h = 1.0 / 14
    u0, f0 = rand_field(rng, *shape), rand_field(rng, *shape)
    u, f = dev(u0), dev(f0)
    S = S_abi()
    ok(k().gs_apply_op_add(C.byref(S), C.byref(u.level(h)), 1.0, u.ptr, f.ptr, stream()))
    assert_field(f.to_xyz(), f0 + O.apply_op(u0, h, 1.0), gsv.GS_NONLINEAR)
    y = dev(f0)
    ok(k().gs_axpy(y.ptr, u.ptr, 1.0, y.span, stream()))
    np.testing.assert_array_equal(y.to_xyz(), f0 + u0)
    ok(k().gs_axpy(y.ptr, u.ptr, -1.0, y.span, stream()))
    np.testing.assert_array_equal(y.to_xyz(), (f0 + u0) - u0)


def test_invalid_arguments_fail_loudly():
    S = S_abi(offsets=[(0, 0, 0), (2, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)])
    v = DevField(8, 8, 8)
    L = v.level(1 / 9)
    rc = k().gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, v.ptr, v.ptr, None, stream())
    assert rc == gsv._abi.GS_EINVAL
    S = S_abi()
    rc = k().gs_jacobi_sweep(C.byref(S), C.byref(L), 0, 0.8, 1.0, v.ptr, v.ptr, v.ptr, None, stream())
    assert rc == gsv._abi.GS_EINVAL  # in-place sweep is refused (Jacobi needs ping-pong)
    bad = gsv.gs_level(8, 8, 8, 4, 40, 0, 0.1)  # pitch < nx+2
    rc = k().gs_jacobi_sweep(C.byref(S), C.byref(bad), 0, 0.8, 1.0, v.ptr, DevField(8, 8, 8).ptr, v.ptr, None,
                             stream())
    assert rc == gsv._abi.GS_EINVAL


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("fd", [(2, 2, 2), (3, 5, 7), (16, 17, 18), (129, 33, 20), (130, 8, 9), (255, 10, 33),
                                (64, 64, 64), (511, 9, 10), (512, 6, 5), (1023, 5, 6), (1024, 4, 3), (1100, 3, 4),
                                (127, 2, 70), (258, 66, 1)])
def test_residual_restrict_fused(fd, mode):
    """gs_residual_restrict == gs_residual + gs_restrict2 bit for bit (and == the oracle's restrict of
    the oracle's residual, to the mode's tolerance); odd and even fine extents, partial tiles."""
    rng = np.random.default_rng(sum(fd) * 3 + mode)
    cd = [x // 2 for x in fd]
    h = 1.0 / (fd[1] + 1)
    v0, f0, w0 = rand_field(rng, *fd), rand_field(rng, *fd, 100.0), rand_field(rng, *fd)
    S = S_abi((6, -1, -1.5, -1, -0.5, -1, -1))
    v, f, w = dev(v0), dev(f0), dev(w0)
    L = v.level(h)
    r = DevField(*fd)
    r.buf.zero_()
    ok(k().gs_residual(C.byref(S), C.byref(L), mode, 0.7, v.ptr, f.ptr, w.ptr, r.ptr, None, stream()))
    ca_ref, ca, cb = DevField(*cd), DevField(*cd), DevField(*cd)
    Lc = ca.level(2 * h)
    ok(k().gs_restrict2(r.ptr, C.byref(r.level(h)), ca_ref.ptr, None, C.byref(Lc), stream()))
    ok(k().gs_residual_restrict(C.byref(S), C.byref(L), mode, 0.7, v.ptr, f.ptr, w.ptr, ca.ptr, cb.ptr,
                                C.byref(Lc), stream()))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ca.to_xyz(), ca_ref.to_xyz())
    np.testing.assert_array_equal(cb.to_xyz(), ca_ref.to_xyz())
    rr, _ = O.residual(v0, f0, h, mode, 0.7, w=w0,
                       stencil=O.Stencil.make((6, -1, -1.5, -1, -0.5, -1, -1), gsv.CANONICAL_OFFSETS))
    assert_field(ca.to_xyz(), O.restrict(rr, cd), mode, f"rr {fd} m{mode}")


def test_residual_restrict_fused_two_rows_per_block():
    """A LINEAR level of >= 2^26 points takes k_rr2's two-coarse-rows-per-block shape: still bit-identical
    to gs_residual + gs_restrict2; odd coarse ny (the last block's second row is outside the level)."""
    fd = (511, 515, 256)
    assert fd[0] * fd[1] * fd[2] >= 1 << 26
    cd = [x // 2 for x in fd]
    h = 1.0 / (fd[1] + 1)
    g = torch.Generator(device="cuda").manual_seed(11)
    v, f = DevField(*fd), DevField(*fd)
    for fld, scale in ((v, 1.0), (f, 100.0)):
        inner = fld.zyx[1:-1, 1:-1, 1:fd[0] + 1]
        inner.copy_((torch.rand(inner.shape, generator=g, device="cuda", dtype=torch.float64) - 0.5) * scale)
    S = S_abi((6, -1, -1.5, -1, -0.5, -1, -1))
    L = v.level(h)
    r = DevField(*fd)
    r.buf.zero_()
    ok(k().gs_residual(C.byref(S), C.byref(L), 0, 0.0, v.ptr, f.ptr, None, r.ptr, None, stream()))
    ca_ref, ca = DevField(*cd), DevField(*cd)
    Lc = ca.level(2 * h)
    ok(k().gs_restrict2(r.ptr, C.byref(r.level(h)), ca_ref.ptr, None, C.byref(Lc), stream()))
    ok(k().gs_residual_restrict(C.byref(S), C.byref(L), 0, 0.0, v.ptr, f.ptr, None, ca.ptr, None, C.byref(Lc),
                                stream()))
    torch.cuda.synchronize()
    assert torch.equal(ca.buf, ca_ref.buf)


def test_residual_restrict_generic_stencil():
    rng = np.random.default_rng(11)
    fd = (37, 11, 9)
    cd = [x // 2 for x in fd]
    vals = (8, -1, -1, -1, -1, -2, -2)
    offs = [(0, 0, 0), (1, 1, 0), (-1, -1, 0), (1, -1, 1), (-1, 1, -1), (0, 1, 1), (0, -1, -1)]
    v0, f0 = rand_field(rng, *fd), rand_field(rng, *fd, 50.0)
    S = S_abi(vals, offs)
    v, f, ca = dev(v0), dev(f0), DevField(*cd)
    ok(k().gs_residual_restrict(C.byref(S), C.byref(v.level(0.1)), 0, 0.5, v.ptr, f.ptr, None, ca.ptr, None,
                                C.byref(ca.level(0.2)), stream()))
    rr, _ = O.residual(v0, f0, 0.1, 0, 0.5, stencil=O.Stencil.make(vals, offs))
    np.testing.assert_array_equal(ca.to_xyz(), O.restrict(rr, cd))


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("fd,m", [((64, 33, 40), 20), ((129, 17, 30), 14), ((512, 6, 12), 6), ((33, 9, 41), 10)])
def test_residual_restrict_slab_top_ghost(fd, m, mode):
    """gs_residual_restrict_slab on the lower slab (local planes 1..m, m even) of a grid, zhi = 1: its
    top ghost planes m+1, m+2 are the grid's own planes, so its coarse planes 1..m/2 must equal the
    whole grid's gs_residual_restrict bit for bit (with zhi = 0 the top fine plane reads as a level
    boundary instead)."""
    rng = np.random.default_rng(sum(fd) + m + 7 * mode)
    cd = [x // 2 for x in fd]
    h = 1.0 / (fd[1] + 1)
    v0, f0, w0 = rand_field(rng, *fd), rand_field(rng, *fd, 100.0), rand_field(rng, *fd)
    S = S_abi()
    v, f, w = dev(v0), dev(f0), dev(w0)
    L = v.level(h)
    ref, got = DevField(*cd), DevField(*cd)
    Lc = ref.level(2 * h)
    ok(k().gs_residual_restrict(C.byref(S), C.byref(L), mode, 0.7, v.ptr, f.ptr, w.ptr, ref.ptr, None, C.byref(Lc),
                                stream()))
    Ls = gsv.gs_level(L.nx, L.ny, m, L.ldy, L.ldz, 0, L.h)
    Lcs = gsv.gs_level(Lc.nx, Lc.ny, m // 2, Lc.ldy, Lc.ldz, 0, Lc.h)
    assert k().gs_residual_restrict_slab_supported(C.byref(S), C.byref(Ls)) == 1
    ok(k().gs_residual_restrict_slab(C.byref(S), C.byref(Ls), mode, 0.7, v.ptr, f.ptr, w.ptr, got.ptr, None,
                                     C.byref(Lcs), 1, stream()))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.to_xyz()[:, :, 1:m // 2 + 1], ref.to_xyz()[:, :, 1:m // 2 + 1])
    # not supported for a generic stencil order
    G = S_abi((6, -1, -1, -1, -1, -1, -1), [(0, 0, 0), (-1, 0, 0), (1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1),
                                            (0, 0, -1)])
    assert k().gs_residual_restrict_slab(C.byref(G), C.byref(Ls), mode, 0.7, v.ptr, f.ptr, w.ptr, got.ptr, None,
                                         C.byref(Lcs), 1, stream()) == gsv._abi.GS_EINVAL
