"""The fused two-sweep kernel (gs_jacobi_sweep2, temporal blocking) against two single fused
sweeps (gs_jacobi_sweep) — bit for bit in every mode — on shapes that exercise every tile edge:
single-wave and multi-wave rows (LDS edge exchange), both wave shapes (rows <= 512 and <= 1024),
ragged y / z tiles, and Z-slabs with internal boundaries on one or both sides (two ghost planes)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
from gpusolve.devfield import DevField  # noqa: E402


def k():
    assert torch.cuda.is_available()
    return gsv.kernels()


def st():
    return torch.cuda.current_stream().cuda_stream


def ok(rc):
    assert rc == 0, k().gs_strerror(rc).decode()


S = None


def stencil():
    global S
    if S is None:
        S = gsv.Stencil().to_abi()
    return S


def rand_full(rng, nx, ny, nz, scale=1.0, extra=0):
    a = np.zeros((nx + 2, ny + 2, nz + 2 + 2 * extra))
    a[1:nx + 1, 1:ny + 1, 1 + extra: nz + 1 + extra] = rng.uniform(-scale, scale, (nx, ny, nz))
    return a


def two_sweeps(v0, f0, w0, mode, h):
    nx, ny, nz = (s - 2 for s in v0.shape)
    v, f, w, alt = DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0), \
        DevField(nx, ny, nz).from_xyz(w0), DevField(nx, ny, nz)
    L = v.level(h)
    for _ in range(2):
        ok(k().gs_jacobi_sweep(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v.ptr, alt.ptr, f.ptr, w.ptr, st()))
        v, alt = alt, v
    return v.to_xyz()


SHAPES = [(1, 1, 1), (2, 5, 3), (5, 4, 33), (127, 9, 17), (128, 8, 8), (129, 13, 40), (257, 6, 10), (500, 7, 9),
          (512, 4, 5), (513, 5, 6), (1024, 3, 4), (64, 64, 64), (200, 33, 70),
          # rows > 512 points: column blocks (k_tb2y XH) in every mode (NEWTON rows of 513-1024 points since r04;
          # GS_NEWTON_XH=0 keeps k_tb2 for them, tests/test_gpu_switches.py)
          (700, 9, 11), (1024, 16, 12), (1025, 7, 9), (1536, 5, 6), (2000, 3, 5)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_sweep2_equals_two_sweeps(shape, mode):
    rng = np.random.default_rng(abs(hash((shape, mode))) % 2**32)
    nx, ny, nz = shape
    h = 1.0 / (ny + 1)
    v0, f0, w0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0), rand_full(rng, *shape)
    ref = two_sweeps(v0, f0, w0, mode, h)
    v, f, w, out = (DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0),
                    DevField(nx, ny, nz).from_xyz(w0), DevField(nx, ny, nz))
    L = v.level(h)
    assert k().gs_jacobi_sweep2_supported_mode(C.byref(stencil()), C.byref(L), mode) >= 1
    ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v.ptr, out.ptr, f.ptr, w.ptr, 0, 0, st()))
    np.testing.assert_array_equal(out.to_xyz(), ref)


@pytest.mark.parametrize("nx", [128, 512])
def test_sweep2_extreme_magnitudes(nx):
    """Whole-row LINEAR pairs test the fast h^2 division's range with floating-point compares (r06, div_hh_n FPC), the
    single sweep with the exponent field: fields whose stencil sums straddle both ends of that range (2^-899, 2^601),
    zeros, denormals and overflow must come out the same — bit for bit, NaNs as NaNs."""
    rng = np.random.default_rng(nx)
    shape = (nx, 6, 7)
    mags = np.array([0.0, 5e-324, 1e-310, 1e-280, 1e-272, 1.3e-271, 1e-270, 1e-200, 1.0, 1e100, 1e180, 4e180, 5e180,
                     1e200, 1e300])

    def field():
        a = rand_full(rng, *shape)
        inner = a[1:nx + 1, 1:7, 1:8]
        inner[...] = np.sign(inner) * rng.choice(mags, inner.shape) * rng.uniform(0.5, 2.0, inner.shape)
        return a

    h = 1.0 / 7
    v0, f0, w0 = field(), field(), rand_full(rng, *shape)
    with np.errstate(all="ignore"):
        ref = two_sweeps(v0, f0, w0, 0, h)
    v, f, w, out = (DevField(*shape).from_xyz(v0), DevField(*shape).from_xyz(f0), DevField(*shape).from_xyz(w0),
                    DevField(*shape))
    L = v.level(h)
    ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), 0, 0.8, 1.0, v.ptr, out.ptr, f.ptr, w.ptr, 0, 0, st()))
    got = out.to_xyz()
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    assert np.array_equal(got[m].view(np.int64), ref[m].view(np.int64))


@pytest.mark.parametrize("nx", [130, 1100])
@pytest.mark.parametrize("lo,hi", [(1, 9), (5, 14), (12, 22), (3, 3), (10, 11)])
@pytest.mark.parametrize("mode", [0, 2])
def test_sweep2_on_slab_with_two_ghost_planes(lo, hi, mode, nx):
    rng = np.random.default_rng(lo * 100 + hi)
    ny, NZ = 11, 22
    h = 1.0 / (ny + 1)
    v0, f0, w0 = rand_full(rng, nx, ny, NZ), rand_full(rng, nx, ny, NZ, 100.0), rand_full(rng, nx, ny, NZ)
    ref = two_sweeps(v0, f0, w0, mode, h)
    nzl = hi - lo + 1

    def slab(a):  # global planes lo-2 .. hi+2 (clamped to the allocation: planes outside are zero)
        out = np.zeros((nx + 2, ny + 2, nzl + 4))
        for k_ in range(nzl + 4):
            g = lo - 2 + k_
            if 0 <= g <= NZ + 1:
                out[:, :, k_] = a[:, :, g]
        return out

    v, f, w, out = (DevField(nx, ny, nzl).from_xyz_ext(slab(v0)), DevField(nx, ny, nzl).from_xyz_ext(slab(f0)),
                    DevField(nx, ny, nzl).from_xyz_ext(slab(w0)), DevField(nx, ny, nzl))
    L = v.level(h, lo - 1)
    zlo, zhi = int(lo > 1), int(hi < NZ)
    ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v.ptr, out.ptr, f.ptr, w.ptr, zlo, zhi,
                            st()))
    got = out.to_xyz()
    np.testing.assert_array_equal(got[:, :, 1:nzl + 1], ref[:, :, lo:hi + 1])


def test_sweep2_rejects_unsupported():
    v = DevField(1030, 3, 4)
    L = v.level(0.25)
    # rows > 1024 points: column blocks in every mode (NEWTON since r03)
    assert k().gs_jacobi_sweep2_supported(C.byref(stencil()), C.byref(L)) >= 1
    for mode in (0, 1, 2):
        assert k().gs_jacobi_sweep2_supported_mode(C.byref(stencil()), C.byref(L), mode) >= 1
        assert "XH" in k().gs_jacobi_sweep2_kernel(C.byref(stencil()), C.byref(L), mode).decode()
    # NEWTON needs newtonV; a non-canonical stencil order has no pair at all
    rc = k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), 2, 0.8, 1.0, v.ptr, DevField(1030, 3, 4).ptr, v.ptr,
                              None, 0, 0, st())
    assert rc == gsv._abi.GS_EINVAL
    perm = gsv.Stencil([6, -1, -1, -1, -1, -1, -1], [gsv.CANONICAL_OFFSETS[i] for i in (0, 2, 1, 3, 4, 5, 6)]).to_abi()
    assert k().gs_jacobi_sweep2_supported(C.byref(perm), C.byref(L)) == 0
    big = DevField(512, 512, 64)
    assert k().gs_jacobi_sweep2_supported(C.byref(stencil()), C.byref(big.level(1 / 513))) == 2


@pytest.mark.parametrize("shape", [(5, 4, 33), (129, 13, 40), (512, 4, 5), (300, 9, 7), (1024, 3, 4), (64, 64, 64),
                                   (1100, 9, 8)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_sweep2_norm_partials(shape, mode):
    """gs_jacobi_sweep2_norm: same output as the plain pair, and its partials sum to ||f - A v_in||^2."""
    rng = np.random.default_rng(sum(shape) * 7 + mode)
    nx, ny, nz = shape
    h = 1.0 / (ny + 1)
    v0, f0, w0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0), rand_full(rng, *shape)
    v, f, w, out, out2 = (DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0),
                          DevField(nx, ny, nz).from_xyz(w0), DevField(nx, ny, nz), DevField(nx, ny, nz))
    L = v.level(h)
    n = k().gs_jacobi_sweep2_num_partials(C.byref(stencil()), C.byref(L), mode)
    assert n >= 1
    parts = torch.full((n,), float("nan"), dtype=torch.float64, device="cuda")
    ok(k().gs_jacobi_sweep2_norm(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v.ptr, out.ptr, f.ptr, w.ptr, 0, 0,
                                 parts.data_ptr(), st()))
    ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v.ptr, out2.ptr, f.ptr, w.ptr, 0, 0, st()))
    np.testing.assert_array_equal(out.to_xyz(), out2.to_xyz())
    nr = k().gs_residual_num_partials(C.byref(stencil()), C.byref(L))
    rparts = torch.zeros((nr,), dtype=torch.float64, device="cuda")
    ok(k().gs_residual(C.byref(stencil()), C.byref(L), mode, 1.0, v.ptr, f.ptr, w.ptr, None, rparts.data_ptr(), st()))
    torch.cuda.synchronize()
    got, want = parts.sum().item(), rparts.sum().item()
    assert np.isfinite(got)
    assert abs(got - want) <= 1e-12 * abs(want)


@pytest.mark.parametrize("shape", [(5, 4, 33), (129, 13, 40), (512, 6, 5), (64, 64, 64), (1024, 6, 5), (1100, 7, 6)])
@pytest.mark.parametrize("mode", [0, 2])
def test_zero_iterate_sweeps(shape, mode):
    """v_in = NULL (the coarse levels' v = 0 after restriction) is bit-identical to a zeroed v_in,
    for the single sweep (with its norm partials) and for the fused pair."""
    rng = np.random.default_rng(sum(shape) + 11 * mode)
    nx, ny, nz = shape
    h = 1.0 / (ny + 1)
    f0, w0 = rand_full(rng, *shape, 100.0), rand_full(rng, *shape)
    zero, f, w = DevField(nx, ny, nz), DevField(nx, ny, nz).from_xyz(f0), DevField(nx, ny, nz).from_xyz(w0)
    a, b = DevField(nx, ny, nz, fill=7.0), DevField(nx, ny, nz, fill=7.0)
    a.from_xyz(np.zeros((nx + 2, ny + 2, nz + 2)))
    b.from_xyz(np.zeros((nx + 2, ny + 2, nz + 2)))
    L = zero.level(h)
    n = k().gs_residual_num_partials(C.byref(stencil()), C.byref(L))
    pa = torch.zeros((n,), dtype=torch.float64, device="cuda")
    pb = torch.zeros((n,), dtype=torch.float64, device="cuda")
    ok(k().gs_jacobi_sweep_norm(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, zero.ptr, a.ptr, f.ptr, w.ptr,
                                pa.data_ptr(), st()))
    ok(k().gs_jacobi_sweep_norm(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, None, b.ptr, f.ptr, w.ptr,
                                pb.data_ptr(), st()))
    np.testing.assert_array_equal(a.to_xyz(), b.to_xyz())
    assert torch.equal(pa, pb)
    if k().gs_jacobi_sweep2_supported_mode(C.byref(stencil()), C.byref(L), mode) >= 1:
        a.from_xyz(np.zeros((nx + 2, ny + 2, nz + 2)))
        b.from_xyz(np.zeros((nx + 2, ny + 2, nz + 2)))
        ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, zero.ptr, a.ptr, f.ptr, w.ptr, 0, 0,
                                st()))
        ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, None, b.ptr, f.ptr, w.ptr, 0, 0,
                                st()))
        np.testing.assert_array_equal(a.to_xyz(), b.to_xyz())


def test_zero_iterate_rejected_in_fas_mode():
    nx = ny = nz = 16
    f, out = DevField(nx, ny, nz), DevField(nx, ny, nz)
    L = f.level(1.0 / 17)
    assert k().gs_jacobi_sweep(C.byref(stencil()), C.byref(L), 1, 0.8, 1.0, None, out.ptr, f.ptr, None, st()) != 0
    assert k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), 1, 0.8, 1.0, None, out.ptr, f.ptr, None, 0, 0,
                                st()) != 0


PRO_SHAPES = [(1, 1, 1), (2, 5, 3), (5, 4, 33), (127, 9, 17), (128, 8, 8), (129, 13, 40), (257, 6, 10),
              (500, 7, 9), (512, 4, 5), (64, 64, 64), (63, 31, 65), (200, 33, 70),
              # rows > 512 points: column blocks (BASELINE config #5's 1024-point rows), edge columns through
              # the workspace; 513 / 1025: a last block of one column
              (513, 5, 6), (700, 9, 11), (1024, 6, 9), (1025, 4, 7), (1100, 13, 5), (1536, 3, 4)]


def prolong_ws(S, L, mode, v, c, sub, Lc, out, f, w, zlo, zhi):
    """gs_jacobi_sweep2_prolong_ws with a workspace of the size the level needs (none for rows <= 512)."""
    n = k().gs_jacobi_sweep2_prolong_ws_elems(C.byref(S), C.byref(L), mode)
    ws = torch.empty(max(n, 1), dtype=torch.float64, device="cuda") if n > 0 else None
    rc = k().gs_jacobi_sweep2_prolong_ws(C.byref(S), C.byref(L), mode, 0.8, 1.0, v, c, sub, C.byref(Lc), out, f, w,
                                         zlo, zhi, ws.data_ptr() if ws is not None else None, n, st())
    torch.cuda.synchronize()
    return rc


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("shape", PRO_SHAPES)
def test_prolong_fused_pair_bit_identical(shape, mode):
    """gs_jacobi_sweep2_prolong == gs_prolong_add then gs_jacobi_sweep2, bit for bit (LINEAR and NEWTON,
    whose newtonV enters both sweeps); odd and even fine extents, partial row tiles and z-chunks."""
    rng = np.random.default_rng(sum(shape) * 13 + mode)
    nx, ny, nz = shape
    cd = [x // 2 for x in shape]
    h = 1.0 / (ny + 1)
    v0, f0, c0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0), rand_full(rng, *[max(c, 0) for c in cd])
    w0 = rand_full(rng, *shape, 0.5)
    L = DevField(nx, ny, nz).level(h)
    supported = k().gs_jacobi_sweep2_prolong_supported(C.byref(stencil()), C.byref(L), mode)
    # the fused prolongation pair exists for every LINEAR and NEWTON shape (NEWTON rows > 512 points: column
    # blocks since r04)
    assert supported == 1, (shape, mode, supported)
    # reference: prolongation + correction stored, then the plain fused pair
    v, f, c, out_ref = (DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0),
                        DevField(*cd).from_xyz(c0), DevField(nx, ny, nz))
    w = DevField(nx, ny, nz).from_xyz(w0) if mode == 2 else None
    wp = w.ptr if w else None
    Lc = c.level(2 * h)
    ok(k().gs_prolong_add(c.ptr, None, C.byref(Lc), v.ptr, C.byref(L), st()))
    ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v.ptr, out_ref.ptr, f.ptr, wp, 0, 0,
                            st()))
    # fused
    v2, out = DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz)
    ok(prolong_ws(stencil(), L, mode, v2.ptr, c.ptr, None, Lc, out.ptr, f.ptr, wp, 0, 0))
    np.testing.assert_array_equal(out.to_xyz(), out_ref.to_xyz())
    if nx > 512:  # the call without a workspace is refused where one is needed
        assert k().gs_jacobi_sweep2_prolong(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v2.ptr, c.ptr, None,
                                            C.byref(Lc), out.ptr, f.ptr, wp, 0, 0, st()) == gsv._abi.GS_EINVAL
    np.testing.assert_array_equal(v2.to_xyz(), v0)  # the input iterate is left as it was


# plane ranges as the Z-slab driver launches them (HipSolver::vcycleSpeculative: bottom pair, top
# planes, interior): odd first planes; an internal range end lies two planes below the top or on it
PRO_SPLITS = [((64, 64, 64), [(1, 2), (63, 64), (3, 62)]),
              ((63, 31, 65), [(1, 2), (63, 65), (3, 62)]),  # odd extent: three top planes
              ((200, 33, 70), [(1, 14), (15, 40), (41, 70)]),
              ((5, 4, 33), [(1, 2), (3, 30), (31, 33)]),
              ((127, 9, 17), [(1, 1), (2, 2), (1, 2), (3, 14), (15, 17), (17, 17)]),  # (2, 2): even start, refused
              # column blocks: config #5's per-rank slab split (bottom pair, top planes, interior)
              ((1024, 7, 24), [(1, 2), (23, 24), (3, 22)]),
              ((700, 11, 19), [(1, 2), (17, 19), (3, 16)]),
              ((1100, 5, 20), [(1, 6), (7, 12), (13, 20)])]


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("coarse_view", [False, True])
@pytest.mark.parametrize("shape,ranges", PRO_SPLITS)
def test_prolong_fused_pair_plane_ranges(shape, ranges, coarse_view, mode):
    """gs_jacobi_sweep2_prolong on plane ranges (z0 > 0, internal sides flagged zlo / zhi, whose
    planes the kernel corrects as it reads them) assembles the whole-level result bit for bit. With
    coarse_view the coarse level is passed as the plane range under the fine one (a Z-slab coarse
    level: coarse z0 = fine z0 / 2, its ghost plane -1 read), else whole (a replicated coarse level).
    LINEAR and NEWTON (newtonV offset with the range like f)."""
    rng = np.random.default_rng(sum(shape) * 7 + coarse_view + 100 * mode)
    nx, ny, nz = shape
    cd = [x // 2 for x in shape]
    h = 1.0 / (ny + 1)
    v0, f0, c0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0), rand_full(rng, *cd)
    L = DevField(nx, ny, nz).level(h)
    v, f, c, out_ref = (DevField(nx, ny, nz).from_xyz(v0), DevField(nx, ny, nz).from_xyz(f0),
                        DevField(*cd).from_xyz(c0), DevField(nx, ny, nz))
    w = DevField(nx, ny, nz).from_xyz(rand_full(rng, *shape, 0.5)) if mode == 2 else None
    Lc = c.level(2 * h)
    ok(prolong_ws(stencil(), L, mode, v.ptr, c.ptr, None, Lc, out_ref.ptr, f.ptr, w.ptr if w else None, 0, 0))
    out = DevField(nx, ny, nz)
    for z1, z2 in ranges:
        off = 8 * (z1 - 1) * L.ldz
        sub = gsv._abi.gs_level(nx, ny, z2 - z1 + 1, L.ldy, L.ldz, z1 - 1, h)
        cptr, cl = c.ptr, Lc
        if coarse_view and z1 % 2 == 1:
            z0c = (z1 - 1) // 2
            cptr = c.ptr + 8 * z0c * Lc.ldz
            cl = gsv._abi.gs_level(Lc.nx, Lc.ny, min((z2 - z1 + 2) // 2, cd[2] - z0c), Lc.ldy, Lc.ldz, z0c, 2 * h)
        rc = prolong_ws(stencil(), sub, mode, v.ptr + off, cptr, None, cl, out.ptr + off, f.ptr + off,
                        w.ptr + off if w else None, int(z1 > 1), int(z2 < nz))
        if z1 % 2 == 0:
            assert rc == gsv._abi.GS_EINVAL  # plane parities must be the global ones
        else:
            ok(rc)
    np.testing.assert_array_equal(out.to_xyz(), out_ref.to_xyz())


def test_prolong_fused_pair_rejects():
    L = DevField(16, 16, 16).level(1 / 17.0)
    assert k().gs_jacobi_sweep2_prolong_supported(C.byref(stencil()), C.byref(L), 1) == 0  # NONLINEAR
    assert k().gs_jacobi_sweep2_prolong_supported(C.byref(stencil()), C.byref(L), 2) == 1  # NEWTON
    f, out, c = DevField(16, 16, 16), DevField(16, 16, 16), DevField(8, 8, 8)
    rc = k().gs_jacobi_sweep2_prolong(C.byref(stencil()), C.byref(L), 2, 0.8, 1.0, f.ptr, c.ptr, None,
                                      C.byref(c.level(1 / 9.0)), out.ptr, f.ptr, None, 0, 0, st())
    assert rc == gsv._abi.GS_EINVAL  # NEWTON needs newtonV
    L2 = DevField(600, 4, 4).level(0.2)
    assert k().gs_jacobi_sweep2_prolong_supported(C.byref(stencil()), C.byref(L2), 0) == 1  # rows > 512: LINEAR
    assert k().gs_jacobi_sweep2_prolong_ws_elems(C.byref(stencil()), C.byref(L2), 0) == 1 * (4 + 4) * 4 * (4 + 2)
    assert k().gs_jacobi_sweep2_prolong_supported(C.byref(stencil()), C.byref(L2), 2) == 1  # NEWTON: column blocks
    assert k().gs_jacobi_sweep2_prolong_ws_elems(C.byref(stencil()), C.byref(L2), 2) == 1 * (4 + 4) * 4 * (4 + 2)
    assert b"XH" in k().gs_jacobi_sweep2_kernel(C.byref(stencil()), C.byref(L2), 2)  # the plain pair too (r04)
    L3 = DevField(512, 4, 4).level(0.2)
    assert k().gs_jacobi_sweep2_prolong_ws_elems(C.byref(stencil()), C.byref(L3), 0) == 0


@pytest.mark.parametrize("mode", [0, 2])
def test_prolong_fused_pair_full_1024_plane_set(mode):
    """Config #5's row length on a full 1024 x 1024 plane set (8 planes): the column-block prolongation pair
    against gs_prolong_add + the plain pair, bit for bit (LINEAR; NEWTON with a newtonV field)."""
    rng = np.random.default_rng(10241 + mode)
    shape = (1024, 1024, 8)
    nx, ny, nz = shape
    cd = [x // 2 for x in shape]
    h = 1.0 / 1025
    v0, f0, c0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0), rand_full(rng, *cd)
    L = DevField(*shape).level(h)
    v, f, c, out_ref = (DevField(*shape).from_xyz(v0), DevField(*shape).from_xyz(f0), DevField(*cd).from_xyz(c0),
                        DevField(*shape))
    w = DevField(*shape).from_xyz(rand_full(rng, *shape, 0.5)) if mode == 2 else None
    wp = w.ptr if w else None
    Lc = c.level(2 * h)
    ok(k().gs_prolong_add(c.ptr, None, C.byref(Lc), v.ptr, C.byref(L), st()))
    ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), mode, 0.8, 1.0, v.ptr, out_ref.ptr, f.ptr, wp, 0, 0, st()))
    v2, out = DevField(*shape).from_xyz(v0), DevField(*shape)
    ok(prolong_ws(stencil(), L, mode, v2.ptr, c.ptr, None, Lc, out.ptr, f.ptr, wp, 0, 0))
    np.testing.assert_array_equal(out.to_xyz(), out_ref.to_xyz())


def test_sweep2_full_1024_plane():
    """A full 1024 x 1024 plane set (the per-rank slab shape of BASELINE config #5, 4 planes) through
    the column-block pair, against two single sweeps, bit for bit."""
    rng = np.random.default_rng(1024)
    shape = (1024, 1024, 4)
    h = 1.0 / 1025
    v0, f0 = rand_full(rng, *shape), rand_full(rng, *shape, 100.0)
    ref = two_sweeps(v0, f0, np.zeros_like(v0), 0, h)
    v, f, out = DevField(*shape).from_xyz(v0), DevField(*shape).from_xyz(f0), DevField(*shape)
    L = v.level(h)
    assert b"XH" in k().gs_jacobi_sweep2_kernel(C.byref(stencil()), C.byref(L), 0)
    ok(k().gs_jacobi_sweep2(C.byref(stencil()), C.byref(L), 0, 0.8, 1.0, v.ptr, out.ptr, f.ptr, None, 0, 0, st()))
    np.testing.assert_array_equal(out.to_xyz(), ref)
