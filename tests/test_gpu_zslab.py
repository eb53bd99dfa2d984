"""Z-slab multi-GPU path on ONE GPU: gs_zslab_loopback_run runs N ranks as N threads with their own
slabs, streams and ghost planes, exchanging through device copies with the same ordering contract
as the RCCL communicator. Every point is computed by the same kernel code as on one GPU, so the
assembled fields must be bit-identical to the single-GPU solve in every mode; the residual
histories differ only by the norm's summation order (rank partials are summed in rank order)."""
import ctypes as C

import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402
from conftest import rel  # noqa: E402


def loopback(params, nranks, min_points, sweeps, solve):
    d = gsv.driver()
    p = params.to_abi()
    nx, ny, nz = params.gridDim
    v = np.zeros((nz + 2, ny + 2, nx + 2))
    cap = 4 * (params.maxiter + 2)
    hist = (C.c_double * cap)()
    cnt = C.c_int(0)
    rc = d.gs_zslab_loopback_run(C.byref(p), nranks, min_points, sweeps, 1 if solve else 0, hist, cap,
                                 C.byref(cnt), v.ctypes.data_as(gsv._abi.dptr))
    assert rc == 0, d.gs_last_error().decode()
    return list(hist[: cnt.value]), v.transpose(2, 1, 0)


def single(params, sweeps, solve):
    with gsv.HipGridData(params) as g:
        gsv.HipSolver.jacobi(g, 0, sweeps)
        hist = gsv.HipSolver.solve(g) if solve else []
        v = g.field(0, "v")
    return hist, v


@pytest.mark.parametrize("dims,nranks", [((33, 17, 40), 2), ((64, 64, 64), 4), ((31, 20, 61), 3),
                                         ((128, 64, 96), 8),
                                         # slabs large enough for the fused pairs (k_tb2y; k_tb2 for rows
                                         # > 512), their depth-2 ghosts and the overlapped boundary planes
                                         ((64, 256, 64), 2), ((32, 512, 64), 4), ((600, 128, 64), 2),
                                         ((48, 512, 70), 3)])
def test_sweeps_bit_identical(dims, nranks):
    p = gsv.GridParams(maxiter=0, gridDim=dims, mode=0)
    _, ref = single(p, 5, False)
    _, got = loopback(p, nranks, 0, 5, False)
    np.testing.assert_array_equal(got[:, :, 1:-1], ref[:, :, 1:-1])


@pytest.mark.parametrize("order", ["1", "2"])
@pytest.mark.parametrize("dims,nranks", [((64, 256, 64), 2), ((600, 128, 64), 2), ((48, 512, 70), 3),
                                         ((1024, 64, 128), 4)])
def test_sweep_sequence_halo_orders(monkeypatch, order, dims, nranks):
    """Ten sweeps in one call (five overlapped pair steps) with both dispatch orders of the pipelined
    sequence forced (GS_HALO_ORDER=1: interior k enqueued before boundary k, as when RCCL's exchange k-1 is
    still settling on the host; 2: boundary first), real concurrency on the GPU: bit-identical."""
    monkeypatch.setenv("GS_HALO_ORDER", order)
    p = gsv.GridParams(maxiter=0, gridDim=dims, mode=0)
    _, ref = single(p, 10, False)
    _, got = loopback(p, nranks, 0, 10, False)
    np.testing.assert_array_equal(got[:, :, 1:-1], ref[:, :, 1:-1])


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("dims,nranks,min_points", [((32, 32, 32), 2, 0), ((31, 31, 63), 4, 0),
                                                    ((48, 40, 64), 3, 4096), ((64, 64, 64), 2, -1),
                                                    ((64, 256, 64), 2, -1), ((32, 512, 64), 4, -1)])
def test_solve_matches_single_gpu(mode, dims, nranks, min_points):
    p = gsv.GridParams(maxiter=3 if mode == 2 else 5, tol=0.0, gridDim=dims, mode=mode)
    ref_h, ref_v = single(p, 0, True)
    h, v = loopback(p, nranks, min_points, 0, True)
    assert len(h) == len(ref_h)
    assert all(math.isfinite(a) for a in ref_h), ref_h
    for a, b in zip(h, ref_h):
        assert rel(a, b) < 1e-12, (a, b)
    # Newton keeps its result in newtonV; v is the last inner correction — equal in every mode
    np.testing.assert_array_equal(v[:, :, 1:-1], ref_v[:, :, 1:-1])


# Column-block rows (> 512 points) on slabs: the LINEAR prolongation pair's edge strip on the boundary and
# interior streams of every rank, and the column-block pairs of the non-linear modes. The non-linear RHS
# overflows where x = i h runs far past 1 (h = 1/(ny+1)), so those shapes keep nx / (ny+1) small; every
# history is asserted finite, so a regression cannot hide behind a shared inf / NaN.
@pytest.mark.parametrize("mode,dims", [(0, (1024, 32, 64)), (1, (600, 300, 24)), (2, (600, 300, 24))])
def test_column_block_solve_matches_single_gpu(mode, dims):
    p = gsv.GridParams(maxiter=3 if mode == 2 else 5, tol=0.0, gridDim=dims, mode=mode)
    ref_h, ref_v = single(p, 0, True)
    h, v = loopback(p, 2, -1, 0, True)
    assert len(h) == len(ref_h)
    assert all(math.isfinite(a) for a in ref_h + h), (ref_h, h)
    for a, b in zip(h, ref_h):
        assert rel(a, b) < 1e-12, (a, b)
    np.testing.assert_array_equal(v[:, :, 1:-1], ref_v[:, :, 1:-1])


def test_example_config_distributed(histories):
    """The reference example (Newton 127^3, 3+3, tol 1e-5) on 4 slabs vs the reference history."""
    c = histories["example_data-2nd_order"]["config"]
    p = gsv.GridParams(maxiter=c["maxiter"], tol=c["tol"], gridDim=(c["X"], c["Y"], c["Z"]), mode=c["mode"],
                       preSmoothing=c["pre"], postSmoothing=c["post"], omega=c["omega"], gamma=c["gamma"])
    h, _ = loopback(p, 4, -1, 0, True)
    ref = histories["example_data-2nd_order"]["history"]
    assert len(h) == len(ref)
    for a, b in zip(h, ref):
        assert rel(a, b) < 1e-6


@pytest.mark.parametrize("dims,nranks,min_points,pre,post", [
    ((64, 128, 128), 2, -1, 2, 2),   # even slabs on every level: the fused prolongation pair throughout
    ((64, 128, 127), 2, -1, 1, 3),   # odd top slab (three top planes first), a single sweep after the pair
    ((48, 96, 130), 2, -1, 2, 2),    # slab of 65 planes: odd z0, the unfused path
    ((32, 64, 96), 3, 4096, 3, 2),   # replicated coarse levels under Z-slab ones
    ((40, 64, 20), 4, -1, 2, 2),     # thin slabs: no overlap, one exchange after the pair
])
def test_fused_prolong_slabs_match_single_gpu(dims, nranks, min_points, pre, post):
    """The first post-smoothing pair fused with the prolongation on Z-slab levels (each rank corrects
    its ghost planes from the coarse planes under them) leaves every field as on one GPU."""
    p = gsv.GridParams(maxiter=4, tol=0.0, gridDim=dims, mode=0, preSmoothing=pre, postSmoothing=post)
    ref_h, ref_v = single(p, 0, True)
    h, v = loopback(p, nranks, min_points, 0, True)
    assert len(h) == len(ref_h)
    for a, b in zip(h, ref_h):
        assert rel(a, b) < 1e-12, (a, b)
    np.testing.assert_array_equal(v[:, :, 1:-1], ref_v[:, :, 1:-1])


def zslab_cases(n=30, seed=7):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        nranks = int(rng.integers(2, 6))
        dims = (int(rng.integers(8, 200)), int(rng.integers(8, 300)), int(rng.integers(4 * nranks, 140)))
        mode = int(rng.choice([0, 0, 1, 2]))
        pre, post = int(rng.integers(1, 4)), int(rng.integers(1, 4))
        min_points = int(rng.choice([-1, 0, 4096]))
        out.append((i, dims, nranks, mode, pre, post, min_points))
    return out


@pytest.mark.parametrize("case", zslab_cases(), ids=lambda c: f"z{c[0]}-{'x'.join(map(str, c[1]))}-r{c[2]}-m{c[3]}")
def test_zslab_random_vs_single(case):
    """Seeded random shapes, rank counts (2-5, uneven slabs), modes, smoothing counts and agglomeration
    thresholds: the loopback Z-slab solve against the single-GPU one, fields bit for bit."""
    _, dims, nranks, mode, pre, post, min_points = case
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=mode, preSmoothing=pre, postSmoothing=post)
    h1, v1 = single(p, 0, True)
    hn, vn = loopback(p, nranks, min_points, 0, True)
    a, b = np.ascontiguousarray(vn[:, :, 1:-1]), np.ascontiguousarray(v1[:, :, 1:-1])
    assert a.tobytes() == b.tobytes() or np.array_equal(a, b, equal_nan=True)
    assert len(hn) == len(h1)
    for a, b in zip(hn, h1):
        if np.isfinite(a) or np.isfinite(b):
            assert rel(a, b) < 1e-12


@pytest.mark.parametrize("dims,nranks", [((511, 127, 127), 2), ((511, 255, 127), 4), ((511, 255, 255), 8)])
def test_newton_fused_update_on_slabs(monkeypatch, dims, nranks):
    """findError's newtonV += v fused into the next compF on Z-slab ranks (k_newton_upd on the owned planes,
    the new newtonV's ghost planes formed as newtonV + 1.0 v): 2-8 loopback slabs, fused (default) and two-pass
    (GS_NO_NEWTON_FUSED_UPDATE) bit-identical to each other and to one GPU, three Newton iterations."""
    import zslab_exec as X
    p = gsv.GridParams(maxiter=3, tol=0.0, gridDim=dims, mode=2)
    ops = {op for op, _ in X.schedule(p, nranks, 0, -1)}
    assert {"newtonFupdate", "ghostsum"} <= ops, ops  # the fused path is the one the slabs take
    ref_h, ref_v = single(p, 0, True)
    h, v = loopback(p, nranks, -1, 0, True)
    monkeypatch.setenv("GS_NO_NEWTON_FUSED_UPDATE", "1")
    h2, v2 = loopback(p, nranks, -1, 0, True)
    assert all(math.isfinite(a) for a in ref_h), ref_h
    assert len(h) == len(h2) == len(ref_h)
    for a, b, c in zip(h, h2, ref_h):
        assert a == b and rel(a, c) < 1e-12, (a, b, c)
    np.testing.assert_array_equal(v[:, :, 1:-1], v2[:, :, 1:-1])
    np.testing.assert_array_equal(v[:, :, 1:-1], ref_v[:, :, 1:-1])


@pytest.mark.parametrize("dims,nranks,touch", [((127, 63, 64), 2, 0), ((127, 63, 96), 3, 2)])
def test_newton_zero_shortcut_agreed_across_ranks(monkeypatch, dims, nranks, touch):
    """The first findError skips the restrictions of a still-zero newtonV, and restrictions exchange ghost planes on
    distributed levels: when ONE rank has handed its newtonV out (gs_grid_field, here the loopback runner's test hook)
    the ranks must agree before deciding, or that rank issues exchanges nobody answers. With the agreement every rank
    restricts (zeros), and the solve is bit-identical to the untouched one."""
    p = gsv.GridParams(maxiter=2, tol=0.0, gridDim=dims, mode=2)
    h, v = loopback(p, nranks, 0, 0, True)
    monkeypatch.setenv("GS_LOOPBACK_TOUCH_NEWTONV", str(touch))
    h2, v2 = loopback(p, nranks, 0, 0, True)
    assert all(math.isfinite(a) for a in h), h
    assert h == h2
    np.testing.assert_array_equal(v[:, :, 1:-1], v2[:, :, 1:-1])
