"""The kernels' division by h^2 (div_hh: a 3-operation path where the hardware division sequence
would not rescale) against the plain IEEE division, bit for bit, over every binade of the numerator
(including zero, denormals, inf/nan and the window edges) and the h^2 of every grid size class."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import gpusolve as gsv  # noqa: E402


def numerators(rng):
    e = rng.integers(-1074, 1024, 400_000)
    m = rng.uniform(1.0, 2.0, e.size)
    a = np.ldexp(m, e) * rng.choice([-1.0, 1.0], e.size)
    edges = [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 2.2250738585072014e-308,
             np.ldexp(1.0, -899), np.ldexp(1.0, -900), np.nextafter(np.ldexp(1.0, -899), 0),
             np.ldexp(1.0, 600), np.ldexp(1.0, 601), np.nextafter(np.ldexp(1.0, 601), 0), 1.0, -1.0]
    typical = rng.normal(0, 1, 200_000) * np.exp(rng.uniform(-40, 40, 200_000))
    return np.concatenate([a, np.array(edges), typical])


@pytest.mark.parametrize("n", [1, 2, 3, 7, 31, 63, 100, 127, 511, 512, 1000, 1023, 2047, 4095, 1 << 20])
def test_div_hh_bitwise(n):
    rng = np.random.default_rng(n)
    hh = (1.0 / (n + 1)) * (1.0 / (n + 1))
    a = numerators(rng)
    d = torch.from_numpy(a).cuda()
    fast, ref = torch.empty_like(d), torch.empty_like(d)
    rc = gsv.diag().gs_debug_div_check(d.data_ptr(), d.numel(), hh, fast.data_ptr(), ref.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    fb = fast.cpu().numpy().view(np.uint64)
    rb = ref.cpu().numpy().view(np.uint64)
    bad = np.nonzero(fb != rb)[0]
    assert bad.size == 0, [(a[i], fast[i].item(), ref[i].item()) for i in bad[:5]]
    # the device division is IEEE: it also agrees with numpy's
    want = (a / hh).view(np.uint64)
    nan = np.isnan(a / hh)
    assert np.array_equal(rb[~nan], want[~nan])


def _values(rng, n, lo, hi):
    e = rng.integers(lo, hi, n)
    return np.ldexp(rng.uniform(1.0, 2.0, n), e) * rng.choice([-1.0, 1.0], n)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_newton_update_quotient_bitwise(seed):
    """NEWTON pairs form r / den through den's reciprocal when both operands lie in the safe window
    (newton_update_y2): bit for bit the IEEE division over every binade of both operands, the window edges,
    zeros, denormals, inf / NaN and rows whose two points fall on different sides of the window."""
    rng = np.random.default_rng(seed)
    n = 400_000
    r = np.concatenate([_values(rng, n, -1074, 1024), rng.normal(0, 1, n) * np.exp(rng.uniform(-60, 60, n))])
    den = np.concatenate([_values(rng, n, -1074, 1024), 1.6e6 + rng.normal(0, 1e3, n)])  # (preFac ~ 6 / h^2)
    edges = [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, 2.2250738585072014e-308, np.ldexp(1.0, -300),
             np.nextafter(np.ldexp(1.0, -300), 0), np.ldexp(1.0, 400), np.nextafter(np.ldexp(1.0, 400), 0),
             np.ldexp(1.0, -400), np.nextafter(np.ldexp(1.0, -400), 0), np.ldexp(1.0, 300),
             np.nextafter(np.ldexp(1.0, 300), 0), 1.0, -1.0, 1.6e6]
    e = np.array(edges)
    rr, dd = np.meshgrid(e, e)
    r = np.concatenate([r, rr.ravel(), -rr.ravel()])
    den = np.concatenate([den, dd.ravel(), dd.ravel()])
    if r.size % 2:
        r, den = r[:-1], den[:-1]
    dr, dden = torch.from_numpy(r).cuda(), torch.from_numpy(den).cuda()
    fast, ref = torch.empty_like(dr), torch.empty_like(dr)
    assert gsv.diag().gs_debug_newton_div_check(dr.data_ptr(), dden.data_ptr(), dr.numel(), 0.8, fast.data_ptr(),
                                                ref.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    fb, rb = fast.cpu().numpy().view(np.uint64), ref.cpu().numpy().view(np.uint64)
    bad = np.nonzero(fb != rb)[0]
    assert bad.size == 0, [(r[i], den[i], fast[i].item(), ref[i].item()) for i in bad[:5]]
