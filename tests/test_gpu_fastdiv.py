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


