"""Pins the CPU oracle (oracle/gs_oracle.cpp) against fixtures produced by the REFERENCE itself
(oracle/_ref/ref_probe linking /root/reference/src/cpu/*.cpp; tests/golden/make_golden.py).

Element-wise operators must match bit for bit; l2 norms and residual histories to 1e-12 relative
(the reference's own OpenMP reduction order moves them by ~1e-14 between thread counts)."""
import numpy as np
import pytest

import oracle as O
from conftest import rel, stencil_from_text


def _stencil(c):
    if "stencil" not in c:
        return None
    vals, offs = stencil_from_text(c["stencil"])
    return O.Stencil.make(vals, offs)


def test_example_config_history(histories):
    h = histories["example_data-2nd_order"]["history"]
    # SURVEY.md Appendix B anchors
    assert h[0] == pytest.approx(281.2891028676857, rel=1e-14)
    assert h[-1] == pytest.approx(0.00093763035084784595, rel=1e-12)
    assert len(h) == 5  # stops after 4 Newton iterations (tol 1e-5)


@pytest.mark.parametrize("name", [
    "m0_n7_2+2", "m1_n7_2+2", "m2_n7_2+2", "m0_n15_2+2", "m0_n16_2+2", "m1_n16_2+2", "m2_n16_2+2",
    "m0_n31_2+2", "m1_n31_2+2", "m2_n31_2+2", "m0_n32_2+2", "m1_n32_2+2", "m2_n32_2+2",
    "m0_n31_1+0", "m1_n32_3+3", "m2_n31_0+2", "m0_17x9x12_2+2", "m1_31x32x33_2+2", "m2_20x33_15_2+2",
    "m0_9x40x23_2+2", "m0_n63_w0.6", "m1_n63_g0.5", "m2_n63_g2.0", "m0_n63_tol1e-3", "m1_n63_tol1e-4",
    "m2_n63_tol1e-6", "m0_n31_permuted", "m0_n31_aniso", "m0_n63_2+2", "m1_n63_2+2",
])
def test_oracle_histories(histories, name):
    if name not in histories:
        name = name.replace("20x33_15", "20x33x15")
    case = histories[name]
    c = case["config"]
    g = O.Grid((c["X"], c["Y"], c["Z"]), mode=c["mode"], maxiter=c["maxiter"], tol=c["tol"], omega=c["omega"],
               gamma=c["gamma"], pre=c["pre"], post=c["post"], stencil=_stencil(c))
    got = g.solve()
    ref = case["history"]
    assert len(got) == len(ref), (got, ref)
    for a, b in zip(got, ref):
        assert rel(a, b) < 1e-12, (a, b)


def test_oracle_levels():
    from conftest import load_json
    levels = load_json("levels.json")
    for key, rows in levels.items():
        dims = tuple(int(x) for x in key.split("x"))
        if max(dims) > 600:
            continue  # allocation-heavy on CPU; the rule is checked on the smaller shapes
        g = O.Grid(dims, maxiter=0)
        assert g.levels() == len(rows)
        for l, (nx, ny, nz, h, has_e) in enumerate(rows):
            d, hh = g.level_info(l)
            assert d == (nx, ny, nz) and hh == h
            assert (g.field(l, "e") is not None) == bool(has_e)


def test_oracle_rhs_bitwise(rhs_arrays):
    for key, ref in rhs_arrays.items():
        _, dims, m, gm = key.split("_")
        nx, ny, nz = (int(x) for x in dims.split("x"))
        got = O.rhs(nx, ny, nz, int(m[1:]), float(gm[1:]))
        np.testing.assert_array_equal(got, ref, err_msg=key)


def _lvl_dims(dims, lvl):
    d = list(dims)
    for _ in range(lvl):
        d = [x // 2 for x in d]
    return d


def test_oracle_ops_bitwise(ops_meta, ops_arrays):
    checked = 0
    for key, info in ops_meta.items():
        a = {k.split("/", 1)[1]: v for k, v in ops_arrays.items() if k.split("/", 1)[0] == key}
        name, mode, lvl = info["name"], info["mode"], info["level"]
        dims = _lvl_dims(info["dims"], lvl)
        h = 1.0 / (dims[1] + 1)
        extra = info["extra"]
        omega, gamma, k = (float(extra[0]), float(extra[1]), int(extra[2])) if extra else (0.8, 1.0, 1)
        if name == "residual":
            r, n = O.residual(a["v"], a["f"], h, mode, gamma, w=a["newtonV"])
            np.testing.assert_array_equal(r, a["r"], err_msg=key)
            assert rel(n, info["norm"]) < 1e-13
        elif name == "jacobi":
            out = O.jacobi(a["v"], a["f"], h, mode, omega, gamma, k, w=a["newtonV"])
            np.testing.assert_array_equal(out, a["v_out"], err_msg=key)
        elif name == "restrict":
            c = O.restrict(a["fine"], _lvl_dims(info["dims"], lvl + 1))
            np.testing.assert_array_equal(c, a["coarse"], err_msg=key)
        elif name == "interpolate":
            e = O.interpolate(a["coarse"], dims)
            np.testing.assert_array_equal(e, a["e"], err_msg=key)
        elif name == "applyStencil":
            out = O.apply_op(a["u"], h, gamma)
            np.testing.assert_array_equal(out, a["r"], err_msg=key)
        elif name == "compF":
            f, n = O.newton_F(a["newtonV"], a["newtonF"], h, gamma)
            # compF writes the interior only; the dumped boundary still holds the constructor's RHS
            np.testing.assert_array_equal(f[1:-1, 1:-1, 1:-1], a["f"][1:-1, 1:-1, 1:-1], err_msg=key)
            assert rel(n, info["norm"]) < 1e-13
        elif name == "vcycle":
            g = O.Grid(info["dims"], mode=mode, maxiter=1)
            for l in range(g.levels()):
                g.field(l, "newtonV")[...] = a[f"newtonV{l}"]
            g.field(0, "v")[...] = a["v"]
            np.testing.assert_array_equal(g.field(0, "f"), a["f"])
            n = g.vcycle()
            np.testing.assert_array_equal(g.field(0, "v"), a["v_out"], err_msg=key)
            assert rel(n, info["norm"]) < 1e-13
        else:
            raise AssertionError(name)
        checked += 1
    assert checked == len(ops_meta) and checked > 50
