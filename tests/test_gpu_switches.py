"""Every A/B switch of the library selects a bit-identical path: a solve under each
switch against the default build's, level 0's iterate compared byte for byte, the history to 1e-12
(paths that change the norm's block structure change its summation order only). The library reads
its switches once per process, so each run is a child process (tests/switch_probe.py), one at a time."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, rel

pytestmark = pytest.mark.gpu

PROBE = os.path.join(REPO, "tests", "switch_probe.py")
SWITCHES = ["GS_COARSE_POINTS", "GS_NEWTON_PRO_POINTS", "GS_RR_NR", "GS_RR_LDS", "GS_NO_FUSED_SWEEPS",
            "GS_NO_FUSED_RR", "GS_NO_FUSED_PROLONG", "GS_NO_SPECULATION", "GS_NO_ZERO_GUESS", "GS_PAIR_XH",
            "GS_TBX_PFD", "GS_PAIR_BIG_CHUNKS", "GS_NO_UNIT_STENCIL", "GS_PAIR_MIN_BLOCKS", "GS_FIT_ROUNDS",
            "GS_NO_PIPELINE", "GS_NO_NEWTON_FUSED_UPDATE", "GS_RR_NTU", "GS_PAIR_ONE_ROUND", "GS_SLAB_ZC", "GS_PAIR_ZC",
            "GS_RR_REVERSE", "GS_HALO_ORDER", "GS_NO_ZERO_Q", "GS_XH_SWIZZLE",
            "GS_MID_ZC", "GS_RR_ZC", "GS_NEWTON_XH", "GS_SPEC_CACHED", "GS_RR_ZC_BIG", "GS_PAIR_ONE_ROUND_MID", "GS_RB_ZC", "GS_RR_NG", "GS_NEWTON_B_FUSED",
            "GS_NO_NEWTON_G", "GS_RR_DMA", "GS_PAIR_FX"]

# (case, solve args) -> the switches whose paths that problem exercises
CASES = {
    "linear256": ((0, 256, 256, 256, 3), [("GS_RR_NTU", "1"), ("GS_NO_FUSED_SWEEPS", "1"), ("GS_NO_FUSED_RR", "1"),
                                          ("GS_NO_FUSED_PROLONG", "1"), ("GS_NO_SPECULATION", "1"),
                                          ("GS_NO_ZERO_GUESS", "1"), ("GS_NO_PIPELINE", "1"), ("GS_RR_LDS", "1"),
                                          ("GS_RR_NR", "2"), ("GS_NO_UNIT_STENCIL", "1"),
                                          ("GS_PAIR_MIN_BLOCKS", "512"), ("GS_FIT_ROUNDS", "0"),
                                          ("GS_COARSE_POINTS", "4096"), ("GS_NO_ZERO_Q", "1"),
                                          ("GS_MID_ZC", "32"), ("GS_RR_ZC", "5"), ("GS_PAIR_ONE_ROUND_MID", "1"),
                                          ("GS_RR_DMA", "2")]),
    "linear2e26": ((0, 512, 512, 256, 2), [("GS_RR_NR", "1"), ("GS_PAIR_BIG_CHUNKS", "0"), ("GS_RR_NTU", "0"),
                                           ("GS_RR_ZC_BIG", "7")]),
    "linear512": ((0, 512, 512, 512, 2), [("GS_PAIR_ONE_ROUND", "0"), ("GS_PAIR_ZC", "96"), ("GS_RR_REVERSE", "0"),
                                          ("GS_SPEC_CACHED", "1"), ("GS_RR_NG", "2"), ("GS_RR_DMA", "2"),
                                          ("GS_PAIR_FX", "0")]),
    "linear_rows700": ((0, 700, 64, 64, 3), [("GS_PAIR_XH", "0"), ("GS_TBX_PFD", "1"), ("GS_XH_SWIZZLE", "0")]),
    # two loopback slabs of 512^3: the interior launches of the overlapped sweeps (z0 != 0)
    "slabs512": ((0, 512, 512, 1024, 2, 2, 2, 2), [("GS_SLAB_ZC", "16"), ("GS_HALO_ORDER", "1")]),
    "newton127": ((2, 127, 127, 127, 2), [("GS_NEWTON_PRO_POINTS", "0"), ("GS_NO_FUSED_PROLONG", "1"),
                                          ("GS_NO_PIPELINE", "1"), ("GS_NO_NEWTON_FUSED_UPDATE", "1"),
                                          ("GS_RR_REVERSE", "0"), ("GS_NO_ZERO_Q", "1")]),
    # two loopback slabs in NEWTON mode: GS_NEWTON_G's pairs on slab plane ranges (ghost planes of the factor)
    "newton_slabs": ((2, 130, 66, 128, 2, 2, 2, 2), [("GS_NO_NEWTON_G", "1")]),
    "newton_rows700": ((2, 700, 12, 10, 2), [("GS_NEWTON_XH", "0"), ("GS_NO_NEWTON_G", "1")]),
    # rows of whole 128-point waves: the NEWTON_B plain and prolongation pairs' FX instances
    "newton256": ((2, 256, 64, 64, 2), [("GS_PAIR_FX", "0")]),
    "newton255": ((2, 255, 127, 127, 2), [("GS_RB_ZC", "10"), ("GS_RR_NG", "2"), ("GS_NEWTON_B_FUSED", "0"),
                                          ("GS_NO_NEWTON_G", "1"), ("GS_RR_DMA", "2")]),
}
PARAMS = [(case, sw, val) for case, (_, sws) in CASES.items() for sw, val in sws]
_default = {}


def run(tmp_path, case, env_extra):
    args, _ = CASES[case]
    out = str(tmp_path / f"{case}_{'_'.join(env_extra) or 'default'}.npz")
    env = {k: v for k, v in os.environ.items() if k not in SWITCHES}
    env.update(env_extra)
    r = subprocess.run([sys.executable, PROBE, out, *map(str, args)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = np.load(out)
    return d["v"], list(d["hist"])


def test_switch_list_matches_integration_doc():
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    for s in SWITCHES:
        assert s in doc, s
    assert {s for _, s, _ in PARAMS} == set(SWITCHES) - {"GS_ZSLAB_MIN_POINTS"}


@pytest.mark.parametrize("case,switch,value", PARAMS)
def test_switch_bit_identical(tmp_path_factory, case, switch, value):
    if case not in _default:
        _default[case] = run(tmp_path_factory.mktemp("d"), case, {})
    v0, h0 = _default[case]
    v, h = run(tmp_path_factory.mktemp("s"), case, {switch: value})
    assert v.tobytes() == v0.tobytes(), f"{switch}={value}: level-0 field differs"
    assert len(h) == len(h0)
    for a, b in zip(h, h0):
        assert rel(a, b) < 1e-12, (switch, a, b)
