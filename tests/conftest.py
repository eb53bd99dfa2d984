import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (os.path.join(REPO, "gpu-solve_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running (BASELINE-size grids)")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def histories():
    return load_json("histories.json")


@pytest.fixture(scope="session")
def large_histories():
    return load_json("large_histories.json")


@pytest.fixture(scope="session")
def ops_meta():
    return load_json("ops.json")


@pytest.fixture(scope="session")
def ops_arrays():
    with np.load(os.path.join(GOLDEN, "ops.npz")) as z:
        return {k.replace("__", "/"): z[k] for k in z.files}


@pytest.fixture(scope="session")
def rhs_arrays():
    with np.load(os.path.join(GOLDEN, "rhs.npz")) as z:
        return {k: z[k] for k in z.files}


def stencil_from_text(text):
    rows = text.strip().splitlines()
    vals = [float(x) for x in rows[0].split()]
    ox, oy, oz = ([int(x) for x in r.split()] for r in rows[1:4])
    return vals, list(zip(ox, oy, oz))


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


@pytest.fixture(scope="session")
def huge_histories():
    return load_json("huge_histories.json")


@pytest.fixture(scope="session")
def config3_histories():
    return load_json("config3_histories.json")
