import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnn-mtl_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libgnnea.so")
    config.addinivalue_line("markers", "slow: large-size property tests")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
        return cache[name]

    return load


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def rel_err(a, b):
    """||a - b||_inf / ||b||_inf (norm-relative)."""
    import numpy as np

    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.max(np.abs(b))
    return float(np.max(np.abs(a - b)) / (den if den > 0 else 1.0))


@pytest.fixture
def relu_band(record_property):
    """Counts of ReLU elements whose branch the oracles took from the tested output (inside the
    rounding band of 0, oracle/local.py / tests/fp64_ref.py), recorded per test as the property
    ``relu_band`` and appended to $GNNEA_BAND_LOG (JSON lines) when set."""
    import json
    from oracle import local
    import fp64_ref
    local.reset_band()
    fp64_ref.reset_band()
    yield
    rec = {"oracle_local": dict(local.BAND), "fp64_ref": dict(fp64_ref.BAND)}
    record_property("relu_band", json.dumps(rec))
    path = os.environ.get("GNNEA_BAND_LOG")
    if path:
        rec["test"] = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
