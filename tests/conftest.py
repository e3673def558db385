import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def vit():
    from vitpkg import vit as v
    return v


@pytest.fixture(scope="session")
def oracle32():
    import oracle_ctypes as oc
    return oc.Oracle("f32")


@pytest.fixture(scope="session")
def oracle64():
    import oracle_ctypes as oc
    return oc.Oracle("f64")


@pytest.fixture(scope="session")
def gpu(vit):
    """Load the HIP library and select device 0 (fails loudly if the .so is missing)."""
    L = vit.lib()
    assert L.vit_init(0) == 0, "vit_init(0) failed"
    vit.check("vit_init")
    return vit


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / den)
