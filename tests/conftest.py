"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs the oracle / host-logic / ABI-surface tests on any CPU box;
`-m gpu` runs the HIP-vs-oracle parity tests (they need an MI355X and call through the C ABI).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path")


def _ensure_built(target_dir, out):
    if not os.path.exists(out):
        subprocess.run(["make", "-C", target_dir, "-j8"], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle():
    import oracle_bind
    _ensure_built(os.path.join(ROOT, "oracle"), oracle_bind.ORACLE_PATH)
    return oracle_bind.Oracle()


@pytest.fixture(scope="session")
def ctx():
    """A yv_ctx on GPU 0 with the reference constants and the committed BRIEF offsets table."""
    import numpy as np
    import ya_vo_amd as yv
    _ensure_built(os.path.join(ROOT, "ya_vo_amd", "csrc"), yv.LIB_PATH)
    c = yv.Context(0)
    c.set_brief_offsets(np.fromfile(os.path.join(TESTS, "golden", "brief_offsets_mt19937_42.bin"), np.int8))
    yield c
    c.close()


@pytest.fixture(scope="session")
def offsets():
    import numpy as np
    return np.fromfile(os.path.join(TESTS, "golden", "brief_offsets_mt19937_42.bin"), np.int8).reshape(256, 4)
