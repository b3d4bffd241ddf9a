import os
import sys

import pytest

# torch before the engine library: one HIP runtime per process, and torch's
# must be the one libopenr_gpu.so binds to (the bench-size tests drive the
# engine through torch-owned device buffers and streams, as bench.py does)
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    """CPU oracle (test infrastructure only)."""
    import _refcpu
    return _refcpu


@pytest.fixture(scope="session")
def product():
    """The GPU product module; fails loudly if the HIP path is unavailable."""
    import openr_amd
    openr_amd.require_gpu()
    return openr_amd.decision


@pytest.fixture(scope="session")
def host_module():
    """The product module for host-only checks (CSR images, layouts): no
    device call is made through it, so it is usable without a GPU."""
    import openr_amd
    return openr_amd.decision
