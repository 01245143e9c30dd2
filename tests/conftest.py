import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

# Registers the package under its importable name `wavelet_compression_amd`
# (the directory name has a dash); loading it does not touch the GPU.
import wcamd  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def wc():
    import wcamd
    wcamd.capi.load_library()
    return wcamd


@pytest.fixture(scope="session")
def ctx(wc):
    c = wc.capi.Context(0)
    yield c
    c.close()
