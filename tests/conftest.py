import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "duckdb-lancedb_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu on the GPU box")
    config.addinivalue_line("markers", "slow: larger parity cases")


@pytest.fixture(scope="session")
def hip():
    """The product library; GPU tests fail loudly (no fallback) if it is missing."""
    import lance_hip

    # one HIP runtime in the process: lance_hip.lib() imports torch before it
    # maps the library (see there); torch's CUDA state is initialised here once
    try:
        import torch

        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except ImportError:
        pass
    lance_hip.lib()
    assert lance_hip.device_count() > 0, "no HIP device visible to liblancedb_hip.so"
    return lance_hip
