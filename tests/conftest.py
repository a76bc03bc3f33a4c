import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# A/B runs (tools/build_ab.sh): the parity tests against a saved variant build of the package
AB_ROOT = os.environ.get("ALAYA_AB_ROOT")
if AB_ROOT:
    sys.path.insert(0, AB_ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def native():
    # torch (bundled HIP runtime) initialises the GPU before the engine's libamdhip64 does: the other
    # order leaves torch without devices in tests that use torch streams (bench.py runs this order)
    try:
        import torch

        torch.cuda.is_available()
    except Exception:  # pragma: no cover - torch is optional for the engine itself
        pass
    if not AB_ROOT:  # (a saved variant is prebuilt and has no sources)
        from alayalite_amd import _build

        _build.build()
    from alayalite_amd import _native

    return _native._ext


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.build()
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def has_gpu(native):
    return native.device_count() > 0


@pytest.fixture(scope="session")
def c1():
    """BASELINE config 1: 1k x 128 U[0,1) base + 10 queries, numpy default_rng(0)."""
    rng = np.random.default_rng(0)
    base = rng.random((1000, 128), dtype=np.float32)
    queries = rng.random((10, 128), dtype=np.float32)
    return base, queries
