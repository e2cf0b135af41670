import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer GPU parity combinations (still part of -m gpu)")
    config.addinivalue_line("markers", "variants: the kernels measured slower than the automatic paths, built into "
                                       "libhmc_amd_variants.so only (HMC_AMD_LIB=hmc_amd/libhmc_amd_variants.so -m variants)")


def pytest_collection_modifyitems(config, items):
    """Tests of the variant kernels run only against the variants library:
    the product library refuses to select them (HMC_EUNSUPPORTED)."""
    if "variants" in os.path.basename(os.environ.get("HMC_AMD_LIB", "")):
        return
    skip = pytest.mark.skip(reason="variant kernels: HMC_AMD_LIB=hmc_amd/libhmc_amd_variants.so pytest -m variants")
    for it in items:
        if "variants" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # test infrastructure (CPU restatement)

    oracle.build()
    return oracle


@pytest.fixture(scope="session", autouse=True)
def _heartbeat():
    """HMC_HEARTBEAT_FILE=path: append a line every 30 s while the session
    runs, so a remote runner that watches its output directory sees progress
    during long full-size tests (their own output is captured by pytest)."""
    path = os.environ.get("HMC_HEARTBEAT_FILE")
    if not path:
        yield
        return
    import threading
    import time

    stop = threading.Event()

    def beat():
        t0 = time.time()
        while not stop.wait(30.0):
            with open(path, "a") as f:
                f.write(f"alive {time.time() - t0:.0f} s\n")

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
