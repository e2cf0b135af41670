import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


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
