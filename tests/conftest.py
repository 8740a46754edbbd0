import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (test infrastructure) and the product libraries once per session -- in
    the build container only (where /root/reference lives).  On a GPU box the libraries built here
    travel with the tree and are used as they are: nothing is compiled inside a GPU run."""
    if not os.path.isdir("/root/reference"):
        yield
        return
    import fcntl
    # one build at a time: pytest-xdist workers each run this fixture, and two makes writing the
    # same .so at once hand a half-written library to a test that loads it
    with open(os.path.join(ROOT, ".pytest_build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "liberasurecode_amd", "csrc")],
                       check=True)
        fcntl.flock(lock, fcntl.LOCK_UN)
    yield
