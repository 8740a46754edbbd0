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
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True)
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "liberasurecode_amd", "csrc")],
                   check=True)
    yield
