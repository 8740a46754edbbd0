"""GPU: concurrency of the drop-in liberasurecode.so.1 -- tests/c/threaded_test.c restates the
reference's test/liberasurecode_threaded_test.c races (create / destroy / encode / decode /
reconstruct / fragments_needed / get_fragment_size vs destroy) and adds a shared-descriptor
stress phase that checks every byte of encode -> decode -> reconstruct round trips run from
8 threads at once (the pooled per-call GPU staging of liberasurecode_amd/csrc/host/hostio.cpp)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "liberasurecode_amd", "lib")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("thr") / "threaded_test")
    subprocess.run(["gcc", "-O2", "-std=gnu99", "-I" + os.path.join(ROOT, "include"), "-o", out,
                    os.path.join(ROOT, "tests", "c", "threaded_test.c"), "-L" + LIB,
                    "-l:liberasurecode.so.1", "-Wl,-rpath," + LIB, "-lpthread"], check=True)
    return out


@pytest.mark.parametrize("backend,k,m,hd", [(6, 10, 5, 0), (3, 10, 5, 4), (6, 4, 2, 0)],
                         ids=["rs_vand_10_5", "flat_xor_hd_10_5_4", "rs_vand_4_2"])
def test_threaded(exe, backend, k, m, hd):
    r = subprocess.run([exe, str(backend), str(k), str(m), str(hd), "8", "4"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "stress 8 threads x 4 ok" in r.stdout
