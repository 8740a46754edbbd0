"""The reference's invalid-argument API tests (test/liberasurecode_test.c:598-1072, restated in
tests/ref_api_invalid.py) against this repo's liberasurecode.so.1.

CPU: in a child process whose LD_LIBRARY_PATH puts the REFERENCE codec libraries (oracle/_ref,
compiled from /root/reference sources) first -- the argument checks and return codes are the
frontend's, so they must hold with any codec behind it.  GPU: in-process with this repo's codecs."""
import json
import os
import subprocess
import sys

import pytest

import ref_api_invalid as R

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = os.path.join(ROOT, "oracle", "_ref")
NAMES = [f.__name__ for f in R.SUITE]


@pytest.fixture(scope="module", params=sorted(R.BACKENDS))
def cpu_results(request):
    if not all(os.path.exists(os.path.join(REF, n)) for n in ("libXorcode.so.1", "liberasurecode_rs_vand.so.1")):
        pytest.skip("oracle/_ref not built (needs /root/reference: make -C oracle)")
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = REF + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    r = subprocess.run([sys.executable, os.path.join(HERE, "ref_api_invalid_run.py"), request.param],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("name", NAMES)
def test_invalid_args_over_reference_codec(cpu_results, name):
    assert cpu_results[name] == "ok", cpu_results[name]


@pytest.mark.gpu
@pytest.mark.parametrize("backend", sorted(R.BACKENDS))
@pytest.mark.parametrize("fn", R.SUITE, ids=NAMES)
def test_invalid_args_gpu(fn, backend):
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    fn(R.BACKENDS[backend])
