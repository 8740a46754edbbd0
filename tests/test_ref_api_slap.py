"""test/libec_slap.c (the reference's API stress test of flat_xor_hd), restated in
tests/ref_api_slap.py, against this repo's liberasurecode.so.1.

CPU: in a child process whose LD_LIBRARY_PATH puts the REFERENCE libXorcode (oracle/_ref, compiled
from /root/reference sources) first.  GPU: in-process with this repo's flat-XOR codec."""
import json
import os
import subprocess
import sys

import pytest

import ref_api_slap as S

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = os.path.join(ROOT, "oracle", "_ref")
IDS = [f"{k}_{m}_{hd}" for k, m, hd in S.CODES]


@pytest.fixture(scope="module")
def cpu_results():
    if not os.path.exists(os.path.join(REF, "libXorcode.so.1")):
        pytest.skip("oracle/_ref not built (needs /root/reference: make -C oracle)")
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = REF + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    r = subprocess.run([sys.executable, os.path.join(HERE, "ref_api_slap_run.py")], capture_output=True, text=True,
                       timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_fill_buffer_matches_reference_arithmetic():
    """fill_buffer (libec_slap.c:146-151) in plain loops, against the vectorised restatement."""
    seed, want = 0, bytearray()
    for i in range(5000):
        seed += i
        want.append(seed & 0xFF)
    assert S.fill_buffer(5000) == bytes(want)


@pytest.mark.parametrize("code", IDS)
def test_slap_over_reference_codec(cpu_results, code):
    assert cpu_results[code] == "ok", cpu_results[code]


@pytest.mark.gpu
@pytest.mark.parametrize("code", S.CODES, ids=IDS)
def test_slap_gpu(code):
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    S.slap(*code)
