"""test/liberasure_rs_isal_stress_test.c (the reference's API stress test, any backend id) restated for
liberasurecode_rs_vand in tests/ref_api_stress.py, against this repo's liberasurecode.so.1:
every 1..4-erasure decode and reconstruct of (10, 4) -- all 1,470 sets -- and 2,000 random 8-erasure
sets of (20, 8).

CPU: in a child process whose LD_LIBRARY_PATH puts the REFERENCE liberasurecode_rs_vand (oracle/_ref,
compiled from /root/reference sources) first; its digests must equal tests/golden/rs_stress.json
(tests/golden/make_stress_golden.py).  GPU: in-process with this repo's codec -- every call checked as
the reference checks it, and the digests of all encoded, decoded and rebuilt bytes equal to the
reference codec's."""
import json
import os
import subprocess
import sys

import pytest

import ref_api_stress as S

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = os.path.join(ROOT, "oracle", "_ref")
GOLDEN = json.load(open(os.path.join(HERE, "golden", "rs_stress.json")))["codes"]
IDS = [f"{k}_{m}" for k, m in S.CODES]


def test_pattern_sets():
    """(10, 4): all C(14,1..4) = 14 + 91 + 364 + 1001 sets, distinct; (20, 8): 2000 sets of exactly 8."""
    p = S.patterns(10, 4)
    assert len(p) == 1470 and len({tuple(x) for x in p}) == 1470
    q = S.patterns(20, 8)
    assert len(q) == 2000 and all(len(set(x)) == 8 and max(x) < 28 for x in q)
    assert GOLDEN["10_4"]["patterns"] == 1470 and GOLDEN["20_8"]["patterns"] == 2000


@pytest.fixture(scope="module")
def cpu_results():
    if not os.path.exists(os.path.join(REF, "liberasurecode_rs_vand.so.1")):
        pytest.skip("oracle/_ref not built (needs /root/reference: make -C oracle)")
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = REF + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    r = subprocess.run([sys.executable, os.path.join(HERE, "ref_api_stress_run.py")], capture_output=True, text=True,
                       timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("code", IDS)
def test_stress_over_reference_codec(cpu_results, code):
    assert isinstance(cpu_results[code], dict), cpu_results[code]
    assert cpu_results[code] == GOLDEN[code]


@pytest.mark.gpu
@pytest.mark.parametrize("code", S.CODES, ids=IDS)
def test_stress_gpu(code):
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    k, m = code
    assert S.stress(k, m) == GOLDEN[f"{k}_{m}"]
