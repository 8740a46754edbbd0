"""GPU: the reference's golden digests (tests/golden/rs_vand.json, made by driving the reference
codec compiled from /root/reference) on the EXACT kernel that runs -- the run-time compiled
bitsliced kernel (knob "bitslice" 2: wait for its compile) and the LDS-table kernels (knob 0) --
whatever earlier tests left in the kernel cache.  A per-process counter of bitsliced launches
(ecamd_bitslice_launches) proves which one ran.  Covers every golden case with 5..8 outputs per
row group over whole 16 KiB tiles (the bitsliced kernel's domain): C5 encode, the C5 rebuild-8
patterns the bench times ({0..7} and the mixed {0,2,4,6,20,22,24,26}) at 4 MiB, inconsistent
("garbage") inputs, ragged tails, k = 24 / 32 -- and, since round 4, every case with 3..4 outputs
over at least one 4 KiB tile, which the one-wave form of the kernel takes (C3 encode and the
decodes {0,1,2,3} / {0,5,10,13} the bench times, at 1 MiB).
Reference: src/builtin/rs_vand/liberasurecode_rs_vand.c:399-410 (encode), :426-481 (decode)."""
import ctypes as C
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as orc
from ecdata import stripe_fragments
from liberasurecode_amd import _lib
from liberasurecode_amd import device as D

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "rs_vand.json")))
BS_TILE = 16384


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def launches():
    f = _lib.dev().ecamd_bitslice_launches
    f.restype = C.c_longlong
    return f()


BS_TILE_WAVE = 4096  # one-wave tiles of 3..4-output maps (knob bs_wave, default 1; round 4)


def _bitsliced_shape(k, outputs, bs):
    return k <= 32 and ((5 <= outputs <= 8 and bs >= BS_TILE) or (3 <= outputs <= 4 and bs >= BS_TILE_WAVE))


ENC = [c for c in GOLD["encode"] if c["pattern"] is None and _bitsliced_shape(c["k"], c["m"], c["bs"])]
DEC = [c for c in GOLD["decode"] if c["ret"] == 0 and _bitsliced_shape(c["k"], len(c["missing"]), c["bs"])]


@pytest.fixture(params=[2, 0], ids=["bitsliced", "lds_tables"])
def mode(request):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", request.param)
    d.ecamd_tune(b"small_chunks", 0)  # one-stripe goldens would otherwise take the small-launch kernel
    yield request.param
    d.ecamd_tune(b"bitslice", 1)
    d.ecamd_tune(b"small_chunks", -1)


def _check_ran(mode, before):
    after = launches()
    if mode == 2:
        assert after > before, "the bitsliced kernel did not run"
    else:
        assert after == before, "the bitsliced kernel ran with the knob off"


def test_cases_cover_the_bench_patterns():
    pats = {(c["k"], c["bs"], tuple(c["missing"]), c["garbage"]) for c in DEC}
    assert (20, 1 << 22, tuple(range(8)), False) in pats
    assert (20, 1 << 22, (0, 2, 4, 6, 20, 22, 24, 26), False) in pats
    assert (20, 1 << 22, tuple(range(8)), True) in pats
    assert any(c["k"] == 20 and c["m"] == 8 and c["bs"] == 1 << 22 for c in ENC)
    c3 = {(c["k"], c["bs"], tuple(c["missing"])) for c in DEC}  # on the one-wave bitsliced kernel
    assert (10, 1 << 20, (0, 5, 10, 13)) in c3 and (10, 1 << 20, (0, 1, 2, 3)) in c3
    assert any(c["k"] == 10 and c["m"] == 4 and c["bs"] == 1 << 20 for c in ENC)


@pytest.mark.parametrize("case", ENC, ids=lambda c: f"{c['k']}-{c['m']}-{c['bs']}")
def test_encode_golden_on_kernel(case, mode):
    k, m, bs = case["k"], case["m"], case["bs"]
    frags = np.zeros((1, k + m, bs), dtype=np.uint8)
    frags[0, :k] = stripe_fragments(case["stripe"], k, bs)
    frags[0, k:] = 0xA5
    lay = D.Layout.alloc(k + m, bs, 1)
    lay.upload_stripes(frags)
    before = launches()
    D.rs_encode(k, m, lay)
    D.synchronize()
    _check_ran(mode, before)
    out = lay.download_stripes()[0]
    assert [sha(out[k + p]) for p in range(m)] == case["parity_sha256"]


@pytest.mark.parametrize("case", DEC, ids=lambda c: f"{c['k']}-{c['m']}-{c['bs']}-{c['missing']}-{c['garbage']}")
def test_decode_golden_on_kernel(case, mode):
    k, m, bs = case["k"], case["m"], case["bs"]
    data = stripe_fragments(case["stripe"], k, bs)
    par = (stripe_fragments(case["stripe"], m, bs, base=0xBAD0) if case["garbage"]
           else orc.encode(k, m, data))
    frags = np.concatenate([data, par])[None].copy()
    for i in case["missing"]:
        frags[0, i] = 0x5A
    lay = D.Layout.alloc(k + m, bs, 1)
    lay.upload_stripes(frags)
    before = launches()
    D.rs_decode(k, m, case["missing"], lay)
    D.synchronize()
    _check_ran(mode, before)
    out = lay.download_stripes()[0]
    assert {str(i): sha(out[i]) for i in case["missing"]} == case["out_sha256"]


def test_batched_c5_patterns_match_golden_stripe(mode):
    """The bench's shape: 32 stripes of k=20 m=8 4 MiB in one batch, every stripe a copy of the
    golden stripe, each rebuild pattern -- all 32 stripes' outputs equal the golden digests."""
    for case in [c for c in DEC if c["bs"] == 1 << 22 and not c["garbage"]]:
        k, m, bs, S = case["k"], case["m"], case["bs"], 8
        data = stripe_fragments(case["stripe"], k, bs)
        full = np.concatenate([data, orc.encode(k, m, data)])
        lay = D.Layout.alloc(k + m, bs, S)
        host = np.broadcast_to(full, (S, k + m, bs)).copy()
        host[:, case["missing"]] = 0x33
        lay.upload_stripes(host)
        before = launches()
        D.rs_decode(k, m, case["missing"], lay)
        D.synchronize()
        _check_ran(mode, before)
        out = lay.download_stripes()
        for s in range(S):
            assert {str(i): sha(out[s, i]) for i in case["missing"]} == case["out_sha256"], (case["missing"], s)
        del host, out
        lay.buf.free()


_SIGCHLD_SCRIPT = r"""
import ctypes as C, os, signal, sys
sys.path.insert(0, %(root)r); sys.path.insert(0, os.path.join(%(root)r, "tests"))
signal.signal(signal.SIGCHLD, signal.SIG_IGN)   # a host that ignores SIGCHLD: children auto-reaped
import numpy as np
import oracle_lib as orc
from ecdata import stripe_fragments
from liberasurecode_amd import _lib, device as D
d = _lib.dev()
d.ecamd_tune(b"bitslice", 2)
k, m, bs = 20, 8, 3 * 16384
lay = D.Layout.alloc(k + m, bs, 2)
lay.fill_splitmix(nfrags=k, stripe0=77)
D.rs_encode(k, m, lay)
D.synchronize()
f = d.ecamd_bitslice_launches; f.restype = C.c_longlong
out = lay.download_stripes()
for s in range(2):
    assert (out[s, k:] == orc.encode(k, m, stripe_fragments(77 + s, k, bs))).all()
print("launches", f(), "failed", d.ecamd_bitslice_wait())
"""


def test_compile_survives_ignored_sigchld(tmp_path):
    """With SIGCHLD ignored the compiler child is reaped by the kernel, so waitpid reports ECHILD:
    the entry must still pick up the code object the child wrote (not fall back to the LDS tables
    for the rest of the process)."""
    env = dict(os.environ, ECAMD_JIT_CACHE=str(tmp_path / "jit"))
    r = subprocess.run([sys.executable, "-c", _SIGCHLD_SCRIPT % {"root": ROOT}], capture_output=True,
                       text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    words = r.stdout.split()
    assert int(words[words.index("launches") + 1]) > 0, r.stdout
    assert int(words[words.index("failed") + 1]) == 0, r.stdout
