"""CPU: the product's flat-XOR planner (symbolic replay of xor_hd_decode & co.) against golden
vectors from the reference libXorcode (tests/golden/xor_codes.json).  Decode / reconstruct run on
INCONSISTENT random buffers, so the exact equations the reference picks are pinned, not just the
recovered data."""
import hashlib
import json
import os

import pytest

import xor_util as X

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "xor_codes.json")))
IDS = [f"{c['k']}_{c['m']}_{c['hd']}" for c in GOLD]


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_tables(case):
    pb, db = X.tables(case["k"], case["m"], case["hd"])
    assert list(pb) == case["parity_bms"]
    assert list(db) == case["data_bms"]


def test_invalid_codes_rejected():
    import ctypes as C
    from liberasurecode_amd import _lib
    pb, db = (C.c_uint * 8)(), (C.c_uint * 32)()
    for k, m, hd in [(4, 3, 3), (3, 3, 4), (16, 6, 3), (21, 6, 4), (11, 5, 3), (5, 6, 3), (4, 5, 4)]:
        assert _lib.host().ecamd_xor_code_tables(k, m, hd, pb, db) == -1


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_encode(case):
    k, m, hd, bs = case["k"], case["m"], case["hd"], case["bs"]
    bufs = X.case_buffers(k, m, bs, k * 100 + m * 10 + hd)
    rc, steps = X.plan(0, k, m, hd)
    assert rc == 0
    out = X.apply_plan(bufs, steps)
    assert sha(b"".join(x.tobytes() for x in out)) == case["encode_sha256"]


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_decode_all_patterns(case):
    k, m, hd, bs = case["k"], case["m"], case["hd"], case["bs"]
    pats = X.xor_patterns(k + m, case["patterns_seed"])
    h = hashlib.sha256()
    rcs = []
    for p in pats:
        bufs = X.case_buffers(k, m, bs, 7 + len(rcs))
        rc, steps = X.plan(1, k, m, hd, p, 1)
        rcs.append(rc)
        for x in X.apply_plan(bufs, steps):
            h.update(x.tobytes())
    assert rcs == case["decode_rc"]
    assert h.hexdigest() == case["decode_sha256"]


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_reconstruct_all_patterns(case):
    k, m, hd, bs = case["k"], case["m"], case["hd"], case["bs"]
    pats = X.xor_patterns(k + m, case["patterns_seed"])
    h = hashlib.sha256()
    rcs = []
    for p in pats:
        if len(p) > 3:
            continue
        for idx in sorted(set(p)):
            bufs = X.case_buffers(k, m, bs, 11 + len(rcs))
            rc, steps = X.plan(2, k, m, hd, p, idx)
            rcs.append(rc)
            for x in X.apply_plan(bufs, steps):
                h.update(x.tobytes())
    assert rcs == case["reconstruct_rc"]
    assert h.hexdigest() == case["reconstruct_sha256"]


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_fragments_needed(case):
    k, m, hd = case["k"], case["m"], case["hd"]
    pats = X.xor_patterns(k + m, case["patterns_seed"])
    fn = []
    for p in pats:
        if len(p) > 3:
            continue
        for split in range(len(p)):
            rc, lst = X.fragments_needed(k, m, hd, p[:split + 1], p[split + 1:])
            fn.append([rc, lst])
    assert fn[:40] == case["fragments_needed_head"]
    assert sha(json.dumps(fn, separators=(",", ":")).encode()) == case["fragments_needed_sha256"]
