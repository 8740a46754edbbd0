"""CPU: pin the flat-XOR oracle (oracle/xor_oracle.py, a buffer-level restatement of the
reference's xor_code.c / xor_hd_code.c) against the reference's golden vectors, exactly as
tests/golden/make_golden.py drove the reference libXorcode.so.1."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

import xor_util as X

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import xor_oracle as XO  # noqa: E402

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "xor_codes.json")))
IDS = [f"{c['k']}_{c['m']}_{c['hd']}" for c in GOLD]


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_oracle_tables_encode(case):
    k, m, hd, bs = case["k"], case["m"], case["hd"], case["bs"]
    code = XO.XorCode(k, m, hd)
    assert code.pbm == case["parity_bms"] and code.dbm == case["data_bms"]
    bufs = X.case_buffers(k, m, bs, k * 100 + m * 10 + hd)
    code.encode(bufs)
    assert hashlib.sha256(b"".join(x.tobytes() for x in bufs)).hexdigest() == case["encode_sha256"]


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_oracle_decode_reconstruct(case):
    k, m, hd, bs = case["k"], case["m"], case["hd"], case["bs"]
    code = XO.XorCode(k, m, hd)
    pats = X.xor_patterns(k + m, case["patterns_seed"])
    h, rcs = hashlib.sha256(), []
    for p in pats:
        bufs = X.case_buffers(k, m, bs, 7 + len(rcs))
        rcs.append(code.decode(bufs, p, 1))
        for x in bufs:
            h.update(x.tobytes())
    assert rcs == case["decode_rc"]
    assert h.hexdigest() == case["decode_sha256"]
    h, rcs = hashlib.sha256(), []
    for p in pats:
        if len(p) > 3:
            continue
        for idx in sorted(set(p)):
            bufs = X.case_buffers(k, m, bs, 11 + len(rcs))
            rcs.append(code.reconstruct_one(bufs, p, idx))
            for x in bufs:
                h.update(x.tobytes())
    assert rcs == case["reconstruct_rc"]
    assert h.hexdigest() == case["reconstruct_sha256"]


def test_oracle_roundtrip_large():
    """Consistent stripes: every decodable pattern restores the original bytes."""
    rng = np.random.default_rng(5)
    for k, m, hd in [(10, 6, 4), (20, 6, 4), (10, 5, 3)]:
        data = rng.integers(0, 256, (k, 4099), dtype=np.uint8)
        parity = XO.encode_bytes(k, m, hd, data)
        full = list(data) + list(parity)
        code = XO.XorCode(k, m, hd)
        for p in X.xor_patterns(k + m, 1)[:200]:
            if len(p) >= hd:
                continue
            bufs = [x.copy() for x in full]
            for i in p:  # lost data is overwritten; lost parity is accumulated into, so zeroed
                bufs[i][:] = 0xA5 if i < k else 0
            assert code.decode(bufs, p, 1) == 0
            assert all((a == b).all() for a, b in zip(bufs, full)), p
