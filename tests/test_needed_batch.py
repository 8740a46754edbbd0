"""CPU: batched fragments_needed planning (ecamd_fragments_needed_batch) against
the reference: flat_xor_hd through the golden digests of xor_hd_fragments_needed
(tests/golden/xor_codes.json, from the reference libXorcode), rs_vand against a restatement of
liberasurecode_rs_vand_min_fragments (src/backends/rs_vand/liberasurecode_rs_vand.c:119-145)."""
import ctypes as C
import hashlib
import json
import os
import random

import pytest

import xor_util as X
from liberasurecode_amd import _lib

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "xor_codes.json")))


def batch(backend, k, m, hd, recon_lists, excl_lists):
    H = _lib.host()
    f = H.ecamd_fragments_needed_batch
    f.restype = C.c_int
    n = len(recon_lists)
    stride = k + m + 1
    flat_r, flat_x = [], []
    for r, x in zip(recon_lists, excl_lists):
        flat_r += list(r) + [-1] * (stride - len(r))
        flat_x += list(x) + [-1] * (stride - len(x))
    needed = (C.c_int * (n * (k + m + 1)))()
    rcs = (C.c_int * max(n, 1))()
    assert f(backend, k, m, hd, _lib.ints(flat_r), _lib.ints(flat_x), stride, n, needed, rcs) == 0
    out = []
    for s in range(n):
        row = list(needed[s * (k + m + 1):(s + 1) * (k + m + 1)])
        lst = row[:row.index(-1)] if -1 in row else row
        out.append([rcs[s], lst if rcs[s] >= 0 else []])
    return out


@pytest.mark.parametrize("case", GOLD, ids=[f"{c['k']}_{c['m']}_{c['hd']}" for c in GOLD])
def test_xor_batch_matches_reference_goldens(case):
    k, m, hd = case["k"], case["m"], case["hd"]
    recon, excl = [], []
    for p in X.xor_patterns(k + m, case["patterns_seed"]):
        if len(p) > 3:
            continue
        for split in range(len(p)):
            recon.append(p[:split + 1])
            excl.append(p[split + 1:])
    got = batch(3, k, m, hd, recon, excl)
    assert got[:40] == case["fragments_needed_head"]
    assert hashlib.sha256(json.dumps(got, separators=(",", ":")).encode()).hexdigest() == \
        case["fragments_needed_sha256"]


def rs_min_fragments(k, m, missing, exclude):
    gone = set(missing) | set(exclude)
    need = [i for i in range(k + m) if i not in gone][:k]
    return [0, need] if len(need) == k else [-1, []]


@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (20, 8), (1, 1)])
def test_rs_batch(k, m):
    rnd = random.Random(k * 10 + m)
    recon, excl = [], []
    for _ in range(500):
        n = rnd.randint(0, k + m)
        idx = rnd.sample(range(k + m), n)
        cut = rnd.randint(0, n)
        recon.append(idx[:cut])
        excl.append(idx[cut:])
    got = batch(6, k, m, 0, recon, excl)
    assert got == [rs_min_fragments(k, m, r, x) for r, x in zip(recon, excl)]


def test_bad_arguments():
    H = _lib.host()
    z = (C.c_int * 64)()
    assert H.ecamd_fragments_needed_batch(1, 4, 2, 0, z, z, 7, 1, z, z) == -1
    assert H.ecamd_fragments_needed_batch(3, 4, 3, 3, z, z, 8, 1, z, z) == -1
