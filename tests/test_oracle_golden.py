"""Pin the CPU oracle (oracle/ec_oracle.c) to golden vectors produced by the reference itself
(tests/golden/make_golden.py drives the reference's liberasurecode_rs_vand.so.1 built from its own
sources).  No GPU needed."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as orc
from ecdata import EDGE_PATTERNS, stripe_fragments

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rs_vand.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("km", sorted(GOLD["generators"]))
def test_generator_matches_reference(km):
    k, m = map(int, km.split(","))
    assert orc.generator(k, m) == GOLD["generators"][km]


def test_generator_systematic_and_parity_row0_ones():
    # liberasurecode_rs_vand_test.c:36-50 (top is identity) and :277-286 (parity row 0 all ones)
    for km in GOLD["generators"]:
        k, m = map(int, km.split(","))
        G = np.array(GOLD["generators"][km]).reshape(k + m, k)
        assert (G[:k] == np.eye(k, dtype=int)).all()
        assert (G[k] == 1).all()


def test_field_inverse_table():
    lib = orc.lib()
    inv = np.zeros(65536, dtype="<u2")
    for x in range(1, 65536):
        inv[x] = lib.orc_gf_inv(x)
    assert sha(inv) == GOLD["gf"]["inverse_table_sha256"]
    # rs_galois_test.c:32-54: x * x^-1 == 1 and inverses are unique
    assert len(set(inv[1:].tolist())) == 65535


def test_field_products():
    lib = orc.lib()
    g = GOLD["gf"]["mul_pairs_seed1234_n20000"]
    for a, b, p in zip(g["a"], g["b"], g["p"]):
        assert lib.orc_gf_mul(a, b) == p
    rng = np.random.default_rng(1234)
    pairs = rng.integers(0, 65536, size=(20000, 2))
    prods = np.array([lib.orc_gf_mul(int(a), int(b)) for a, b in pairs], "<u2")
    assert sha(prods) == g["sha256_all_u16le"]
    for a, b, p in GOLD["gf"]["edge"]:
        assert lib.orc_gf_mul(a, b) == p


def _clmul_mod(a, b):
    r = 0
    for i in range(16):
        if (b >> i) & 1:
            r ^= a << i
    for i in range(31, 15, -1):
        if (r >> i) & 1:
            r ^= 0x1100B << (i - 16)
    return r


def test_field_is_carryless_mod_poly():
    # rs_galois_mult == carry-less multiplication mod 0x1100b
    lib = orc.lib()
    rng = np.random.default_rng(7)
    for a, b in rng.integers(0, 65536, size=(3000, 2)):
        assert lib.orc_gf_mul(int(a), int(b)) == _clmul_mod(int(a), int(b))


@pytest.mark.parametrize("case", GOLD["encode"], ids=lambda c: f"{c['k']}-{c['m']}-{c['bs']}-{c['pattern']}")
def test_encode_vectors(case):
    k, m, bs = case["k"], case["m"], case["bs"]
    if case["pattern"] is None:
        data = stripe_fragments(case["stripe"], k, bs)
    else:
        data = np.stack([EDGE_PATTERNS[case["pattern"]](bs) for _ in range(k)])
    par = orc.encode(k, m, data)
    assert [sha(p) for p in par] == case["parity_sha256"]
    if "parity_hex" in case:
        assert [p.tobytes().hex() for p in par] == case["parity_hex"]


def _frags(case):
    k, m, bs = case["k"], case["m"], case["bs"]
    data = stripe_fragments(case["stripe"], k, bs)
    if case["garbage"]:
        par = stripe_fragments(case["stripe"], m, bs, base=0xBAD0)
    else:
        par = orc.encode(k, m, data)
    frags = [np.array(x) for x in list(data) + list(par)]
    for i in case["missing"]:
        frags[i][:] = 0
    return frags


@pytest.mark.parametrize("case", GOLD["decode"],
                         ids=lambda c: f"{c['k']}-{c['m']}-{c['bs']}-{c['missing']}-{c['garbage']}")
def test_decode_vectors(case):
    frags = _frags(case)
    rc = orc.decode(case["k"], case["m"], frags, case["missing"])
    assert rc == case["ret"]
    for i, h in case["out_sha256"].items():
        assert sha(frags[int(i)]) == h


@pytest.mark.parametrize("case", GOLD["reconstruct"],
                         ids=lambda c: f"{c['k']}-{c['m']}-{c['missing']}-{c['dest']}-{c['garbage']}")
def test_reconstruct_vectors(case):
    frags = _frags(case)
    rc = orc.reconstruct(case["k"], case["m"], frags, case["missing"], case["dest"])
    assert rc == case["ret"]
    assert sha(frags[case["dest"]]) == case["out_sha256"]


@pytest.mark.parametrize("case", GOLD["inverse"], ids=lambda c: f"{c['k']}-{c['missing']}")
def test_inverse_vectors(case):
    k, m = case["k"], case["m"]
    G = orc.generator(k, m)
    dmat = orc.ints([G[r * k + c] for r in case["rows"] for c in range(k)])
    inv = orc.ints([0] * (k * k))
    orc.lib().orc_gauss_inverse(dmat, inv, k)
    assert list(inv) == case["inverse"]
