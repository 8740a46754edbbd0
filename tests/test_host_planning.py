"""CPU tests of the product's host planning library (libecamd_host.so): generator, inversion,
decode / reconstruct maps and LDS split tables, checked against the reference's golden vectors.
The maps are applied with an independent numpy GF(2^16) (tests/gfnp.py), so these tests pin the
planning logic the GPU kernels are fed with, without a GPU."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import gfnp
from ecdata import stripe_fragments
from liberasurecode_amd import _lib

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rs_vand.json")))
H = _lib.host()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def generator(k, m):
    out = (C.c_int * ((k + m) * k))()
    assert H.ecamd_rs_generator(k, m, out) == 0
    return list(out)


@pytest.mark.parametrize("km", sorted(GOLD["generators"]))
def test_generator(km):
    k, m = map(int, km.split(","))
    assert generator(k, m) == GOLD["generators"][km]


def test_field():
    g = GOLD["gf"]["mul_pairs_seed1234_n20000"]
    for a, b, p in zip(g["a"], g["b"], g["p"]):
        assert H.ecamd_gf16_mul(a, b) == p
    inv = np.array([0] + [H.ecamd_gf16_inv(x) for x in range(1, 65536)], dtype="<u2")
    assert sha(inv) == GOLD["gf"]["inverse_table_sha256"]


@pytest.mark.parametrize("case", GOLD["inverse"], ids=lambda c: f"{c['k']}-{c['missing']}")
def test_inverse(case):
    k, m = case["k"], case["m"]
    G = generator(k, m)
    a = _lib.ints([G[r * k + c] for r in case["rows"] for c in range(k)])
    inv = (C.c_int * (k * k))()
    assert H.ecamd_gf16_invert(a, inv, k) == 0
    assert list(inv) == case["inverse"]


def _frags(case):
    k, m, bs = case["k"], case["m"], case["bs"]
    data = stripe_fragments(case["stripe"], k, bs)
    if case["garbage"]:
        par = stripe_fragments(case["stripe"], m, bs, base=0xBAD0)
    else:
        G = np.array(generator(k, m)).reshape(k + m, k)
        par = np.stack(gfnp.apply_map(G[k:], list(data)))
    frags = [np.array(x) for x in list(data) + list(par)]
    for i in case["missing"]:
        frags[i][:] = 0
    return frags


SMALL_DEC = [c for c in GOLD["decode"] if c["bs"] <= 65536]
SMALL_REC = [c for c in GOLD["reconstruct"] if c["bs"] <= 65536]


@pytest.mark.parametrize("case", SMALL_DEC,
                         ids=lambda c: f"{c['k']}-{c['m']}-{c['bs']}-{c['missing']}-{c['garbage']}")
def test_decode_map(case):
    k, m = case["k"], case["m"]
    G = _lib.ints(generator(k, m))
    inputs = (C.c_int * k)()
    outputs = (C.c_int * (k + m))()
    coeff = (C.c_int * ((k + m) * k))()
    nout = C.c_int()
    rc = H.ecamd_rs_decode_map(G, k, m, _lib.ints(case["missing"] + [-1]), 1, inputs, outputs,
                               coeff, C.byref(nout))
    assert rc == case["ret"]
    if rc != 0:
        return
    frags = _frags(case)
    rows = np.array(coeff[:nout.value * k]).reshape(nout.value, k)
    outs = gfnp.apply_map(rows, [frags[i] for i in inputs])
    got = {str(outputs[r]): sha(outs[r]) for r in range(nout.value)}
    assert got == case["out_sha256"]


@pytest.mark.parametrize("case", SMALL_REC,
                         ids=lambda c: f"{c['k']}-{c['m']}-{c['missing']}-{c['dest']}-{c['garbage']}")
def test_reconstruct_map(case):
    k, m = case["k"], case["m"]
    G = _lib.ints(generator(k, m))
    inputs = (C.c_int * k)()
    coeff = (C.c_int * k)()
    nin = C.c_int()
    rc = H.ecamd_rs_reconstruct_map(G, k, m, _lib.ints(case["missing"] + [-1]), case["dest"],
                                    inputs, C.byref(nin), coeff)
    assert rc == case["ret"]
    frags = _frags(case)
    n = nin.value
    if n == 0:
        out = np.zeros(case["bs"], dtype=np.uint8)
    else:
        out = gfnp.apply_map(np.array(coeff[:n]).reshape(1, n), [frags[inputs[j]] for j in range(n)])[0]
    assert sha(out) == case["out_sha256"]


@pytest.mark.parametrize("width", [2, 4, 8])
def test_split_tables(width):
    rng = np.random.default_rng(width)
    R, K = width, 3
    coeff = rng.integers(0, 65536, size=(R, K))
    coeff[0, 0] = 1
    coeff[-1, -1] = 0
    nbytes = K * 512 * width * 2
    img = np.zeros(nbytes, dtype=np.uint8)
    assert H.ecamd_split_tables(_lib.ints(coeff.reshape(-1)), R, K, 0, width, 0, K,
                                img.ctypes.data) == nbytes
    ent = img.view("<u2").reshape(K, 2, 256, width)
    for j in range(K):
        for x in rng.integers(0, 65536, size=64):
            for r in range(R):
                v = int(ent[j, 0, x & 0xFF, r]) ^ int(ent[j, 1, x >> 8, r])
                assert v == int(gfnp.mul_vec(int(coeff[r, j]), np.array([x], np.uint16))[0])
