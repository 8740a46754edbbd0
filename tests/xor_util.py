"""Helpers for the flat-XOR HD tests: pattern generation identical to tests/golden/make_golden.py
and a ctypes view of the product planner (libecamd_host.so)."""
import ctypes as C
import itertools
import random

import numpy as np

from ecdata import stripe_fragments
from liberasurecode_amd import _lib

XOR_CODES = ([(3, 3, 3)] + [(k, 6, 3) for k in range(6, 16)] + [(k, 5, 3) for k in range(5, 11)]
             + [(k, 6, 4) for k in range(6, 21)] + [(k, 5, 4) for k in range(5, 11)])


def xor_patterns(n, seed):
    rnd = random.Random(seed)
    pats = [list(p) for r in (1, 2) for p in itertools.combinations(range(n), r)]
    threes = [list(p) for p in itertools.combinations(range(n), 3)]
    pats += threes if len(threes) <= 400 else rnd.sample(threes, 400)
    fours = [list(p) for p in itertools.combinations(range(n), 4)]
    pats += rnd.sample(fours, min(40, len(fours)))
    for p in pats[::3]:
        rnd.shuffle(p)
    return pats


def case_buffers(k, m, bs, seed):
    return [np.array(x) for x in stripe_fragments(seed, k + m, bs, base=0x50A)]


def tables(k, m, hd):
    pb = (C.c_uint * m)()
    db = (C.c_uint * k)()
    assert _lib.host().ecamd_xor_code_tables(k, m, hd, pb, db) == 0
    return pb, db


def plan(op, k, m, hd, missing=(), arg=0):
    """(rc, [(output_index, source_mask)]) from the product planner."""
    H = _lib.host()
    H.ecamd_xor_plan.restype = C.c_int
    pb, db = tables(k, m, hd)
    outs = (C.c_int * (k + m))()
    srcs = (C.c_uint64 * (k + m))()
    n = C.c_int()
    rc = H.ecamd_xor_plan(op, k, m, hd, pb, db, _lib.ints(list(missing) + [-1]), arg, outs, srcs,
                          C.byref(n))
    return rc, [(outs[i], srcs[i]) for i in range(n.value)]


def apply_plan(bufs, steps):
    """Evaluate a plan on host buffers (every output from the ORIGINAL contents)."""
    orig = [b.copy() for b in bufs]
    out = [b.copy() for b in bufs]
    for idx, mask in steps:
        acc = np.zeros_like(orig[0])
        for j in range(len(orig)):
            if mask >> j & 1:
                acc ^= orig[j]
        out[idx] = acc
    return out


def fragments_needed(k, m, hd, recon, excl):
    pb, db = tables(k, m, hd)
    needed = (C.c_int * (k + m + 1))(*([-7] * (k + m + 1)))
    rc = _lib.host().ecamd_xor_fragments_needed(k, m, hd, pb, db, _lib.ints(list(recon) + [-1]),
                                               _lib.ints(list(excl) + [-1]), needed)
    lst = []
    if rc >= 0:
        for i in range(k + m + 1):
            if needed[i] == -1:
                break
            lst.append(needed[i])
    return rc, lst
