#!/usr/bin/env python3
"""Generate tests/golden/*.json from the REFERENCE itself.

Runs in the build container only (needs /root/reference): `make -C oracle ref` compiles the
reference's liberasurecode_rs_vand.so.1 and libXorcode.so.1 from their own sources into
oracle/_ref/, and this script drives them through ctypes on splitmix64 inputs (tests/ecdata.py).
The committed JSON holds only data: inputs are described by their seeds, outputs by SHA-256
(full hex for tiny blocks).  Reference entry points used:
  make_systematic_matrix / liberasurecode_rs_vand_{encode,decode,reconstruct} / gaussj_inversion /
  square_matrix_multiply   (src/builtin/rs_vand/liberasurecode_rs_vand.c:58-558)
  init_xor_hd_code + xor_code_t ops / xor_reconstruct_one / xor_hd_fragments_needed
                           (src/builtin/xor_codes/xor_hd_code.c:209-708, xor_code.c:180-314)
"""
import ctypes as C
import hashlib
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from ecdata import EDGE_PATTERNS, splitmix_bytes, stripe_fragments  # noqa: E402

REF = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "_ref")
IP = C.POINTER(C.c_int)
CPP = C.POINTER(C.c_char_p)


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def load_rs():
    lib = C.CDLL(os.path.join(REF, "liberasurecode_rs_vand.so.1"))
    lib.make_systematic_matrix.restype = IP
    lib.make_systematic_matrix.argtypes = [C.c_int, C.c_int]
    lib.init_liberasurecode_rs_vand.argtypes = [C.c_int, C.c_int]
    for fn in ("liberasurecode_rs_vand_encode",):
        getattr(lib, fn).argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
    lib.liberasurecode_rs_vand_decode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, IP,
                                                  C.c_int, C.c_int]
    lib.liberasurecode_rs_vand_reconstruct.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                                       IP, C.c_int, C.c_int]
    lib.gaussj_inversion.argtypes = [IP, IP, C.c_int]
    lib.square_matrix_multiply.argtypes = [IP, IP, IP, C.c_int]
    return lib


class Bufs:
    """k+m host buffers addressable as char** arrays."""

    def __init__(self, arrs):
        self.arrs = [np.ascontiguousarray(a) for a in arrs]
        self.ptrs = [a.ctypes.data for a in self.arrs]

    def array(self, lo, hi):
        t = (C.c_void_p * (hi - lo))(*self.ptrs[lo:hi])
        return t


def gen_matrix(lib, k, m):
    lib.init_liberasurecode_rs_vand(k, m)
    p = lib.make_systematic_matrix(k, m)
    return [p[i] for i in range((k + m) * k)]


def as_ip(vals):
    return (C.c_int * len(vals))(*vals)


def rs_cases(lib):
    out = {"generators": {}, "gf": {}, "encode": [], "decode": [], "reconstruct": [],
           "inverse": []}
    dims = [(1, 1), (2, 1), (3, 3), (4, 2), (4, 4), (4, 8), (5, 1), (5, 2), (5, 3), (6, 6),
            (8, 4), (10, 4), (10, 5), (10, 10), (12, 1), (12, 2), (12, 3), (12, 6), (16, 16),
            (20, 8), (24, 8), (32, 32), (64, 64), (100, 28)]
    for k, m in dims:
        out["generators"][f"{k},{m}"] = gen_matrix(lib, k, m)

    # Field: all inverses (1x1 gaussj) and a product sample (1x1 square_matrix_multiply).
    inv = np.zeros(65536, dtype="<u2")
    a = (C.c_int * 1)()
    b = (C.c_int * 1)()
    pr = (C.c_int * 1)()
    for x in range(1, 65536):
        a[0] = x
        lib.gaussj_inversion(a, b, 1)
        inv[x] = b[0]
    out["gf"]["inverse_table_sha256"] = sha(inv.tobytes())
    rng = np.random.default_rng(1234)
    pairs = rng.integers(0, 65536, size=(20000, 2))
    prods = []
    for x, y in pairs:
        a[0] = int(x)
        b[0] = int(y)
        lib.square_matrix_multiply(a, b, pr, 1)
        prods.append(pr[0])
    out["gf"]["mul_pairs_seed1234_n20000"] = {"a": [int(v) for v in pairs[:256, 0]],
                                              "b": [int(v) for v in pairs[:256, 1]],
                                              "p": prods[:256],
                                              "sha256_all_u16le": sha(np.array(prods, "<u2").tobytes())}
    edge = [(0x8000, 2), (2, 0x8000), (0xFFFF, 0xFFFF), (1, 61447), (0x100B, 0x8000)]
    out["gf"]["edge"] = []
    for x, y in edge:
        a[0], b[0] = x, y
        lib.square_matrix_multiply(a, b, pr, 1)
        out["gf"]["edge"].append([x, y, pr[0]])

    case_id = [0]

    def next_id():
        case_id[0] += 1
        return case_id[0]

    def encode_case(k, m, bs, pattern=None):
        G = gen_matrix(lib, k, m)
        sid = next_id()
        if pattern is None:
            data = stripe_fragments(sid, k, bs)
        else:
            data = np.stack([EDGE_PATTERNS[pattern](bs) for _ in range(k)])
        par = np.zeros((m, bs), dtype=np.uint8)
        bufs = Bufs(list(data) + list(par))
        lib.liberasurecode_rs_vand_encode(as_ip(G), bufs.array(0, k), bufs.array(k, k + m), k, m, bs)
        rec = {"k": k, "m": m, "bs": bs, "stripe": sid, "pattern": pattern,
               "parity_sha256": [sha(bufs.arrs[k + p]) for p in range(m)]}
        if bs <= 64:
            rec["parity_hex"] = [bufs.arrs[k + p].tobytes().hex() for p in range(m)]
        out["encode"].append(rec)
        return sid, data, [bufs.arrs[k + p].copy() for p in range(m)]

    def frags_for(k, m, bs, garbage, sid):
        data = stripe_fragments(sid, k, bs)
        if garbage:
            par = stripe_fragments(sid, m, bs, base=0xBAD0)
        else:
            G = gen_matrix(lib, k, m)
            par = np.zeros((m, bs), dtype=np.uint8)
            bufs = Bufs(list(data) + list(par))
            lib.liberasurecode_rs_vand_encode(as_ip(G), bufs.array(0, k), bufs.array(k, k + m), k,
                                              m, bs)
            par = np.stack(bufs.arrs[k:])
        return list(data) + list(par)

    def decode_case(k, m, bs, missing, garbage):
        G = gen_matrix(lib, k, m)
        sid = next_id()
        frags = frags_for(k, m, bs, garbage, sid)
        for i in missing:
            frags[i] = np.zeros(bs, dtype=np.uint8)
        bufs = Bufs(frags)
        ml = as_ip(list(missing) + [-1])
        ret = lib.liberasurecode_rs_vand_decode(as_ip(G), bufs.array(0, k), bufs.array(k, k + m),
                                                k, m, ml, bs, 1)
        rec = {"k": k, "m": m, "bs": bs, "stripe": sid, "garbage": garbage,
               "missing": list(missing), "ret": ret,
               "out_sha256": {str(i): sha(bufs.arrs[i]) for i in missing}}
        if bs <= 64:
            rec["out_hex"] = {str(i): bufs.arrs[i].tobytes().hex() for i in missing}
        out["decode"].append(rec)

    def reconstruct_case(k, m, bs, missing, dest, garbage):
        G = gen_matrix(lib, k, m)
        sid = next_id()
        frags = frags_for(k, m, bs, garbage, sid)
        for i in missing:
            frags[i] = np.zeros(bs, dtype=np.uint8)
        bufs = Bufs(frags)
        ml = as_ip(list(missing) + [-1])
        ret = lib.liberasurecode_rs_vand_reconstruct(as_ip(G), bufs.array(0, k),
                                                     bufs.array(k, k + m), k, m, ml, dest, bs)
        rec = {"k": k, "m": m, "bs": bs, "stripe": sid, "garbage": garbage,
               "missing": list(missing), "dest": dest, "ret": ret,
               "out_sha256": sha(bufs.arrs[dest])}
        if bs <= 64:
            rec["out_hex"] = bufs.arrs[dest].tobytes().hex()
        out["reconstruct"].append(rec)

    # encode
    for k, m, bs in [(1, 1, 16), (2, 1, 16), (4, 2, 2), (4, 2, 64), (4, 2, 65536), (10, 4, 2),
                     (10, 4, 30), (10, 4, 64), (10, 4, 1000), (10, 4, 4096), (10, 4, 4098),
                     (10, 4, 1 << 20), (12, 6, 4096), (10, 10, 512), (4, 8, 512), (5, 3, 48),
                     (20, 8, 4096), (20, 8, 1 << 22), (16, 16, 2048), (32, 32, 1024),
                     (100, 28, 256)]:
        encode_case(k, m, bs)
    for p in EDGE_PATTERNS:
        encode_case(10, 4, 4096, p)
        encode_case(20, 8, 512, p)

    # decode (consistent and garbage inputs)
    dec = [(4, 2, 64, [0, 1]), (4, 2, 4096, [0, 4]), (4, 2, 4096, [5]), (4, 2, 65536, [2, 3]),
           (10, 4, 4096, [0, 1, 2, 3]), (10, 4, 4096, [0, 5, 10, 13]), (10, 4, 4096, [10, 11, 12, 13]),
           (10, 4, 4096, [3]), (10, 4, 4096, [13]), (10, 4, 4096, [9, 12]), (10, 4, 30, [1, 2, 11]),
           (10, 4, 1000, [4, 6, 7, 8]), (10, 4, 4096, [0, 1, 2, 3, 4]),
           (20, 8, 4096, list(range(8))), (20, 8, 4096, [0, 2, 4, 6, 20, 22, 24, 26]),
           (12, 6, 4096, [1, 3, 5, 13, 15, 17]), (10, 10, 512, list(range(0, 20, 2))),
           (4, 8, 512, [0, 1, 2, 3, 4, 5, 6, 7]), (1, 1, 16, [0]), (5, 3, 48, [4, 6, 7])]
    for k, m, bs, miss in dec:
        for garbage in (False, True):
            decode_case(k, m, bs, miss, garbage)
    decode_case(10, 4, 1 << 20, [0, 1, 2, 3], False)
    decode_case(20, 8, 1 << 22, list(range(8)), False)

    rec = [(10, 4, 4096, [0, 5, 10, 13]), (20, 8, 4096, list(range(8))),
           (10, 4, 4096, [1, 12]), (4, 2, 64, [1, 5]), (12, 6, 1000, [2, 7, 12, 14, 16]),
           (20, 8, 4096, [0, 2, 4, 6, 20, 22, 24, 26])]
    for k, m, bs, miss in rec:
        for d in miss:
            for garbage in (False, True):
                reconstruct_case(k, m, bs, miss, d, garbage)
    # destination not in the missing list (the reference computes it anyway)
    reconstruct_case(10, 4, 4096, [0, 5], 3, False)
    reconstruct_case(20, 8, 1 << 22, list(range(8)), 3, False)

    # Round 3: every pattern the bench times, pinned at full size, and shapes that take the
    # bitsliced 8-output kernel (>= 5 outputs, whole 16 KiB tiles, k <= 32) -- appended, so the
    # stripe ids of the cases above stay the same
    decode_case(10, 4, 1 << 20, [0, 5, 10, 13], False)                  # C3 mixed
    decode_case(20, 8, 1 << 22, [0, 2, 4, 6, 20, 22, 24, 26], False)    # C5 mixed
    decode_case(20, 8, 1 << 22, list(range(8)), True)                   # C5, inconsistent inputs
    decode_case(20, 8, 3 * 16384 + 2, [1, 3, 5, 7, 9, 21, 23, 25], True)  # tiles + ragged tail
    decode_case(12, 6, 65536, [1, 3, 5, 13, 15, 17], False)
    decode_case(24, 8, 65536, [0, 1, 2, 3, 24, 25, 26, 27], True)
    decode_case(10, 6, 65536, [0, 1, 2, 3, 4], False)                     # 5 outputs
    for k, m, bs in [(20, 8, 3 * 16384 + 2), (12, 6, 65536), (24, 8, 65536), (32, 8, 32768),
                     (10, 5, 65536)]:
        encode_case(k, m, bs)
    for d in (0, 6, 20, 26):
        reconstruct_case(20, 8, 1 << 22, [0, 2, 4, 6, 20, 22, 24, 26], d, False)
    reconstruct_case(10, 4, 1 << 20, [0, 5, 10, 13], 5, False)

    # decoding-matrix inverses for listed patterns
    for k, m, miss in [(10, 4, [0, 1, 2, 3]), (10, 4, [0, 5, 10, 13]), (20, 8, list(range(8))),
                       (4, 2, [1, 5]), (12, 6, [0, 2, 4, 13, 15, 17])]:
        G = gen_matrix(lib, k, m)
        rows = [i for i in range(k + m) if i not in miss][:k]
        dmat = [G[r * k + c] for r in rows for c in range(k)]
        a = as_ip(dmat)
        inv_ = (C.c_int * (k * k))()
        lib.gaussj_inversion(a, inv_, k)
        out["inverse"].append({"k": k, "m": m, "missing": miss, "rows": rows,
                               "inverse": [inv_[i] for i in range(k * k)]})
    return out


class XorCodeT(C.Structure):
    # include/xor_codes/xor_code.h:54-65
    _fields_ = [("k", C.c_int), ("m", C.c_int), ("hd", C.c_int),
                ("parity_bms", C.POINTER(C.c_uint)), ("data_bms", C.POINTER(C.c_uint)),
                ("decode", C.c_void_p), ("encode", C.c_void_p), ("fragments_needed", C.c_void_p)]


XOR_CODES = ([(3, 3, 3)] + [(k, 6, 3) for k in range(6, 16)] + [(k, 5, 3) for k in range(5, 11)]
             + [(k, 6, 4) for k in range(6, 21)] + [(k, 5, 4) for k in range(5, 11)])


def load_xor():
    lib = C.CDLL(os.path.join(REF, "libXorcode.so.1"))
    XP = C.POINTER(XorCodeT)
    lib.init_xor_hd_code.restype = XP
    lib.init_xor_hd_code.argtypes = [C.c_int, C.c_int, C.c_int]
    lib.xor_code_encode.argtypes = [XP, C.c_void_p, C.c_void_p, C.c_int]
    lib.xor_hd_decode.argtypes = [XP, C.c_void_p, C.c_void_p, IP, C.c_int, C.c_int]
    lib.xor_reconstruct_one.argtypes = [XP, C.c_void_p, C.c_void_p, IP, C.c_int, C.c_int]
    lib.xor_hd_fragments_needed.argtypes = [XP, IP, IP, IP]
    return lib


def xor_patterns(n, seed):
    """Deterministic erasure patterns: all of size 1 and 2, a sample of size 3 and 4 (the
    reference's own test covers every pattern below hd, test/builtin/xor_codes/test_xor_hd_code.c)."""
    import random
    rnd = random.Random(seed)
    pats = [list(p) for r in (1, 2) for p in itertools.combinations(range(n), r)]
    threes = [list(p) for p in itertools.combinations(range(n), 3)]
    pats += threes if len(threes) <= 400 else rnd.sample(threes, 400)
    fours = [list(p) for p in itertools.combinations(range(n), 4)]
    pats += rnd.sample(fours, min(40, len(fours)))
    # order inside a missing list matters to the reference (it walks the list): shuffle some
    for p in pats[::3]:
        rnd.shuffle(p)
    return pats


def xor_case_buffers(k, m, bs, seed):
    return [np.array(x) for x in stripe_fragments(seed, k + m, bs, base=0x50A)]


def xor_cases(lib, bs=48):
    """Per code: tables, encode (accumulating into non-zero parity), decode / reconstruct on
    INCONSISTENT random buffers for every listed pattern, fragments_needed."""
    out = []
    for k, m, hd in XOR_CODES:
        code = lib.init_xor_hd_code(k, m, hd)
        rec = {"k": k, "m": m, "hd": hd, "bs": bs,
               "parity_bms": [code.contents.parity_bms[i] for i in range(m)],
               "data_bms": [code.contents.data_bms[i] for i in range(k)]}
        bufs = xor_case_buffers(k, m, bs, k * 100 + m * 10 + hd)
        b = Bufs(bufs)
        lib.xor_code_encode(code, b.array(0, k), b.array(k, k + m), bs)
        rec["encode_sha256"] = sha(b"".join(x.tobytes() for x in b.arrs))
        pats = xor_patterns(k + m, k * 1000 + m * 10 + hd)
        rec["patterns_seed"] = k * 1000 + m * 10 + hd
        rcs, h = [], hashlib.sha256()
        for p in pats:
            bb = Bufs(xor_case_buffers(k, m, bs, 7 + len(rcs)))
            rc = lib.xor_hd_decode(code, bb.array(0, k), bb.array(k, k + m), as_ip(p + [-1]), bs, 1)
            rcs.append(rc)
            for x in bb.arrs:
                h.update(x.tobytes())
        rec["decode_rc"] = rcs
        rec["decode_sha256"] = h.hexdigest()
        rcs, h = [], hashlib.sha256()
        for p in pats:
            if len(p) > 3:
                continue
            for idx in sorted(set(p)):
                bb = Bufs(xor_case_buffers(k, m, bs, 11 + len(rcs)))
                rc = lib.xor_reconstruct_one(code, bb.array(0, k), bb.array(k, k + m),
                                             as_ip(p + [-1]), idx, bs)
                rcs.append(rc)
                for x in bb.arrs:
                    h.update(x.tobytes())
        rec["reconstruct_rc"] = rcs
        rec["reconstruct_sha256"] = h.hexdigest()
        fn = []
        for p in pats:
            if len(p) > 3:
                continue
            for split in range(len(p)):
                recon, excl = p[:split + 1], p[split + 1:]
                needed = (C.c_int * (k + m + 1))(*([-7] * (k + m + 1)))
                rc = lib.xor_hd_fragments_needed(code, as_ip(recon + [-1]), as_ip(excl + [-1]),
                                                 needed)
                lst = []
                if rc >= 0:
                    for i in range(k + m + 1):
                        if needed[i] == -1:
                            break
                        lst.append(needed[i])
                fn.append([rc, lst])
        rec["fragments_needed_head"] = fn[:40]
        rec["fragments_needed_sha256"] = sha(json.dumps(fn, separators=(",", ":")).encode())
        out.append(rec)
    return out


def main():
    import sys
    rs = load_rs()
    data = rs_cases(rs)
    with open(os.path.join(HERE, "rs_vand.json"), "w") as f:
        json.dump(data, f, separators=(",", ":"))
    print("rs_vand.json:", {k: len(v) for k, v in data.items()})
    if "--rs-only" in sys.argv:
        return
    xd = xor_cases(load_xor())
    with open(os.path.join(HERE, "xor_codes.json"), "w") as f:
        json.dump(xd, f, separators=(",", ":"))
    print("xor_codes.json:", len(xd), "codes")


if __name__ == "__main__":
    main()
