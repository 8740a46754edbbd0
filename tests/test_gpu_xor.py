"""GPU parity of the drop-in libXorcode.so.1 (flat-XOR HD codes) against golden vectors from the
reference libXorcode, and the reference's own unit test run against our library."""
import ctypes as C
import hashlib
import json
import os
import subprocess

import pytest

import xor_util as X

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "xor_codes.json")))
IDS = [f"{c['k']}_{c['m']}_{c['hd']}" for c in GOLD]
IP = C.POINTER(C.c_int)


class XorCodeT(C.Structure):
    _fields_ = [("k", C.c_int), ("m", C.c_int), ("hd", C.c_int),
                ("parity_bms", C.POINTER(C.c_uint)), ("data_bms", C.POINTER(C.c_uint)),
                ("decode", C.c_void_p), ("encode", C.c_void_p), ("fragments_needed", C.c_void_p)]


@pytest.fixture(scope="module")
def lib():
    lib = C.CDLL(os.path.join(ROOT, "liberasurecode_amd", "lib", "libXorcode.so.1"))
    XP = C.POINTER(XorCodeT)
    lib.init_xor_hd_code.restype = XP
    lib.init_xor_hd_code.argtypes = [C.c_int, C.c_int, C.c_int]
    lib.xor_code_encode.argtypes = [XP, C.c_void_p, C.c_void_p, C.c_int]
    lib.xor_hd_decode.argtypes = [XP, C.c_void_p, C.c_void_p, IP, C.c_int, C.c_int]
    lib.xor_reconstruct_one.argtypes = [XP, C.c_void_p, C.c_void_p, IP, C.c_int, C.c_int]
    lib.xor_hd_fragments_needed.argtypes = [XP, IP, IP, IP]
    return lib


def ptrs(arrs, lo, hi):
    return (C.c_void_p * (hi - lo))(*[a.ctypes.data for a in arrs[lo:hi]])


def ints(v):
    return (C.c_int * len(v))(*v)


@pytest.mark.parametrize("case", GOLD, ids=IDS)
def test_libxorcode_golden(lib, case):
    k, m, hd, bs = case["k"], case["m"], case["hd"], case["bs"]
    code = lib.init_xor_hd_code(k, m, hd)
    assert bool(code)
    assert [code.contents.parity_bms[i] for i in range(m)] == case["parity_bms"]
    assert [code.contents.data_bms[i] for i in range(k)] == case["data_bms"]
    bufs = X.case_buffers(k, m, bs, k * 100 + m * 10 + hd)
    lib.xor_code_encode(code, ptrs(bufs, 0, k), ptrs(bufs, k, k + m), bs)
    assert hashlib.sha256(b"".join(x.tobytes() for x in bufs)).hexdigest() == case["encode_sha256"]
    pats = X.xor_patterns(k + m, case["patterns_seed"])
    rcs, h = [], hashlib.sha256()
    for p in pats:
        bb = X.case_buffers(k, m, bs, 7 + len(rcs))
        rcs.append(lib.xor_hd_decode(code, ptrs(bb, 0, k), ptrs(bb, k, k + m), ints(p + [-1]), bs, 1))
        for x in bb:
            h.update(x.tobytes())
    assert rcs == case["decode_rc"]
    assert h.hexdigest() == case["decode_sha256"]
    rcs, h = [], hashlib.sha256()
    for p in pats:
        if len(p) > 3:
            continue
        for idx in sorted(set(p)):
            bb = X.case_buffers(k, m, bs, 11 + len(rcs))
            rcs.append(lib.xor_reconstruct_one(code, ptrs(bb, 0, k), ptrs(bb, k, k + m),
                                               ints(p + [-1]), idx, bs))
            for x in bb:
                h.update(x.tobytes())
    assert rcs == case["reconstruct_rc"]
    assert h.hexdigest() == case["reconstruct_sha256"]


def test_reference_xor_unit_test_runs_on_our_library():
    """test/builtin/xor_codes/test_xor_hd_code.c (compiled from the reference source, linked by
    soname) against OUR libXorcode.so.1: every failure pattern below hd for every code."""
    exe = os.path.join(ROOT, "oracle", "_ref", "test_xor_hd_code_so")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built")
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.join(ROOT, "liberasurecode_amd", "lib"))
    probe = subprocess.run(["ldd", exe], env=env, capture_output=True, text=True).stdout
    assert os.path.join("liberasurecode_amd", "lib", "libXorcode.so.1") in probe
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert (r.stdout + r.stderr).count("Running") == 38


@pytest.mark.parametrize("k,m,hd,bs", [(10, 6, 4, (1 << 20) + 13), (20, 6, 4, 3), (15, 6, 3, 65537),
                                       (5, 5, 4, 1), (3, 3, 3, 777777)])
def test_libxorcode_vs_oracle_ragged(lib, k, m, hd, bs):
    """Large and odd blocksizes on inconsistent random buffers: every byte equals the buffer-level
    oracle (oracle/xor_oracle.py) for a sample of decode and reconstruct patterns."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import xor_oracle as XO
    code = lib.init_xor_hd_code(k, m, hd)
    oc = XO.XorCode(k, m, hd)
    rng = np.random.default_rng(k * 7 + bs)
    pats = X.xor_patterns(k + m, 99)
    sample = [pats[i] for i in sorted(set(rng.integers(0, len(pats), 12).tolist()))]
    base = [rng.integers(0, 256, bs, dtype=np.uint8) for _ in range(k + m)]
    bb, ob = [x.copy() for x in base], [x.copy() for x in base]
    lib.xor_code_encode(code, ptrs(bb, 0, k), ptrs(bb, k, k + m), bs)
    oc.encode(ob)
    assert all((a == b).all() for a, b in zip(bb, ob))
    for p in sample:
        bb, ob = [x.copy() for x in base], [x.copy() for x in base]
        rc = lib.xor_hd_decode(code, ptrs(bb, 0, k), ptrs(bb, k, k + m), ints(p + [-1]), bs, 1)
        assert rc == oc.decode(ob, p, 1)
        assert all((a == b).all() for a, b in zip(bb, ob)), p
        if len(p) <= 3:
            idx = p[-1]
            bb, ob = [x.copy() for x in base], [x.copy() for x in base]
            rc = lib.xor_reconstruct_one(code, ptrs(bb, 0, k), ptrs(bb, k, k + m), ints(p + [-1]),
                                         idx, bs)
            assert rc == oc.reconstruct_one(ob, p, idx)
            assert all((a == b).all() for a, b in zip(bb, ob)), (p, idx)
