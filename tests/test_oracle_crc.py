"""CPU: the checksum oracle (oracle/ec_oracle.c orc_crc32 / orc_crc32_alt) pinned to zlib (the
reference's payload / metadata checksum) and to the reference's own legacy checksum
src/utils/chksum/crc32.c compiled into oracle/_ref/libref_crc32.so; the legacy known-answer
headers of test/liberasurecode_test.c:2239-2315 pin it further through tests/test_frontend_cpu.py."""
import ctypes as C
import os
import zlib

import numpy as np
import pytest

import ec_api
import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "libref_crc32.so")
LENGTHS = [0, 1, 2, 3, 15, 16, 17, 59, 255, 1023, 1024, 1025, 65537]


def test_zlib():
    rng = np.random.default_rng(1)
    for n in LENGTHS:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.crc32(b) == zlib.crc32(b)


def test_legacy_vs_python_restatement():
    rng = np.random.default_rng(2)
    for n in LENGTHS[:9]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.crc32(b, legacy=True) == ec_api.crc32_legacy(b)


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built")
def test_legacy_vs_reference():
    ref = C.CDLL(REF)
    ref.liberasurecode_crc32_alt.restype = C.c_int
    ref.liberasurecode_crc32_alt.argtypes = [C.c_int, C.c_char_p, C.c_size_t]
    rng = np.random.default_rng(3)
    for n in LENGTHS + [1 << 20]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.crc32(b, legacy=True) == ref.liberasurecode_crc32_alt(0, b, n) & 0xFFFFFFFF
    # high-bit-heavy inputs exercise the sign extension
    b = bytes([0xFF] * 4096)
    assert O.crc32(b, legacy=True) == ref.liberasurecode_crc32_alt(0, b, 4096) & 0xFFFFFFFF
