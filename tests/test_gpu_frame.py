"""GPU parity of the device-resident framed path (include/ecamd.h "on-device framing"):
zlib / legacy CRC32 on the device against the oracle, and whole fragments (80-byte header +
payload) against the framing restatement of tests/ec_api.py (pinned to the reference's
known-answer headers, test/liberasurecode_test.c:2239-2315) with parity from the oracles."""
import os
import subprocess
import sys
import zlib

import numpy as np
import pytest

import ec_api
import oracle_lib as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import xor_oracle as XO  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from liberasurecode_amd import _lib, frame
    assert _lib.dev().ecamd_init() == 0
    return frame


@pytest.fixture(params=[(8, 0, 0), (7, 0, 0), (6, 0, 0), (5, 0, 0), (4, 0, 0), (8, 1, 0), (6, 1, 0),
                        (4, 1, 0), (5, 1, 32), (5, 1, 64), (4, 0, 8)],
                ids=["byte_tables", "mixed3", "mixed2", "mixed1", "nibble_tables", "byte_pos",
                     "mixed2_pos", "nibble_pos", "mixed1_pos_span32", "mixed1_pos_span64",
                     "nibble_span8"])
def bits(request):
    from liberasurecode_amd import _lib
    d = _lib.dev()
    _lib.check(d.ecamd_tune(b"crc_bits", request.param[0]), "tune")
    _lib.check(d.ecamd_tune(b"crc_pos", request.param[1]), "tune")
    _lib.check(d.ecamd_tune(b"crc_span_kib", request.param[2]), "tune")
    yield request.param[0] * 100 + request.param[1] * 10 + request.param[2]
    for key, default in ((b"crc_bits", 0), (b"crc_pos", 1), (b"crc_span_kib", 0)):
        d.ecamd_tune(key, default)


CRC_LENGTHS = [0, 1, 15, 16, 17, 100, 1023, 1024, 1025, 4096, 16383, 16384, 16400, 65536 + 13,
               (1 << 20), (1 << 20) + 7, 3 * (1 << 20) + 1]


def test_crc32_lengths(F, bits):
    from liberasurecode_amd.device import DeviceBuffer
    rng = np.random.default_rng(bits)
    for n in CRC_LENGTHS:
        nbuf = 5
        stride = max((n + 15) // 16 * 16, 16)
        host = rng.integers(0, 256, nbuf * stride, dtype=np.uint8)
        d = DeviceBuffer(host.size)
        d.upload(host)
        got = F.crc32(d, nbuf, n, stride)
        want = [zlib.crc32(host[i * stride:i * stride + n].tobytes()) for i in range(nbuf)]
        assert got.tolist() == want, n
        if n <= (1 << 20):
            got = F.crc32(d, nbuf, n, stride, legacy=True)
            want = [O.crc32(host[i * stride:i * stride + n], legacy=True) for i in range(nbuf)]
            assert got.tolist() == want, ("legacy", n)


def test_crc32_edge_patterns(F):
    from liberasurecode_amd.device import DeviceBuffer
    n = 70000
    for fill in (0x00, 0xFF, 0x80):
        host = np.full(n, fill, dtype=np.uint8)
        d = DeviceBuffer(n + 16)
        d.upload(host)
        assert F.crc32(d, 1, n, (n + 15) // 16 * 16)[0] == zlib.crc32(host.tobytes())
        assert F.crc32(d, 1, n, (n + 15) // 16 * 16, legacy=True)[0] == O.crc32(host, legacy=True)


def expected_stripe(backend, k, m, hd, obj: bytes, ct, legacy=False):
    """The fragments liberasurecode_encode returns for obj (restated)."""
    a = k * (4 if backend == ec_api.EC_BACKEND_FLAT_XOR_HD else 2)
    bs = (len(obj) + a - 1) // a * a // k
    data = np.zeros((k, bs), dtype=np.uint8)
    flat = np.frombuffer(obj, dtype=np.uint8)
    data.reshape(-1)[:len(flat)] = flat
    if backend == ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND:
        parity = O.encode(k, m, data)
    else:
        parity = XO.encode_bytes(k, m, hd, data)
    frags = []
    for i, payload in enumerate(list(data) + list(parity)):
        p = payload.tobytes()
        if ct == ec_api.CHKSUM_CRC32 and legacy:
            hdr = ec_api.expected_header(i, bs, len(obj), backend, ct, b"", with_crc=False,
                                         legacy=True)
            hdr = _with_crc(hdr, O.crc32(p, legacy=True), legacy=True)
        else:
            hdr = ec_api.expected_header(i, bs, len(obj), backend, ct, p, legacy=legacy)
        frags.append(hdr + p)
    return frags


def _with_crc(hdr, crc, legacy):
    import struct
    meta = bytearray(hdr[:59])
    meta[21:25] = struct.pack("<I", crc)
    mcrc = O.crc32(bytes(meta), legacy=True) if legacy else zlib.crc32(bytes(meta))
    return bytes(meta) + hdr[59:67] + struct.pack("<I", mcrc) + hdr[71:]


CODES = [("rs", 4, 2, 0), ("rs", 10, 4, 0), ("rs", 20, 8, 0), ("rs", 1, 1, 0),
         ("xor", 3, 3, 3), ("xor", 10, 6, 4), ("xor", 10, 5, 3)]
SIZES = [1, 1000, 12345, 65536 * 4, 1048576 + 4]


def _backend(name):
    return (ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND if name == "rs"
            else ec_api.EC_BACKEND_FLAT_XOR_HD)


def _objects(S, size, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(S)]


def _upload_objects(objs, stride):
    from liberasurecode_amd.device import DeviceBuffer
    host = np.zeros((len(objs), stride), dtype=np.uint8)
    for s, o in enumerate(objs):
        host[s, :len(o)] = np.frombuffer(o, dtype=np.uint8)
    d = DeviceBuffer(max(host.size, 16))
    d.upload(host.reshape(-1))
    return d


@pytest.mark.parametrize("code", CODES, ids=[f"{c[0]}_{c[1]}_{c[2]}" for c in CODES])
@pytest.mark.parametrize("ct", [ec_api.CHKSUM_CRC32, ec_api.CHKSUM_NONE])
def test_frame_encode_bytes(F, code, ct):
    name, k, m, hd = code
    be = _backend(name)
    for size in SIZES:
        if k == 20 and size > 65536 * 4:
            continue
        S = 3
        objs = _objects(S, size, size + k)
        fb = F.FrameBatch(be, k, m, size, S, hd=hd or 3, checksum=ct)
        d_obj = _upload_objects(objs, fb.obj_stride)
        fb.encode(d_obj)
        got = fb.fragments()
        for s in range(S):
            want = expected_stripe(be, k, m, hd, objs[s], ct)
            for i in range(k + m):
                assert got[s, i].tobytes() == want[i], (size, s, i)


def test_frame_encode_legacy_crc(F, monkeypatch):
    monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", "1")
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    for size in (999, 300000):
        objs = _objects(2, size, 77)
        fb = F.FrameBatch(be, 4, 2, size, 2)
        fb.encode(_upload_objects(objs, fb.obj_stride))
        got = fb.fragments()
        for s in range(2):
            want = expected_stripe(be, 4, 2, 0, objs[s], ec_api.CHKSUM_CRC32, legacy=True)
            for i in range(6):
                assert got[s, i].tobytes() == want[i], (size, s, i)


def test_frame_md5_type_stored_not_computed(F):
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    objs = _objects(1, 5000, 5)
    fb = F.FrameBatch(be, 4, 2, 5000, 1, checksum=ec_api.CHKSUM_MD5)
    fb.encode(_upload_objects(objs, fb.obj_stride))
    got = fb.fragments()
    want = expected_stripe(be, 4, 2, 0, objs[0], ec_api.CHKSUM_MD5)
    assert all(got[0, i].tobytes() == want[i] for i in range(6))


DECODE = [("rs", 10, 4, 0, [0, 1, 2, 3]), ("rs", 10, 4, 0, [0, 5, 10, 13]),
          ("rs", 20, 8, 0, [0, 2, 4, 6, 20, 22, 24, 26]), ("rs", 4, 2, 0, [4, 5]),
          ("xor", 10, 6, 4, [0, 1, 2]), ("xor", 3, 3, 3, [1, 4]), ("xor", 10, 5, 3, [9, 12])]


@pytest.mark.parametrize("case", DECODE, ids=[f"{c[0]}_{c[1]}_{c[2]}_{len(c[4])}" for c in DECODE])
def test_frame_decode_roundtrip(F, case):
    from liberasurecode_amd.device import DeviceBuffer
    name, k, m, hd, missing = case
    be = _backend(name)
    for size in (777, 1048576 * 2 + 6):
        S = 2
        objs = _objects(S, size, 3 + size)
        fb = F.FrameBatch(be, k, m, size, S, hd=hd or 3)
        fb.encode(_upload_objects(objs, fb.obj_stride))
        frags = fb.fragments()
        for i in missing:
            frags[:, i, :] = 0xA5  # lost: garbage in the slot
        fb.upload_fragments(frags)
        out = DeviceBuffer(fb.obj_stride * S)
        fb.decode(missing, out)
        host = out.download(fb.obj_stride * S).reshape(S, fb.obj_stride)
        for s in range(S):
            assert host[s, :size].tobytes() == objs[s], (size, s)


RECON = [("rs", 10, 4, 0, [3, 11], 3), ("rs", 10, 4, 0, [3, 11], 11), ("rs", 20, 8, 0,
         list(range(8)), 5), ("xor", 10, 6, 4, [2, 12, 5], 12), ("xor", 3, 3, 3, [0, 3], 0)]


@pytest.mark.parametrize("case", RECON, ids=[f"{c[0]}_{c[1]}_{c[2]}_d{c[5]}" for c in RECON])
def test_frame_reconstruct_byte_equal(F, case):
    """liberasurecode_test.c:1331: a reconstructed fragment equals the original, header
    included."""
    name, k, m, hd, missing, dest = case
    be = _backend(name)
    size = 1048576 + 12
    S = 2
    objs = _objects(S, size, 11)
    fb = F.FrameBatch(be, k, m, size, S, hd=hd or 3)
    fb.encode(_upload_objects(objs, fb.obj_stride))
    orig = fb.fragments()
    frags = orig.copy()
    for i in missing:
        frags[:, i, :] = 0x5A
    fb.upload_fragments(frags)
    fb.reconstruct(missing, dest)
    got = fb.fragments()
    assert np.array_equal(got[:, dest], orig[:, dest])


def test_frame_verify(F):
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    size = 10 * 1048576
    S = 2
    objs = _objects(S, size, 21)
    fb = F.FrameBatch(be, 10, 4, size, S)
    fb.encode(_upload_objects(objs, fb.obj_stride))
    st, crc = fb.verify()
    assert not st.any()
    frags = fb.fragments()
    for s in range(S):
        for i in range(14):
            assert crc[s, i] == zlib.crc32(frags[s, i, 80:].tobytes())
    frags[0, 3, 80 + 123456] ^= 1      # payload bit flip
    frags[1, 7, 4] ^= 1                # header: size field (metadata checksum breaks too)
    frags[1, 9, 60] ^= 1               # magic
    frags[0, 12, 0] = 11               # idx (metadata checksum breaks too)
    fb.upload_fragments(frags)
    st, _ = fb.verify()
    assert st[0, 3] == 16
    assert st[1, 7] & 8 and st[1, 7] & 2
    assert st[1, 9] & 1
    assert st[0, 12] & 4 and st[0, 12] & 2
    mask = np.ones_like(st, dtype=bool)
    for s, i in [(0, 3), (1, 7), (1, 9), (0, 12)]:
        mask[s, i] = False
    assert not st[mask].any()


def test_frame_large_c3_roundtrip(F):
    """BASELINE C3 shape: 10 MiB objects, RS(10,4), CRC32; decode with 4 data fragments lost."""
    from liberasurecode_amd.device import DeviceBuffer
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    size, S = 10 * 1048576, 8
    objs = _objects(S, size, 99)
    fb = F.FrameBatch(be, 10, 4, size, S)
    fb.encode(_upload_objects(objs, fb.obj_stride))
    frags = fb.fragments()
    for s in (0, S - 1):
        want = expected_stripe(be, 10, 4, 0, objs[s], ec_api.CHKSUM_CRC32)
        assert all(frags[s, i].tobytes() == want[i] for i in range(14))
    frags[:, :4] = 0
    fb.upload_fragments(frags)
    out = DeviceBuffer(fb.obj_stride * S)
    fb.decode([0, 1, 2, 3], out)
    host = out.download(fb.obj_stride * S).reshape(S, fb.obj_stride)
    assert all(host[s, :size].tobytes() == objs[s] for s in range(S))


def test_frame_errors(F):
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    d = _lib.dev()
    buf = DeviceBuffer(1 << 16)
    # unsupported backend, bad xor code, too many missing, bad stride
    assert d.ecamd_frame_encode(1, 4, 2, 0, 2, buf.ptr, 4096, 4000, buf.ptr, 6 * 2048, 2048, 1,
                                None) < 0
    assert d.ecamd_frame_encode(3, 4, 3, 3, 2, buf.ptr, 4096, 4000, buf.ptr, 7 * 2048, 2048, 1,
                                None) < 0
    assert d.ecamd_frame_encode(6, 4, 2, 0, 2, buf.ptr, 4096, 4000, buf.ptr, 6 * 1072, 1072, 1,
                                None) < 0  # frag_stride < 80 + 1000 rounded
    assert d.ecamd_frame_decode(6, 4, 2, 0, _lib.ints([0, 1, 2, -1]), buf.ptr, 6 * 2048, 2048, 1,
                                buf.ptr, 4096, 4000, None) < 0


@pytest.mark.parametrize("k,m", [(10, 4), (20, 8), (10, 12), (4, 2)])
def test_frame_encode_copy_through_matches_split(F, k, m):
    """Objects that fill the k payloads exactly take the copy-through launch (data read from the
    object and written to the payloads while the parity is computed); its fragments equal the
    split-then-encode path's and the restated reference framing."""
    from liberasurecode_amd import _lib
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    size = k * 65536
    objs = _objects(3, size, k * 31 + m)
    out = []
    for unfused in (0, 1):
        _lib.check(_lib.dev().ecamd_tune(b"frame_unfused", unfused), "tune")
        fb = F.FrameBatch(be, k, m, size, 3)
        fb.encode(_upload_objects(objs, fb.obj_stride))
        out.append(fb.fragments())
    _lib.dev().ecamd_tune(b"frame_unfused", 0)
    assert np.array_equal(out[0], out[1])
    want = expected_stripe(be, k, m, 0, objs[2], ec_api.CHKSUM_CRC32)
    assert all(out[0][2, i].tobytes() == want[i] for i in range(k + m))


@pytest.mark.parametrize("k,m,missing", [(10, 4, [0, 1, 2, 3]), (10, 4, [0, 5, 10, 13]),
                                         (20, 8, [0, 2, 4, 6, 20, 22, 24, 26]), (10, 12, [1, 2, 3, 4, 5, 6, 7, 8, 9]),
                                         (4, 2, [3])])
def test_frame_decode_join_matches_split(F, k, m, missing):
    """Objects that fill the payloads exactly decode in one launch (lost data computed into the
    object, surviving data copied through); same objects as decode-then-join."""
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    size, S = k * 65536, 3
    objs = _objects(S, size, 17 * k + m)
    for unfused in (0, 1):
        _lib.check(_lib.dev().ecamd_tune(b"frame_unfused", unfused), "tune")
        fb = F.FrameBatch(be, k, m, size, S)
        fb.encode(_upload_objects(objs, fb.obj_stride))
        frags = fb.fragments()
        frags[:, missing] = 0x3C
        fb.upload_fragments(frags)
        out = DeviceBuffer(fb.obj_stride * S)
        fb.decode(missing, out)
        host = out.download(fb.obj_stride * S).reshape(S, fb.obj_stride)
        assert all(host[s, :size].tobytes() == objs[s] for s in range(S)), unfused
        survivors = [i for i in range(k + m) if i not in missing]
        assert np.array_equal(fb.fragments()[:, survivors], frags[:, survivors])
    _lib.dev().ecamd_tune(b"frame_unfused", 0)


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("bs", [100, 1000, 65536, (1 << 20) + 6, 3 * (1 << 20)])
@pytest.mark.parametrize("legacy", [0, 1])
def test_percall_crc_handoff(F, bs, legacy, fuse):
    """ecamd_percall_crc_*: while armed, the per-call host path checksums every input and output
    fragment on the GPU (chunk CRCs combined on the host); each equals zlib / the legacy CRC of
    the final bytes.  This is what liberasurecode.so.1 stamps into the headers.  From 16 KiB of
    fragments (below, the inputs' zlib CRC32s are taken on the host during the call); fragments of at most 64 KiB fold the checksums into the
    small-launch codec kernel (ecamd_map_apply_strided_crc); with that off (fuse "0", run in a child:
    ECAMD_PERCALL_FUSE_CRC is read once) the separate ecamd_crc32 pass serves them."""
    if fuse == "0":
        here = os.path.dirname(os.path.abspath(__file__))
        env = dict(os.environ, ECAMD_PERCALL_FUSE_CRC="0",
                   PYTHONPATH=os.pathsep.join([os.path.dirname(here), here, os.environ.get("PYTHONPATH", "")]))
        r = subprocess.run([sys.executable, "-c", f"import test_gpu_frame as t; t._crc_handoff({bs}, {legacy}, False)"],
                           cwd=os.path.dirname(os.path.abspath(__file__)), env=env, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        return
    _crc_handoff(bs, legacy, True)


def _crc_handoff(bs, legacy, fused):
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    import ctypes as C
    from liberasurecode_amd import _lib
    d = _lib.dev()
    k, m = 10, 4
    rng = np.random.default_rng(bs + legacy)
    data = [rng.integers(0, 256, bs, dtype=np.uint8) for _ in range(k)]
    parity = [np.zeros(bs, dtype=np.uint8) for _ in range(m)]
    G = O.generator(k, m)
    rows = G[k * k:]
    inp = (C.c_void_p * k)(*[x.ctypes.data for x in data])
    out = (C.c_void_p * m)(*[x.ctypes.data for x in parity])
    d.ecamd_percall_crc_arm(legacy)
    try:
        assert d.ecamd_host_map_apply(_lib.ints(rows), m, k, inp, out, bs) == 0
        big = bs * (k + m) >= 16 << 10
        for i, buf in enumerate(data + parity):
            c = C.c_uint32()
            found = d.ecamd_percall_crc_lookup(buf.ctypes.data, bs, C.byref(c)) == 0
            # below 16 KiB of fragments no GPU checksum: the inputs' zlib CRC32s are taken on the host while
            # the kernel runs (not the legacy CRC), the outputs' are left to the caller
            assert found == (big or (i < k and not legacy)), (i, bs, legacy)
            if found:
                assert c.value == O.crc32(buf, legacy=bool(legacy))
        c = C.c_uint32()
        assert d.ecamd_percall_crc_lookup(data[0].ctypes.data, bs + 1, C.byref(c)) != 0
    finally:
        d.ecamd_percall_crc_disarm()
    assert np.array_equal(np.stack(parity), O.encode(k, m, np.stack(data)))


@pytest.mark.parametrize("k,m,bs,S", [(10, 4, 1 << 20, 3), (4, 2, 8192, 7), (6, 3, 3 * 8192, 5),
                                      (8, 4, 64 * 8192, 2), (3, 2, 40 * 8192, 9), (12, 6, 16384, 4),
                                      (20, 8, 4 * 8192, 3)])
@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("mb", [1, 4, "nib", "nib1", "bs", "bs2", "bs4", "bsl", "bsn", "bsn4", "bsw"])
def test_frame_encode_fused_crc_matches_split(F, k, m, bs, S, legacy, mb, monkeypatch):
    """CHKSUM_CRC32 framed encode of objects that fill the payloads: the fused launch (codec +
    copy-through + payload checksums folded per range) against the copy-through encode + separate
    CRC pass, and the restated reference framing for one stripe (zlib and legacy CRC)."""
    from liberasurecode_amd import _lib
    if legacy:
        monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", "1")
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    size = k * bs
    objs = _objects(S, size, k * 7 + m + bs)
    out = []
    bsv = str(mb).startswith("bs")
    # the bitsliced crc variant: bsw its one-wave form (the default, knob frame_crc_wave) over whole
    # 4 KiB tiles, the other bs* the 16 KiB-tile form (frame_crc_wave 0) over whole 16 KiB tiles; other
    # payload sizes fall back to the LDS-table fused kernel or the copy-through encode + CRC pass
    bs_fits = m <= 8 and bs % (4096 if mb == "bsw" else 16384) == 0
    _lib.check(_lib.dev().ecamd_tune(b"frame_crc_wave", -1 if mb == "bsw" else 0), "tune")
    _lib.check(_lib.dev().ecamd_tune(b"frame_crc_mb", {"nib": 4, "nib1": 1}.get(mb, 4 if bsv else mb)), "tune")
    _lib.check(_lib.dev().ecamd_tune(b"frame_crc_pos", {"bs2": 2, "bs4": 4, "bsl": 0, "bsn": 0, "bsn4": 4}.get(mb, 1)),
               "tune")
    _lib.check(_lib.dev().ecamd_tune(b"frame_crc_lane", 1 if mb in ("bsl", "bsn", "bsn4") else 0), "tune")
    # bsn*: the crc variant's piece tables as nibble fields (knob frame_crc_bs_nib)
    _lib.check(_lib.dev().ecamd_tune(b"frame_crc_bs_nib", 1 if mb in ("bsn", "bsn4") else 0), "tune")
    _lib.check(_lib.dev().ecamd_tune(b"frame_crc_nib", 1 if mb in ("nib", "nib1") else 0), "tune")
    _lib.check(_lib.dev().ecamd_tune(b"frame_crc_bs", 1 if bsv else 0), "tune")
    _lib.check(_lib.dev().ecamd_tune(b"bitslice", 2 if bsv else 1), "tune")
    try:
        for fused in (1, 0):
            _lib.check(_lib.dev().ecamd_tune(b"frame_crc_fused", fused), "tune")
            n0 = _bs_launches()
            fb = F.FrameBatch(be, k, m, size, S)
            fb.encode(_upload_objects(objs, fb.obj_stride))
            out.append(fb.fragments())
            if fused and bsv and bs_fits:
                assert _bs_launches() > n0, "the bitsliced crc variant did not run"
            elif fused and bsv and m <= 4:
                assert _bs_launches() == n0, "a bitsliced kernel ran on a shape it does not take"
    finally:
        _lib.dev().ecamd_tune(b"frame_crc_fused", 1)
        _lib.dev().ecamd_tune(b"frame_crc_mb", 0)
        _lib.dev().ecamd_tune(b"frame_crc_nib", -1)  # the library default
        _lib.dev().ecamd_tune(b"frame_crc_bs", -1)
        _lib.dev().ecamd_tune(b"frame_crc_pos", -1)
        _lib.dev().ecamd_tune(b"frame_crc_lane", -1)
        _lib.dev().ecamd_tune(b"frame_crc_bs_nib", -1)
        _lib.dev().ecamd_tune(b"frame_crc_wave", -1)
        _lib.dev().ecamd_tune(b"bitslice", 1)
    assert np.array_equal(out[0], out[1])
    if bs <= (1 << 16):
        want = expected_stripe(be, k, m, 0, objs[S - 1], ec_api.CHKSUM_CRC32, legacy=legacy)
        assert all(out[0][S - 1, i].tobytes() == want[i] for i in range(k + m))


@pytest.mark.parametrize("k,m,size", [(10, 4, 1 << 20), (10, 4, 3 * (1 << 20) + 7), (4, 2, 3 * 4 * 16384 - 6),
                                      (6, 3, 6 * 16384 + 6 * 100), (12, 6, 65536 * 12 - 24), (20, 8, 20 * 40000),
                                      (10, 4, 10 * (5 * 16384 + 16)), (3, 2, 3 * 16384 - 2)])
@pytest.mark.parametrize("legacy", [False, True])
def test_frame_encode_cover_crc_matches(F, k, m, size, legacy, monkeypatch):
    """CHKSUM_CRC32 framed encode of payloads that are not whole 16 KiB tiles (Swift's 1 MiB segments,
    bs = 104858): the bitsliced crc variant over each payload's whole tiles, the codec and CRC32 of
    the rest on their own, the finalize folding them together (knob frame_crc_cover) -- against the
    copy-through encode + separate CRC pass, and the restated reference framing for one stripe."""
    from liberasurecode_amd import _lib
    if legacy:
        monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", "1")
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    S = 3
    objs = _objects(S, size, k * 11 + m + size)
    out = []
    _lib.check(_lib.dev().ecamd_tune(b"bitslice", 2), "tune")
    try:
        # (frame_crc_cover, bs_realign, frame_tail_bs): the crc variant reads the object chunks
        # realigned from aligned loads + the neighbour lane's (default) or with unaligned loads; the
        # payloads' rest by split + plain encode of their last tiles (default) or the LDS-table launch
        # (+ frame_tail_fork 2: the rest and its CRC32 on the side stream beside the crc variant;
        # + frame_tail_tiles 0: the rest's whole 4 KiB tiles by the split + re-encode too)
        # + wave 0: the 16 KiB-tile crc variant instead of its one-wave form (knob frame_crc_wave)
        for cover, realign, tail, fork, tt, wave in ((1, 1, 1, 1, 1, 1), (0, 1, 1, 1, 1, 1), (1, 0, 1, 1, 1, 1),
                                                     (1, 1, 0, 1, 1, 1), (1, 1, 1, 2, 1, 1), (1, 1, 1, 1, 0, 1),
                                                     (1, 1, 1, 1, 1, 0), (1, 0, 0, 2, 1, 0)):
            _lib.check(_lib.dev().ecamd_tune(b"frame_crc_cover", cover), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_crc_wave", -1 if wave else 0), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"bs_realign", realign), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_tail_bs", tail), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_tail_fork", fork), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_tail_tiles", tt), "tune")
            n0 = _bs_launches()
            fb = F.FrameBatch(be, k, m, size, S)
            fb.encode(_upload_objects(objs, fb.obj_stride))
            out.append(fb.fragments())
            bs = fb.blocksize
            last = size - (k - 1) * bs
            # (the one-wave crc form, knob frame_crc_wave, covers whole 4 KiB tiles)
            if cover and last >= (4096 if wave else 16384):
                assert _bs_launches() > n0, "the bitsliced crc variant did not run"
            elif cover:
                assert _bs_launches() == n0, "a bitsliced kernel ran on a shape it does not take"
    finally:
        _lib.dev().ecamd_tune(b"frame_crc_cover", 1)
        _lib.dev().ecamd_tune(b"bitslice", 1)
        _lib.dev().ecamd_tune(b"bs_realign", -1)
        _lib.dev().ecamd_tune(b"frame_tail_bs", 1)
        _lib.dev().ecamd_tune(b"frame_tail_fork", -1)
        _lib.dev().ecamd_tune(b"frame_tail_tiles", -1)
        _lib.dev().ecamd_tune(b"frame_crc_wave", -1)
    assert all(np.array_equal(o, out[1]) for o in out)
    want = expected_stripe(be, k, m, 0, objs[S - 1], ec_api.CHKSUM_CRC32, legacy=legacy)
    assert all(out[0][S - 1, i].tobytes() == want[i] for i in range(k + m))


@pytest.mark.parametrize("k,m,size", [(10, 4, 10 * 104858 - 4), (4, 2, 4 * 65536 + 6), (10, 4, (10 << 20) + 10)])
def test_frame_encode_realigned_loads_match(F, k, m, size):
    """Copy-through encode of objects whose chunks start at offsets that are not multiples of 16:
    the aligned-loads-realigned-in-registers kernel (knob stream_realign 1, gf16_realign_kernel; 2:
    the window's second chunk from the next lane) writes the same fragments as the unaligned-load
    kernel, with and without CRC32."""
    from liberasurecode_amd import _lib
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    S = 3
    objs = _objects(S, size, k * 17 + size)
    for ct in (ec_api.CHKSUM_CRC32, ec_api.CHKSUM_NONE):
        out = []
        try:
            for ra in (2, 1, 0):  # 2: one aligned load per lane, the next chunk from the next lane (DPP)
                _lib.check(_lib.dev().ecamd_tune(b"stream_realign", ra), "tune")
                fb = F.FrameBatch(be, k, m, size, S, checksum=ct)
                fb.encode(_upload_objects(objs, fb.obj_stride))
                out.append(fb.fragments())
        finally:
            _lib.dev().ecamd_tune(b"stream_realign", 0)
        assert np.array_equal(out[0], out[2]) and np.array_equal(out[1], out[2])
        want = expected_stripe(be, k, m, 0, objs[1], ct)
        assert all(out[0][1, i].tobytes() == want[i] for i in range(k + m))


@pytest.mark.parametrize("k,m,size", [(10, 4, 1 << 20), (10, 4, (1 << 20) + 7), (10, 4, 3 * 104858 + 5),
                                      (4, 2, 1), (4, 2, 100), (6, 3, 6 * 4096 - 2), (8, 4, 777777),
                                      (20, 8, 4096 * 20 + 40), (12, 6, 65536 * 12 - 24)])
@pytest.mark.parametrize("ct", [1, 2])
def test_frame_encode_padded_copy_matches_split(F, k, m, size, ct):
    """Objects that do not fill the k payloads (any size; Swift's 1 MiB segments at k=10 give
    bs = 104858): the copy-through launch reads the object's chunks at unaligned offsets and zeros
    past its end.  Fragments equal the split-then-encode path's and the restated framing."""
    from liberasurecode_amd import _lib
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    S = 3
    objs = _objects(S, size, k * 13 + m + size)
    out = []
    try:
        # (frame_copy_padded, bitslice): the copy-through launch on the bitsliced kernel (one-wave
        # tiles with realigned loads when the object chunks are unaligned, knob bs_wave_copy 2), on
        # the LDS tables, and the split-then-encode path
        # (+ frame_tail_bs: the payloads' rest past the whole tiles by split + plain encode, or not;
        # + bs_prefetch: the copy-through kernel's next-input loads ahead of its copy stores, 0 / 2 / 4;
        # + frame_tail_fork: the rest on the side stream by default (1-4 KiB, no checksum), never, always;
        # + bs_copy_ring 2 / 4: the inputs through an LDS ring, realigned on the LDS read)
        for padded, mode, tail, pf, fork, ring in ((1, 2, 1, 2, 1, 0), (1, 0, 1, 2, 1, 0), (0, 1, 1, 2, 1, 0),
                                                   (1, 2, 0, 2, 0, 0), (1, 2, 1, 0, 1, 0), (1, 2, 1, 4, 1, 0),
                                                   (1, 2, 1, 2, 0, 0), (1, 2, 1, 2, 2, 0), (1, 2, 1, 2, 1, 2),
                                                   (1, 2, 1, 2, 1, 4)):
            _lib.check(_lib.dev().ecamd_tune(b"bs_copy_ring", ring), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_copy_padded", padded), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"bitslice", mode), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_tail_bs", tail), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"bs_prefetch", pf), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_tail_fork", fork), "tune")
            fb = F.FrameBatch(be, k, m, size, S, checksum=ct)
            fb.encode(_upload_objects(objs, fb.obj_stride))
            out.append(fb.fragments())
    finally:
        _lib.dev().ecamd_tune(b"frame_copy_padded", 1)
        _lib.dev().ecamd_tune(b"bitslice", 1)
        _lib.dev().ecamd_tune(b"frame_tail_bs", 1)
        _lib.dev().ecamd_tune(b"bs_prefetch", -1)
        _lib.dev().ecamd_tune(b"frame_tail_fork", -1)
        _lib.dev().ecamd_tune(b"bs_copy_ring", 0)
    assert all(np.array_equal(o, out[2]) for o in out)
    want = expected_stripe(be, k, m, 0, objs[1], ct)
    assert all(out[0][1, i].tobytes() == want[i] for i in range(k + m))


@pytest.mark.parametrize("k,m,size,missing", [(10, 4, 1 << 20, [0, 1, 2, 3]), (10, 4, (1 << 20) + 7, [9, 3, 11]),
                                              (4, 2, 100, [3]), (4, 2, 5, [0, 1]), (6, 3, 6 * 4096 - 2, [5, 6]),
                                              (8, 4, 777777, [7, 0, 8, 9]), (12, 6, 65536 * 12 - 24, [11, 10, 1])])
def test_frame_decode_padded_join_matches_split(F, k, m, size, missing):
    """Decode straight into objects that do not fill the payloads: unaligned object chunks, nothing
    written past an object's end (guard bytes between objects stay intact)."""
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    S = 3
    objs = _objects(S, size, k * 17 + m + size)
    fb = F.FrameBatch(be, k, m, size, S)
    fb.encode(_upload_objects(objs, fb.obj_stride))
    stride = (size + 16 + 15) // 16 * 16  # 16+ guard bytes after every object
    got = []
    try:
        # (frame_copy_padded, bitslice, bs_prefetch): the one-wave bitsliced decode-join (copy-through,
        # next input's loads ahead of the copy stores: 2 default, 0, 4), the LDS tables, decode + join;
        # frame_tail_fork: the LDS-table rest beside the bitsliced launch by default (1-4 KiB), never, always;
        # bs_copy_ring 2 / 4: the bitsliced decode-join's inputs through an LDS ring
        for padded, mode, pf, fork, ring in ((1, 2, 2, 1, 0), (1, 2, 0, 1, 0), (1, 2, 4, 1, 0), (1, 0, 2, 1, 0),
                                             (1, 2, 2, 0, 0), (1, 2, 2, 2, 0), (1, 2, 2, 1, 2), (1, 2, 2, 1, 4),
                                             (0, 1, 2, 1, 0)):
            _lib.check(_lib.dev().ecamd_tune(b"bs_copy_ring", ring), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_copy_padded", padded), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"bitslice", mode), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"bs_prefetch", pf), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"frame_tail_fork", fork), "tune")
            host = np.full(S * stride, 0xA5, dtype=np.uint8)
            d = DeviceBuffer(host.size)
            d.upload(host)
            fb.decode(missing, d, obj_stride=stride)
            got.append(d.download().reshape(S, stride))
    finally:
        _lib.dev().ecamd_tune(b"frame_copy_padded", 1)
        _lib.dev().ecamd_tune(b"bitslice", 1)
        _lib.dev().ecamd_tune(b"bs_prefetch", -1)
        _lib.dev().ecamd_tune(b"frame_tail_fork", -1)
        _lib.dev().ecamd_tune(b"bs_copy_ring", 0)
    assert all(np.array_equal(g, got[-1]) for g in got)
    for s in range(S):
        assert got[0][s, :size].tobytes() == objs[s]
        assert (got[0][s, size:] == 0xA5).all()


@pytest.mark.parametrize("size", [10 << 20, (10 << 20) + 7])
def test_frame_paths_split_into_launches(F, size):
    """Copy-through encode and decode-join passes split into several launches (knob
    tiles_per_slot 1: at most one 4 KiB tile per resident workgroup per launch, so 9 stripes of
    1 MiB payloads take 3 launches per pass) give the same fragments and objects as one launch."""
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    k, m, S = 10, 4, 9
    objs = _objects(S, size, 4242 + size)
    frags, joined = [], []
    try:
        for tps in (0, 1):
            _lib.check(_lib.dev().ecamd_tune(b"tiles_per_slot", tps), "tune")
            fb = F.FrameBatch(be, k, m, size, S, checksum=ec_api.CHKSUM_CRC32)
            fb.encode(_upload_objects(objs, fb.obj_stride))
            frags.append(fb.fragments())
            stride = (size + 16 + 15) // 16 * 16
            d = DeviceBuffer(S * stride)
            d.upload(np.full(S * stride, 0xA5, dtype=np.uint8))
            fb.decode([0, 3, 10], d, obj_stride=stride)
            joined.append(d.download().reshape(S, stride))
    finally:
        _lib.dev().ecamd_tune(b"tiles_per_slot", 0)
    assert np.array_equal(frags[0], frags[1])
    assert np.array_equal(joined[0], joined[1])
    for s in range(S):
        assert joined[1][s, :size].tobytes() == objs[s]
        assert (joined[1][s, size:] == 0xA5).all()


COPY_SIZES = [1, 15, 16, 17, 100, 4 * 16 + 3, 339, 407, 777777, 10 * 104858, 10 * 104858 - 3, 1048581,
              (1 << 20) * 10 + 6, (1 << 20) * 10]


@pytest.mark.parametrize("name,k,m,hd", [("rs", 10, 4, 0), ("rs", 4, 2, 0), ("xor", 10, 6, 4),
                                         ("xor", 3, 3, 3), ("rs", 20, 8, 0)])
@pytest.mark.parametrize("missing", [[], "parity"])
def test_frame_systematic_decode_stream_join(F, name, k, m, hd, missing):
    """Decode with every data fragment present (src/erasurecode.c:597-607: fragments_to_string
    only) runs the streaming join: payload chunks read at unaligned offsets j*bs when bs % 16 != 0,
    each chunk straddling two payloads one lane's merged store, the object's last partial chunk
    byte by byte.  Objects equal the originals, guard bytes after each object stay intact, and the
    one-workgroup-per-tile grid and the first-version join (knob frame_copy_stream 0) agree."""
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    be = _backend(name)
    lost = list(range(k, k + min(m, 2))) if missing == "parity" else []
    S = 3
    for size in COPY_SIZES:
        if k == 20 and size > (1 << 20):
            continue
        objs = _objects(S, size, k * 7 + size)
        fb = F.FrameBatch(be, k, m, size, S, hd=hd or 3)
        fb.encode(_upload_objects(objs, fb.obj_stride))
        stride = (size + 16 + 15) // 16 * 16 + 32
        got = []
        try:
            # (stream kernel, one workgroup per tile, lanes per tile, chunks per lane, DPP neighbour
            # chunks on the realigning path)
            # every shape, then tiles starting on aligned object chunks (frame_join_align)
            for knob, grid, lanes, u, dpp, obj in ((1, 0, 256, 4, 0, 0), (1, 1, 256, 4, 0, 0), (0, 0, 256, 4, 0, 0),
                                                   (1, 1, 64, 1, 0, 0), (1, 1, 64, 4, 0, 0), (1, 1, 128, 1, 0, 0),
                                                   (1, 0, 64, 1, 0, 0), (1, 1, 256, 1, 1, 0), (1, 1, 64, 1, 1, 0),
                                                   (1, 1, 256, 4, 1, 0), (1, 0, 128, 1, 1, 0), (1, 1, 256, 1, 1, 1),
                                                   (1, 1, 128, 1, 0, 1), (1, 1, 64, 4, 1, 1)):
                _lib.check(_lib.dev().ecamd_tune(b"frame_join_align", obj), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_stream", knob), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_grid", grid), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_threads", lanes), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_u", u), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_dpp", dpp), "tune")
                d = DeviceBuffer(S * stride)
                d.upload(np.full(S * stride, 0xA5, dtype=np.uint8))
                fb.decode(lost, d, obj_stride=stride)
                got.append(d.download().reshape(S, stride))
        finally:
            _lib.dev().ecamd_tune(b"frame_copy_stream", 1)
            _lib.dev().ecamd_tune(b"frame_copy_grid", 1)
            _lib.dev().ecamd_tune(b"frame_copy_threads", 0)
            _lib.dev().ecamd_tune(b"frame_copy_u", 0)
            _lib.dev().ecamd_tune(b"frame_copy_dpp", -1)
            _lib.dev().ecamd_tune(b"frame_join_align", -1)
        for i in range(1, len(got)):
            assert np.array_equal(got[0], got[i]), (size, i)
        for s in range(S):
            assert got[0][s, :size].tobytes() == objs[s], (size, s)
            assert (got[0][s, size:] == 0xA5).all(), (size, s)


@pytest.mark.parametrize("name,k,m,hd", [("xor", 10, 6, 4), ("xor", 3, 3, 3), ("rs", 10, 4, 0)])
def test_frame_split_stream_matches_first_version(F, name, k, m, hd):
    """prepare_fragments_for_encode on the streaming split kernel (XOR framed encode always; RS
    with the copy-through launch off): fragments byte-equal to the first-version split kernel and
    to the restated framing, for sizes with bs % 16 != 0 and tiny objects."""
    from liberasurecode_amd import _lib
    be = _backend(name)
    S = 3
    for size in COPY_SIZES:
        objs = _objects(S, size, k * 11 + size)
        out = []
        try:
            _lib.check(_lib.dev().ecamd_tune(b"frame_unfused", 1), "tune")
            # (stream kernel, lanes per tile, chunks per lane, DPP neighbour chunks)
            for knob, lanes, u, dpp in ((1, 256, 4, 0), (0, 256, 4, 0), (1, 64, 1, 0), (1, 128, 1, 0),
                                        (1, 64, 4, 0), (1, 256, 1, 1), (1, 64, 1, 1), (1, 256, 4, 1)):
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_stream", knob), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_threads", lanes), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_u", u), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_copy_dpp", dpp), "tune")
                fb = F.FrameBatch(be, k, m, size, S, hd=hd or 3, checksum=ec_api.CHKSUM_CRC32)
                fb.encode(_upload_objects(objs, fb.obj_stride))
                out.append(fb.fragments())
        finally:
            _lib.dev().ecamd_tune(b"frame_copy_stream", 1)
            _lib.dev().ecamd_tune(b"frame_unfused", 0)
            _lib.dev().ecamd_tune(b"frame_copy_threads", 0)
            _lib.dev().ecamd_tune(b"frame_copy_u", 0)
            _lib.dev().ecamd_tune(b"frame_copy_dpp", -1)
        for i in range(1, len(out)):
            assert np.array_equal(out[0], out[i]), (size, i)
        want = expected_stripe(be, k, m, hd, objs[2], ec_api.CHKSUM_CRC32)
        assert all(out[0][2, i].tobytes() == want[i] for i in range(k + m)), size


@pytest.mark.parametrize("k,m,tiles,extra", [(24, 6, 3, 48), (27, 5, 2, 4000), (21, 8, 1, 16), (24, 6, 3, 0)])
def test_frame_bitsliced_wide_ragged(F, k, m, tiles, extra):
    """More than 20 inputs (the stream kernel's limit per pass) with payloads that are not whole
    16 KiB tiles: the bitsliced kernel could cover the whole tiles only, and the table passes of
    such maps cannot run the remainder on the stream kernel, so the framed encode / decode-join
    must not fail after a partial write: either the LDS-table kernels take the whole fragment, or
    (round 4, ecamd_frame_api.hip encode_tail) the bitsliced kernel takes the payloads' whole tiles
    as a range of its own and the rest runs as split + plain encode.  Whole tiles (extra 0) take
    the bitsliced kernel (launch counter)."""
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    S = 2
    bs = tiles * 16384 + extra
    size = k * bs - 5 if extra else k * bs
    objs = _objects(S, size, k + m + extra)
    lost = list(range(0, 2 * m, 2))[:m]
    try:
        _lib.check(_lib.dev().ecamd_tune(b"bitslice", 2), "tune")
        n0 = _bs_launches()
        fb = F.FrameBatch(be, k, m, size, S, checksum=ec_api.CHKSUM_NONE)
        fb.encode(_upload_objects(objs, fb.obj_stride))
        got = fb.fragments()
        bad = got.copy()
        bad[:, lost] = 0x6B
        fb.upload_fragments(bad)
        stride = (size + 16 + 15) // 16 * 16
        d = DeviceBuffer(S * stride)
        d.upload(np.full(S * stride, 0xA5, dtype=np.uint8))
        fb.decode(lost, d, obj_stride=stride)
        joined = d.download().reshape(S, stride)
        ran = _bs_launches() - n0
    finally:
        _lib.dev().ecamd_tune(b"bitslice", 1)
    for s in range(S):
        want = expected_stripe(be, k, m, 0, objs[s], ec_api.CHKSUM_NONE)
        assert all(got[s, i].tobytes() == want[i] for i in range(k + m)), s
        assert joined[s, :size].tobytes() == objs[s]
        assert (joined[s, size:] == 0xA5).all()
    if extra == 0:
        assert ran > 0, ran


def _bs_launches():
    import ctypes as C
    from liberasurecode_amd import _lib
    f = _lib.dev().ecamd_bitslice_launches
    f.restype = C.c_longlong
    return f()


@pytest.mark.parametrize("k,m,size", [(20, 8, 20 * (1 << 20)), (20, 8, 20 * 65536 - 1000),
                                      (12, 6, 12 * 3 * 16384 + 7), (10, 5, 10 * (1 << 20))])
@pytest.mark.parametrize("missing", [None, "data", "mixed"])
def test_frame_bitsliced_copy_through(F, k, m, size, missing):
    """Framed encode (copy-through) and decode-join of 5..8-output maps on the bitsliced kernel
    (knob bitslice 2: waits for its compile; the launch counter proves it ran) give the same
    fragments / objects as the LDS-table kernels (knob 0) and the restated framing: the kernel
    stores each input into its payload slot (encode) or object chunk (decode) as it loads it, and
    takes only the whole 16 KiB tiles every object chunk holds (objects shorter than the payloads)."""
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    S = 2
    objs = _objects(S, size, k + m + size)
    lost = (None if missing is None else list(range(min(m, 8))) if missing == "data"
            else [0, 2, 4, 6, k, k + 2, k + 4, k + 6][:m])
    frags, joined = [], []
    try:
        # (bitslice, bs_realign): unaligned object chunks (bs % 16 != 0) read as aligned chunks + the
        # neighbour lane's, realigned (default), or with unaligned loads
        # + bs_late_copy: each input's copy stores after its network and the next input's loads
        for mode, realign, late in ((2, 1, 0), (0, 1, 0), (2, 0, 0), (2, 1, 1)):
            _lib.check(_lib.dev().ecamd_tune(b"bitslice", mode), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"bs_realign", realign), "tune")
            _lib.check(_lib.dev().ecamd_tune(b"bs_late_copy", late), "tune")
            n0 = _bs_launches()
            # no checksum: with CRC32 a one-pass map that fits takes the fused CRC kernel instead
            fb = F.FrameBatch(be, k, m, size, S, checksum=ec_api.CHKSUM_NONE)
            fb.encode(_upload_objects(objs, fb.obj_stride))
            got = fb.fragments()
            frags.append(got)
            if lost is not None:
                bad = got.copy()
                bad[:, lost] = 0x6B
                fb.upload_fragments(bad)
                stride = (size + 16 + 15) // 16 * 16
                d = DeviceBuffer(S * stride)
                d.upload(np.full(S * stride, 0xA5, dtype=np.uint8))
                fb.decode(lost, d, obj_stride=stride)
                joined.append(d.download().reshape(S, stride))
            ran = _bs_launches() - n0
            assert (ran > 0) == (mode == 2), (mode, ran)
    finally:
        _lib.dev().ecamd_tune(b"bitslice", 1)
        _lib.dev().ecamd_tune(b"bs_realign", -1)
        _lib.dev().ecamd_tune(b"bs_late_copy", -1)
    assert all(np.array_equal(f, frags[1]) for f in frags)
    want = expected_stripe(be, k, m, 0, objs[1], ec_api.CHKSUM_NONE)
    assert all(frags[0][1, i].tobytes() == want[i] for i in range(k + m))
    if lost is not None:
        assert all(np.array_equal(j, joined[1]) for j in joined)
        for s in range(S):
            assert joined[0][s, :size].tobytes() == objs[s]
            assert (joined[0][s, size:] == 0xA5).all()


@pytest.mark.parametrize("k,m,hd", [(10, 6, 4), (3, 3, 3), (12, 6, 4), (10, 5, 3), (20, 6, 4)])
@pytest.mark.parametrize("ct", [ec_api.CHKSUM_CRC32, ec_api.CHKSUM_NONE])
def test_frame_xor_copy_through_matches_split(F, k, m, hd, ct):
    """Framed flat-XOR encode on the copy-through XOR launch (round 4, knob frame_xor_copy): the whole
    4 KiB tiles every object chunk holds in one pass (object chunks -> data payloads + parity), the
    rest by the streaming split + the XOR of that range; with CRC32 the bitsliced crc variant over the
    whole 16 KiB tiles (the code as a 0 / 1 matrix) -- fragments equal the split-then-XOR path's and
    the restated framing, over sizes with bs % 16 != 0 (Swift's segments), whole tiles, chunks shorter
    than a tile and tiny objects."""
    from liberasurecode_amd import _lib
    be = ec_api.EC_BACKEND_FLAT_XOR_HD
    S = 3
    for size in (1 << 20, 10 * 104858 - 3, 777777, k * 4096, k * 4096 + 2, 4096 * 3 + 5, 100, 1,
                 k * 3 * 16384, 2 * k * 16384 + 6):
        objs = _objects(S, size, k * 31 + m + size)
        out = []
        try:
            # (frame_xor_copy, bitslice): with CRC32 and bitslice 2 the checksums fold into the bitsliced
            # crc variant run as a 0 / 1 matrix (launch counter); bitslice 0 the copy-through XOR + CRC
            # pass; frame_xor_copy 0 the split + XOR path; frame_tail_fork 0 / 2: the payloads' rest after
            # the whole tiles on the caller's stream / always on the side stream (default: no checksum, 1-4 KiB)
            for on, mode, fork in ((1, 2, 1), (1, 0, 1), (0, 1, 1), (1, 2, 0), (1, 2, 2)):
                _lib.check(_lib.dev().ecamd_tune(b"frame_xor_copy", on), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"bitslice", mode), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"frame_tail_fork", fork), "tune")
                n0 = _bs_launches()
                fb = F.FrameBatch(be, k, m, size, S, hd=hd, checksum=ct)
                fb.encode(_upload_objects(objs, fb.obj_stride))
                out.append(fb.fragments())
                last = size - (k - 1) * fb.blocksize
                if mode == 2 and ct == ec_api.CHKSUM_CRC32 and last >= 16384 and m <= 8 and fb.blocksize % 2 == 0:
                    assert _bs_launches() > n0, ("crc variant did not run", size)
        finally:
            _lib.dev().ecamd_tune(b"frame_xor_copy", 1)
            _lib.dev().ecamd_tune(b"bitslice", 1)
            _lib.dev().ecamd_tune(b"frame_tail_fork", -1)
        assert all(np.array_equal(o, out[2]) for o in out), size
        want = expected_stripe(be, k, m, hd, objs[S - 1], ct)
        assert all(out[0][S - 1, i].tobytes() == want[i] for i in range(k + m)), size


@pytest.mark.parametrize("k,m,hd,missing", [(10, 6, 4, [0, 1, 2]), (10, 6, 4, [3, 11, 14]), (3, 3, 3, [1, 4]),
                                            (10, 5, 3, [9, 12]), (20, 6, 4, [19, 0, 7]), (12, 6, 4, [5])])
def test_frame_xor_decode_join_matches(F, k, m, hd, missing):
    """Framed flat-XOR decode with data lost (round 4, knob frame_xor_copy): the plan's 0 / 1 matrix over
    the surviving fragments as one decode-join launch (lost data straight into the objects, surviving
    data copied there) against decode in place + join; objects equal the originals, guard bytes after
    every object intact, over sizes with unaligned chunks (Swift's segments), whole tiles and tiny
    objects, on the bitsliced and the LDS-table kernels."""
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import DeviceBuffer
    be = ec_api.EC_BACKEND_FLAT_XOR_HD
    S = 3
    for size in (1 << 20, 10 * 104858 - 3, 777777, k * 3 * 16384, 100, 1):
        objs = _objects(S, size, k * 29 + m + size)
        fb = F.FrameBatch(be, k, m, size, S, hd=hd)
        fb.encode(_upload_objects(objs, fb.obj_stride))
        bad = fb.fragments()
        bad[:, missing] = 0x6B
        fb.upload_fragments(bad)
        stride = (size + 16 + 15) // 16 * 16
        got = []
        try:
            for on, mode in ((1, 2), (1, 0), (0, 1)):
                _lib.check(_lib.dev().ecamd_tune(b"frame_xor_copy", on), "tune")
                _lib.check(_lib.dev().ecamd_tune(b"bitslice", mode), "tune")
                d = DeviceBuffer(S * stride)
                d.upload(np.full(S * stride, 0xA5, dtype=np.uint8))
                fb.decode(missing, d, obj_stride=stride)
                got.append(d.download().reshape(S, stride))
                fb.upload_fragments(bad)  # the in-place decode rewrites the lost slots
        finally:
            _lib.dev().ecamd_tune(b"frame_xor_copy", 1)
            _lib.dev().ecamd_tune(b"bitslice", 1)
        for g in got:
            for s in range(S):
                assert g[s, :size].tobytes() == objs[s], (size, s)
                assert (g[s, size:] == 0xA5).all(), (size, s)


def test_stream_contexts_bounded(F):
    """A caller that creates and destroys a stream per request (a proxy) must not grow the library's
    per-stream contexts (side stream + events + CRC scratch, ecamd_device.hip StreamCtx): 1000 streams,
    each used once by a Swift-shaped framed encode (1 MiB segment, k=10: bs = 104858, the payloads'
    rest forked to the side stream without checksum; CRC32 scratch with it), half destroyed through
    ecamd_stream_destroy, half behind the library's back by hipStreamDestroy.  The context count stays
    at the cap and every sampled stripe is byte-exact against the restated framing."""
    import ctypes
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import Stream
    d = _lib.dev()
    # hipStreamDestroy behind the library's back, on the library's own HIP runtime (a ctypes load of
    # "libamdhip64.so" may open another copy than the one libecamd and torch share, by test order)
    d.ecamd_stream_destroy_unmanaged.argtypes = [ctypes.c_void_p]
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    k, m, size = 10, 4, 1 << 20
    objs = _objects(1, size, 4242)
    fbs = {ct: F.FrameBatch(be, k, m, size, 1, checksum=ct) for ct in (ec_api.CHKSUM_NONE, ec_api.CHKSUM_CRC32)}
    want = {ct: expected_stripe(be, k, m, 0, objs[0], ct) for ct in fbs}
    d_obj = _upload_objects(objs, fbs[ec_api.CHKSUM_NONE].obj_stride)
    peak = 0
    for i in range(1000):
        ct = ec_api.CHKSUM_CRC32 if i % 3 == 2 else ec_api.CHKSUM_NONE
        s = Stream()
        fbs[ct].encode(d_obj, stream=s)
        if i % 50 in (0, 2):
            s.synchronize()
            got = fbs[ct].fragments()
            assert all(got[0, f].tobytes() == want[ct][f] for f in range(k + m)), (i, ct)
        if i % 2:
            s.destroy()
        else:
            s.synchronize()
            assert d.ecamd_stream_destroy_unmanaged(ctypes.c_void_p(s.handle)) == 0
            s.handle = None
        peak = max(peak, d.ecamd_stream_contexts())
    assert peak <= 17, peak  # the cap (16) + the context being created


def test_stream_contexts_threaded(F):
    """Stream contexts under concurrency: 8 threads, each creating a stream per request, running a Swift-shaped
    framed encode (side-stream fork, CRC32 scratch on every third request) into its own fragments, checking the
    bytes and destroying the stream -- contexts are created, evicted and released while other threads' calls are
    in flight (busy contexts are never released).  The count stays bounded."""
    import threading
    from liberasurecode_amd import _lib
    from liberasurecode_amd.device import Stream
    d = _lib.dev()
    be = ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND
    k, m, size = 10, 4, 1 << 20
    objs = _objects(1, size, 777)
    want = {ct: expected_stripe(be, k, m, 0, objs[0], ct) for ct in (ec_api.CHKSUM_NONE, ec_api.CHKSUM_CRC32)}
    errors, peak = [], [0]
    lock = threading.Lock()

    def worker(tid):
        try:
            fbs = {ct: F.FrameBatch(be, k, m, size, 1, checksum=ct) for ct in want}
            d_obj = _upload_objects(objs, fbs[ec_api.CHKSUM_NONE].obj_stride)
            for i in range(40):
                ct = ec_api.CHKSUM_CRC32 if (i + tid) % 3 == 0 else ec_api.CHKSUM_NONE
                s = Stream()
                fbs[ct].encode(d_obj, stream=s)
                s.synchronize()
                got = fbs[ct].fragments()
                if not all(got[0, f].tobytes() == want[ct][f] for f in range(k + m)):
                    errors.append((tid, i, ct))
                s.destroy()
                with lock:
                    peak[0] = max(peak[0], d.ecamd_stream_contexts())
        except Exception as e:  # noqa: BLE001
            errors.append((tid, repr(e)))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]
    assert peak[0] <= 16 + 8, peak[0]


@pytest.mark.gpu
@pytest.mark.parametrize("be,k,m,size", [
    ("rs", 10, 4, 10 << 20), ("rs", 10, 4, 10 * 104858 - 4), ("rs", 4, 2, 4 * 65536 + 6), ("rs", 3, 2, 3 * 4096 * 5),
    ("rs", 6, 3, 6 * 16384 + 6 * 100), ("rs", 10, 4, 10 * (4096 + 16)), ("xor", 3, 3, 3 * 65536),
    ("xor", 3, 3, 3 * 104858 - 4), ("rs", 20, 8, 20 * 40000), ("rs", 12, 6, 12 * 65536),
    ("rs", 10, 4, 10 * 23 * 4096), ("rs", 4, 2, 4 * 4096)])
@pytest.mark.parametrize("form", [(6, 2, 4, 0, 4), (4, 1, 1, 2, 3), (12, 4, 3, 0, 4), (6, 2, 1, 4, 2), (4, 2, 1, 4, 1),
                                  (4, 2, 1, 3, 4), (4, 2, 1, 2, 4, 1)])
@pytest.mark.parametrize("legacy", [False, True])
def test_frame_encode_crc_wave_matches(F, be, k, m, size, form, legacy, monkeypatch):
    """CHKSUM_CRC32 framed encode on the crc variant in one-wave 4 KiB tiles (knobs frame_crc_wave =
    waves per workgroup, frame_crc_wave_pos = position sets, frame_crc_wave_per = tiles per wave,
    frame_crc_wave_pf = chunks of the next input prefetched, 60% of the tiles in those runs when
    longer than one, frame_crc_wave_mb = piece dwords on byte tables (the rest on nibble tables);
    bitslice.cpp CW form, crc_combine_kernel) against the 16 KiB-tile crc variant / the codec + CRC
    pass, and the restated reference framing for the last stripe.  frame_crc_wave_strict makes a
    declined form an error, so the new kernel is the one that ran."""
    from liberasurecode_amd import _lib
    if legacy:
        monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", "1")
    code = (ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND if be == "rs" else ec_api.EC_BACKEND_FLAT_XOR_HD)
    hd = 3 if m == 3 else 4
    S = 3
    objs = _objects(S, size, k * 13 + m + size)
    d = _lib.dev()
    out = []
    _lib.check(d.ecamd_tune(b"bitslice", 2), "tune")
    try:
        for w in (0, form[0]):
            _lib.check(d.ecamd_tune(b"frame_crc_wave", w), "tune")
            _lib.check(d.ecamd_tune(b"frame_crc_wave_pos", form[1]), "tune")
            _lib.check(d.ecamd_tune(b"frame_crc_wave_per", form[2]), "tune")
            _lib.check(d.ecamd_tune(b"frame_crc_wave_pf", form[3]), "tune")
            _lib.check(d.ecamd_tune(b"frame_crc_wave_big", 60 if form[2] > 1 else 0), "tune")
            _lib.check(d.ecamd_tune(b"frame_crc_wave_mb", form[4]), "tune")
            # form[5]: a piece's last dword looked up in global memory (knob frame_crc_wave_l1, round 6 A/B)
            _lib.check(d.ecamd_tune(b"frame_crc_wave_l1", form[5] if len(form) > 5 else 0), "tune")
            _lib.check(d.ecamd_tune(b"frame_crc_wave_strict", 1 if w else 0), "tune")
            fb = F.FrameBatch(code, k, m, size, S, hd=hd)
            fb.encode(_upload_objects(objs, fb.obj_stride))
            out.append(fb.fragments())
    finally:
        for kn in (b"frame_crc_wave", b"frame_crc_wave_pos", b"frame_crc_wave_per", b"frame_crc_wave_pf",
                   b"frame_crc_wave_big", b"frame_crc_wave_mb", b"frame_crc_wave_strict", b"frame_crc_wave_l1"):
            d.ecamd_tune(kn, -1)
        d.ecamd_tune(b"bitslice", 1)
    assert np.array_equal(out[0], out[1])
    want = expected_stripe(code, k, m, hd if be == "xor" else 0, objs[S - 1], ec_api.CHKSUM_CRC32, legacy=legacy)
    assert all(out[1][S - 1, i].tobytes() == want[i] for i in range(k + m))
