"""Child process of tests/test_gpu_percall_env.py: the per-call API (liberasurecode_encode / _decode /
_reconstruct_fragment through this repo's liberasurecode.so.1) under whatever ECAMD_PERCALL_* settings
the parent put in the environment (they are read once per process).  RS(10,4) and flat_xor_hd (10,6,4)
objects of 4 KiB,
64 KiB and 1 MiB (+5 bytes), CHKSUM_NONE and CHKSUM_CRC32: every fragment compared with the restated
framing over the oracle codec (test_gpu_frontend.rs_expected), a decode of 4 lost data fragments and a
reconstruct of a lost parity.  Prints one JSON line {"ok": true, "digest": sha256 of all outputs, "posts" /
"server_launches": the resident small server's counters}.

PERCALL_SLEEP_US: a pause after every call (the server's idle exit between calls).  PERCALL_THREADS=N:
the RS(10,4) calls of 4 KiB and 16 KiB fragments, 30 rounds, in N threads at once (each thread its own
server, up to the library's limit; the rest launch) -- every result checked, no digest."""
import ctypes as C
import hashlib
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import torch  # noqa: E402,F401  (one HIP runtime per process: torch's)

import ec_api as E  # noqa: E402
from test_gpu_frontend import payload_bytes, rs_expected, xor_expected  # noqa: E402


def _counters():
    from liberasurecode_amd import _lib
    d = _lib.dev()
    out = {}
    for key, name in (("posts", "ecamd_small_server_posts"), ("server_launches", "ecamd_small_server_launches"),
                      ("rewrites", "ecamd_small_server_rewrites")):
        fn = getattr(d, name)
        fn.restype = C.c_longlong
        out[key] = fn()
    return out


def _pause():
    us = int(os.environ.get("PERCALL_SLEEP_US", "0"))
    if us:
        time.sleep(us / 1e6)


def threads_main(n):
    k, m = 10, 4
    errors = []
    cases = []
    for ct in (E.CHKSUM_NONE, E.CHKSUM_CRC32):
        for size in (4096 * k, 16384 * k - 7):
            data = payload_bytes(size, size + ct)
            cases.append((ct, data, rs_expected(k, m, data, ct)))
    descs = {ct: E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, hd=m, ct=ct) for ct in (E.CHKSUM_NONE, E.CHKSUM_CRC32)}

    def work(t):
        try:
            for rnd in range(30):
                for ct, data, want in cases[t % len(cases):] + cases[:t % len(cases)]:
                    desc = descs[ct]
                    rc, dp, pp, flen = E.encode(desc, data)
                    assert rc == 0, ("encode", rc)
                    frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
                    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
                    assert frags == want, ("fragments", t, rnd, ct, len(data))
                    rc, out = E.decode(desc, frags[4:], flen, force=1)
                    assert rc == 0 and out == data, ("decode", t, rnd, ct, len(data), rc)
                    _pause()
        except AssertionError as e:  # noqa: PERF203
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(n)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:3]
    for desc in descs.values():
        assert E.lib().liberasurecode_instance_destroy(desc) == 0
    print(json.dumps(dict({"ok": True, "threads": n}, **_counters())))


def churn_main():
    """PERCALL_CHURN=1: the server's cached argument slots and table placements under churn (one thread, one
    kernel key: W = 4 outputs, 4-byte lanes).  (1) Two large RS(10,4) encodes (6 workgroups), then N one-
    workgroup encodes of distinct sizes (every one rewrites a slot; N around 512 brings both slots' 8-bit
    generations back round to the large calls'), then a third large encode -- the workgroups that sat out
    the small calls must not reuse the large calls' arguments.  (2) RS(10,4) encode and decode alternating
    (each slot's tables in its half of the LDS), and RS(10,4) encode alternating with an RS(20,8) decode of 4
    lost data fragments (20 inputs: tables over half the LDS, placed at 0).  Every output checked."""
    k, m = 10, 4
    ct = E.CHKSUM_NONE
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, hd=m, ct=ct)
    desc20 = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 20, 8, hd=8, ct=ct)
    assert desc > 0 and desc20 > 0
    cache = {}

    def enc(d, kk, mm, size):
        if (kk, size) not in cache:
            data = payload_bytes(size, size * 7 + kk)
            cache[(kk, size)] = (data, rs_expected(kk, mm, data, ct))
        data, want = cache[(kk, size)]
        rc, dp, pp, flen = E.encode(d, data)
        assert rc == 0, ("encode", kk, size, rc)
        frags = E.fragments(dp, kk, flen) + E.fragments(pp, mm, flen)
        E.lib().liberasurecode_encode_cleanup(d, dp, pp)
        assert frags == want, ("fragments", kk, size)
        return data, frags, flen

    def dec(d, data, frags, flen, lost):
        rc, out = E.decode(d, frags[lost:], flen, force=1)
        assert rc == 0 and out == data, ("decode", len(data), rc)

    before = _counters()["posts"]
    small = [k * bs for bs in range(514, 1025, 2)]  # fragments of 514..1024 bytes: one workgroup of 4-byte lanes
    large = [k * (6000 + 2 * j) for j in range(16)]  # ~6 KiB fragments: 6 workgroups
    calls = 0
    for rep, n in enumerate((510, 511, 512, 513, 514)):
        enc(desc, k, m, large[3 * rep])
        enc(desc, k, m, large[3 * rep + 1])
        for i in range(n):
            enc(desc, k, m, small[i % len(small)])
        enc(desc, k, m, large[3 * rep + 2])
        calls += n + 3
    alt_rewrites = []
    for size in (k * 700, k * 3000):
        data, frags, flen = enc(desc, k, m, size)
        dec(desc, data, frags, flen, 4)
        r0 = _counters()["rewrites"]
        for _ in range(50):  # both argument blocks stay cached in the two slots
            enc(desc, k, m, size)
            dec(desc, data, frags, flen, 4)
            calls += 2
        alt_rewrites.append(_counters()["rewrites"] - r0)
        data20, frags20, flen20 = enc(desc20, 20, 8, 2 * size)
        for _ in range(50):
            enc(desc, k, m, size)
            dec(desc, data, frags, flen, 4)
            enc(desc, k, m, size)
            dec(desc20, data20, frags20, flen20, 4)
            calls += 4
    for d in (desc, desc20):
        assert E.lib().liberasurecode_instance_destroy(d) == 0
    out = _counters()
    print(json.dumps(dict({"ok": True, "calls": calls, "posted": out["posts"] - before,
                           "alternating_rewrites": alt_rewrites}, **out)))


def main():
    if os.environ.get("PERCALL_THREADS"):
        return threads_main(int(os.environ["PERCALL_THREADS"]))
    if os.environ.get("PERCALL_CHURN"):
        return churn_main()
    h = hashlib.sha256()
    # liberasurecode_rs_vand (10, 4) and flat_xor_hd (10, 6, 4): 4 / 3 data fragments lost
    for be, k, m, hd, lost in ((E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, 4, 4), (E.EC_BACKEND_FLAT_XOR_HD, 10, 6, 4, 3)):
        for ct in (E.CHKSUM_NONE, E.CHKSUM_CRC32):
            desc = E.create(be, k, m, hd=hd, ct=ct)
            assert desc > 0, desc
            for size in (4096, 65536 + 5, (1 << 20) + 5):
                data = payload_bytes(size, size * 3 + ct)
                rc, dp, pp, flen = E.encode(desc, data)
                assert rc == 0, ("encode", size, rc)
                _pause()
                frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
                E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
                want = rs_expected(k, m, data, ct) if be == E.EC_BACKEND_LIBERASURECODE_RS_VAND \
                    else xor_expected(k, m, hd, data, ct)
                assert frags == want, ("fragments", be, ct, size,
                                       [(i, [o for o in range(len(f)) if f[o] != w[o]][:8])
                                        for i, (f, w) in enumerate(zip(frags, want)) if f != w])
                rc, out = E.decode(desc, frags[lost:], flen, force=1)
                assert rc == 0 and out == data, ("decode", be, ct, size, rc)
                _pause()
                rc, rec = E.reconstruct(desc, frags[:k] + frags[k + 1:], flen, k)
                assert rc == 0 and rec == frags[k], ("reconstruct", be, ct, size, rc)
                for f in frags:
                    h.update(f)
            assert E.lib().liberasurecode_instance_destroy(desc) == 0
    print(json.dumps(dict({"ok": True, "digest": h.hexdigest()}, **_counters())))


if __name__ == "__main__":
    main()
