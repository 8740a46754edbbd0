#!/usr/bin/env python3
"""Per-call small server probe (round 6): RS(10,4) CHKSUM_NONE objects of one size, a caller repeating
one operation (N encodes, then N decodes) or alternating encode and decode; median latency per call and
the server's counters over each phase (posts, slot rewrites, kernel launches).  One JSON line per phase.
usage: server_probe.py [size] [N]"""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (one HIP runtime per process: torch's)

import ec_api as E  # noqa: E402
from liberasurecode_amd import _lib  # noqa: E402


def counters():
    d = _lib.dev()
    out = {}
    for key in ("posts", "rewrites", "launches"):
        fn = getattr(d, "ecamd_small_server_" + key)
        fn.restype = C.c_longlong
        out[key] = fn()
    return out


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    k, m = 10, 4
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, hd=m, ct=E.CHKSUM_NONE)
    data = os.urandom(size)

    def enc():
        t0 = time.perf_counter()
        rc, dp, pp, flen = E.encode(desc, data)
        t1 = time.perf_counter()
        assert rc == 0
        frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
        E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
        return t1 - t0, frags, flen

    def dec(frags, flen):
        t0 = time.perf_counter()
        rc, got = E.decode(desc, frags[m:], flen)
        t1 = time.perf_counter()
        assert rc == 0 and got == data
        return t1 - t0

    _, frags, flen = enc()
    dec(frags, flen)
    for phase in ("repeat_encode", "repeat_decode", "alternate", "repeat_encode", "alternate"):
        c0 = counters()
        te, td = [], []
        for _ in range(n):
            if phase in ("repeat_encode", "alternate"):
                te.append(enc()[0])
            if phase in ("repeat_decode", "alternate"):
                td.append(dec(frags, flen))
        c1 = counters()
        rec = {"phase": phase, "size": size, "calls": n,
               "server": os.environ.get("ECAMD_PERCALL_SERVER", "1")}
        if te:
            rec["encode_us"] = round(statistics.median(te) * 1e6, 1)
        if td:
            rec["decode_us"] = round(statistics.median(td) * 1e6, 1)
        rec.update({key: c1[key] - c0[key] for key in c0})
        print(json.dumps(rec), flush=True)
    E.lib().liberasurecode_instance_destroy(desc)


if __name__ == "__main__":
    main()
