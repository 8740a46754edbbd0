#!/usr/bin/env python3
"""Per-call latency of the drop-in API (liberasurecode_encode / _decode through
liberasurecode.so.1 -> liberasurecode_rs_vand.so.1 -> GPU), one thread, RS(10,4), object sizes
4 KiB .. 16 MiB; median of N calls.  Prints one JSON line per size."""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ec_api  # noqa: E402


def main():
    desc = ec_api.create(ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, ct=ec_api.CHKSUM_CRC32)
    assert desc > 0, desc
    for size in [4096, 65536, 1 << 20, 4 << 20, 16 << 20]:
        data = os.urandom(size)
        enc, dec = [], []
        for it in range(30):
            t0 = time.perf_counter()
            rc, d, p, flen = ec_api.encode(desc, data)
            t1 = time.perf_counter()
            assert rc == 0
            frags = ec_api.fragments(d, 10, flen) + ec_api.fragments(p, 4, flen)
            ec_api.lib().liberasurecode_encode_cleanup(desc, d, p)
            avail = frags[4:]
            t1b = time.perf_counter()
            rc, out = ec_api.decode(desc, avail, flen)
            t2 = time.perf_counter()
            assert rc == 0 and out == data
            if it >= 5:
                enc.append(t1 - t0)
                dec.append(t2 - t1b)  # includes the ctypes copy-out of the decoded object
        me, md = statistics.median(enc), statistics.median(dec)
        print(json.dumps({"size": size, "encode_us": round(me * 1e6, 1),
                          "decode_4lost_us": round(md * 1e6, 1),
                          "encode_GiBps": round(size / me / 2**30, 2),
                          "decode_GiBps": round(size / md / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
