#!/usr/bin/env python3
"""One thread, RS(10,4), CHKSUM_NONE: `n` liberasurecode_encode calls of one `size`-byte object through
this repo's frontend and codec (development probe, round 5), for a rocprofv3 HIP-API / kernel /
copy trace of what a small call does.  usage: percall_trace.py [size] [n] [checksum type: 0 none, 2 CRC32]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ec_api  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ct = int(sys.argv[3]) if len(sys.argv) > 3 else ec_api.CHKSUM_NONE
    desc = ec_api.create(ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, ct=ct)
    assert desc > 0, desc
    data = os.urandom(size)
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        rc, d, p, flen = ec_api.encode(desc, data)
        ts.append(time.perf_counter() - t0)
        assert rc == 0
        ec_api.lib().liberasurecode_encode_cleanup(desc, d, p)
    ts = sorted(ts[10:])
    print({"size": size, "ct": ct, "median_us": round(ts[len(ts) // 2] * 1e6, 1)})
    ec_api.lib().liberasurecode_instance_destroy(desc)


if __name__ == "__main__":
    main()
