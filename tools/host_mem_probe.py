#!/usr/bin/env python3
"""Host-side cost of pinned memory (development tool): CPU memcpy bandwidth into / out of
hipHostMalloc'd buffers vs ordinary pageable buffers, and the per-call cost of hipMemcpyAsync
for small pinned transfers."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def bw(dst, src, reps=20):
    np.copyto(dst, src)
    t0 = time.perf_counter()
    for _ in range(reps):
        np.copyto(dst, src)
    return dst.nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    d = _lib.dev()
    n = 16 << 20
    p = C.c_void_p()
    _lib.check(d.ecamd_host_alloc(C.byref(p), n), "host alloc")
    pinned = np.ctypeslib.as_array((C.c_uint8 * n).from_address(p.value))
    pool = d.ecamd_pool_alloc
    pool.restype = C.c_void_p
    pool.argtypes = [C.c_int64]
    q = pool(n)
    pooled = np.ctypeslib.as_array((C.c_uint8 * n).from_address(q))
    a = np.frombuffer(os.urandom(n), dtype=np.uint8).copy()
    b = np.empty(n, np.uint8)
    out = {"pageable_to_pageable": bw(b, a), "pageable_to_pinned": bw(pinned, a),
           "pinned_to_pageable": bw(b, pinned), "pageable_to_pool": bw(pooled, a),
           "pool_to_pageable": bw(b, pooled)}
    # per-call cost of small async copies from pinned memory
    st = D.Stream()
    dev = D.DeviceBuffer(n)
    for size in (4096, 65536, 600 << 10):
        reps = 200
        t0 = time.perf_counter()
        for _ in range(reps):
            d.ecamd_memcpy_async(C.c_void_p(dev.ptr), p, C.c_int64(size), 0, st.handle)
        st.synchronize()
        out[f"h2d_async_{size}_us"] = (time.perf_counter() - t0) / reps * 1e6
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
