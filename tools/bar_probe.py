#!/usr/bin/env python3
"""Probe (development tool, round 5): can the host write device memory directly (large BAR), and how
fast is a small H2D through it compared with hipMemcpyAsync?  Allocates fine-grained device memory
(hipExtMallocWithFlags), writes 4 KiB into it from the host with memmove, reads it back with a D2H
copy, and times 1000 x (host write 4 KiB + hipStreamSynchronize) vs 1000 x (hipMemcpyAsync 4 KiB +
sync).  One JSON line."""
import ctypes as C
import json
import time

import torch  # noqa: F401

hip = C.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
out = {}
n = 4096
for name, flags in (("finegrained", 1), ("uncached", 3)):
    p = C.c_void_p()
    rc = hip.hipExtMallocWithFlags(C.byref(p), 1 << 20, flags)
    out[name + "_rc"] = rc
    if rc != 0:
        continue
    src = bytes(range(256)) * (n // 256)
    try:
        C.memmove(p.value, src, n)
        back = C.create_string_buffer(n)
        hip.hipMemcpy(back, p, n, 2)  # hipMemcpyDeviceToHost
        out[name + "_host_write_ok"] = back.raw == src
        t0 = time.perf_counter()
        for _ in range(1000):
            C.memmove(p.value, src, n)
        out[name + "_host_write_us"] = round((time.perf_counter() - t0) * 1e3, 3)
    except Exception as e:  # noqa: BLE001
        out[name + "_error"] = repr(e)
d = C.c_void_p()
hip.hipMalloc(C.byref(d), 1 << 20)
h = C.c_void_p()
hip.hipHostMalloc(C.byref(h), 1 << 20, 0)
t0 = time.perf_counter()
for _ in range(1000):
    hip.hipMemcpyAsync(d, h, n, 1, None)
    hip.hipStreamSynchronize(None)
out["memcpy_async_sync_us"] = round((time.perf_counter() - t0) * 1e3, 3)
print(json.dumps(out))
