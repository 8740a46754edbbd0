#!/usr/bin/env python3
"""End-to-end (host memory -> GPU -> host memory) rates for DESIGN.md.

1. pipeline: S stripes of k x F in PINNED host memory; batches of B stripes run
   H2D(data) -> encode kernel -> D2H(parity) on 3 rotating streams, so PCIe in, the kernel and
   PCIe out of consecutive batches overlap.  Same for decode (H2D k available -> D2H rebuilt).
2. per-call API: liberasurecode_encode / liberasurecode_decode (liberasurecode.so.1) from
   pageable memory on T threads, 10 MiB objects (C3) -- the drop-in path as Swift would use it.
Rates are GiB/s of object data (k*F per stripe).  Prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

GIB = float(1 << 30)


def pinned(nbytes):
    p = C.c_void_p()
    _lib.check(_lib.dev().ecamd_host_alloc(C.byref(p), nbytes), "host_alloc")
    return p.value


def pipeline(k, m, F, S, B, missing):
    d = _lib.dev()
    h_in = pinned(S * k * F)
    h_out = pinned(S * max(m, len(missing)) * F)
    C.memset(h_in, 0x5A, S * k * F)
    nslot = 3
    lays = [D.Layout.alloc(k + m, F, B) for _ in range(nslot)]
    streams = [D.Stream() for _ in range(nslot)]

    def run(decode):
        nb = S // B
        t0 = time.perf_counter()
        for b in range(nb):
            lay, st = lays[b % nslot], streams[b % nslot]
            ins = ([i for i in range(k + m) if i not in missing][:k]) if decode else list(range(k))
            outs = missing if decode else list(range(k, k + m))
            for s in range(B):
                for j, f in enumerate(ins):
                    src = h_in + ((b * B + s) * k + j) * F
                    dst = lay.buf.ptr + s * lay.stripe_stride + f * lay.frag_stride
                    _lib.check(d.ecamd_memcpy_async(dst, src, F, 0, st.handle), "h2d")
            if decode:
                D.rs_decode(k, m, missing, lay, stream=st)
            else:
                D.rs_encode(k, m, lay, stream=st)
            for s in range(B):
                for j, f in enumerate(outs):
                    src = lay.buf.ptr + s * lay.stripe_stride + f * lay.frag_stride
                    dst = h_out + ((b * B + s) * len(outs) + j) * F
                    _lib.check(d.ecamd_memcpy_async(dst, src, F, 1, st.handle), "d2h")
        for st in streams:
            st.synchronize()
        return (S // B) * B * k * F / GIB / (time.perf_counter() - t0)

    run(False)  # warm
    enc = max(run(False) for _ in range(2))
    dec = max(run(True) for _ in range(2))
    return enc, dec


def per_call(k, m, F, threads, objects):
    import ec_api as E
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, hd=m)
    assert desc > 0, desc
    data = os.urandom(k * F)

    def enc_job(_):
        rc, dp, pp, flen = E.encode(desc, data)
        assert rc == 0
        E.lib().liberasurecode_encode_cleanup(desc, dp, pp)

    rc, dp, pp, flen = E.encode(desc, data)
    frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    avail = frags[m:] if m <= k else frags[:k]

    def dec_job(_):
        rc, out = E.decode(desc, avail, flen)
        assert rc == 0

    # The caller's own read of the results, GIL-free (ctypes.memmove releases the GIL; string_at,
    # which dec_job's E.decode uses, holds it for the whole 10 MiB copy, so 8 Python threads
    # serialise on it -- a harness limit, not the library's): every output byte copied once into
    # a per-thread buffer, for encode (the k + m fragments) and decode (the object) alike.
    import ctypes as C
    import threading
    tls = threading.local()

    def scratch():
        if not hasattr(tls, "buf"):
            tls.buf = C.create_string_buffer(k * F + (k + m) * (flen + 64))
        return C.addressof(tls.buf)

    arr = (C.c_char_p * len(avail))(*avail)

    def enc_consume(_):
        rc, dp, pp, fl = E.encode(desc, data)
        assert rc == 0
        dst = scratch()
        for i in range(k):
            C.memmove(dst + i * fl, dp[i], fl)
        for i in range(m):
            C.memmove(dst + (k + i) * fl, pp[i], fl)
        E.lib().liberasurecode_encode_cleanup(desc, dp, pp)

    def dec_consume(_):
        out, olen = C.c_void_p(), C.c_uint64()
        rc = E.lib().liberasurecode_decode(desc, arr, len(avail), flen, 0, C.byref(out), C.byref(olen))
        assert rc == 0
        C.memmove(scratch(), out.value, olen.value)
        E.lib().liberasurecode_decode_cleanup(desc, out)

    res = {}
    with ThreadPoolExecutor(threads) as ex:
        for name, job in (("encode", enc_job), ("decode", dec_job), ("encode_consumed", enc_consume),
                          ("decode_consumed", dec_consume)):
            list(ex.map(job, range(threads)))
            t0 = time.perf_counter()
            list(ex.map(job, range(objects)))
            res[name] = objects * k * F / GIB / (time.perf_counter() - t0)
    E.lib().liberasurecode_instance_destroy(desc)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=96)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--objects", type=int, default=64)
    ap.add_argument("--per-call-only", action="store_true",
                    help="only the per-call API leg (A/B runs of frontend switches)")
    args = ap.parse_args()
    k, m, F = 10, 4, 1 << 20
    if args.per_call_only:
        pc = per_call(k, m, F, args.threads, args.objects)
        print(json.dumps({"per_call_api_encode_gibs": round(pc["encode"], 2),
                          "per_call_api_decode_gibs": round(pc["decode"], 2),
                          "per_call_api_encode_consumed_gibs": round(pc["encode_consumed"], 2),
                          "per_call_api_decode_consumed_gibs": round(pc["decode_consumed"], 2),
                          "threads": args.threads, "objects": args.objects,
                          "frontend_zero_all": os.environ.get("ECAMD_FRONTEND_ZERO_ALL", "0"),
                          "copy_threads": os.environ.get("ECAMD_COPY_THREADS", "4")}))
        return
    enc, dec = pipeline(k, m, F, args.stripes, args.batch, [0, 1, 2, 3])
    pc = per_call(k, m, F, args.threads, args.objects)
    print(json.dumps({"e2e_pipeline_encode_gibs": round(enc, 2),
                      "e2e_pipeline_decode_gibs": round(dec, 2),
                      "per_call_api_encode_gibs": round(pc["encode"], 2),
                      "per_call_api_decode_gibs": round(pc["decode"], 2),
                      "config": f"k={k} m={m} F=1MiB, pipeline {args.stripes} stripes in batches of "
                                f"{args.batch} on 3 streams from pinned memory; per-call API "
                                f"{args.objects} x 10 MiB objects on {args.threads} threads"}))


if __name__ == "__main__":
    main()
