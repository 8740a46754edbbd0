#!/usr/bin/env python3
"""Kernel-geometry sweep and bandwidth ceilings on one GPU (development tool).

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24): every variant is timed
once per round, R rounds, median reported.  Ceilings on the same 3.5 GiB working set:
  xor10to4  -- the flat-XOR kernel reading the same 10 fragments and writing 4 (no LDS work)
  d2d       -- hipMemcpyAsync device-to-device (bytes read + written)
"""
import argparse
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def timed(fn, stream, reps=3):
    a, b = D.Event(), D.Event()
    fn()
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    return a.elapsed_ms(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--F", type=int, default=1 << 20)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.jsonl"))
    args = ap.parse_args()
    k, m, F, S = args.k, args.m, args.F, args.S
    lay = D.Layout.alloc(k + m, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=k, stream=st)
    d = _lib.dev()
    algo = S * (k + m) * F

    variants = {}
    geoms = [(256, 3), (256, 4), (512, 2), (1024, 1)]
    for (threads, wgs), (tag, nt, ch, abl) in itertools.product(
            geoms, [("nt", 1, 0, 0), ("plain", 0, 0, 0), ("ch1", 1, 1, 0), ("ch2", 1, 2, 0),
                    ("abl1", 1, 1, 1), ("abl2", 1, 2, 1)]):
        def enc(threads=threads, wgs=wgs, nt=nt, ch=ch, abl=abl):
            d.ecamd_tune(b"threads", threads)
            d.ecamd_tune(b"wgs_per_cu", wgs)
            d.ecamd_tune(b"nt", nt)
            d.ecamd_tune(b"exp_ch", ch)
            d.ecamd_tune(b"ablate", abl)
            D.rs_encode(k, m, lay, stream=st)
        variants[f"enc_{tag}_t{threads}_w{wgs}"] = enc

    def reset():
        for key in (b"threads", b"wgs_per_cu", b"exp_ch", b"ablate"):
            d.ecamd_tune(key, 0)
        d.ecamd_tune(b"nt", 1)

    def dec():
        reset()
        D.rs_decode(k, m, list(range(min(m, k))), lay, stream=st)
    variants["dec_default"] = dec

    def enc_default():
        reset()
        D.rs_encode(k, m, lay, stream=st)
    variants["enc_default"] = enc_default

    masks = [(1 << k) - 1] * m

    def xor():
        D.xor_apply(masks, lay, list(range(k)), list(range(k, k + m)), stream=st)
    variants["xor10to4"] = xor

    half = lay.buf.nbytes // 2 // 16 * 16

    def d2d():
        _lib.check(d.ecamd_memcpy_async(lay.buf.ptr + half, lay.buf.ptr, half, 2, st.handle), "d2d")
    variants["d2d"] = d2d

    def scopy():
        _lib.check(d.ecamd_debug_stream_copy(lay.buf.ptr + half, lay.buf.ptr, half, st.handle),
                   "stream copy")
    variants["stream_copy"] = scopy

    for pad in (256, 4096, 65536 + 256):
        fs = F + pad
        buf = D.DeviceBuffer(fs * (k + m) * S)
        lp = D.Layout(buf, k + m, F, S, fs, fs * (k + m))
        lp.fill_splitmix(nfrags=k, stream=st)

        def encp(lp=lp):
            reset()
            D.rs_encode(k, m, lp, stream=st)
        variants[f"enc_pad{pad}"] = encp

    reset()
    D.rs_encode(k, m, lay, stream=st)
    st.synchronize()
    ref = lay.buf.download(lay.stripe_stride * 2)
    for ch in (1, 2):
        for threads, wgs in geoms:
            d.ecamd_tune(b"threads", threads)
            d.ecamd_tune(b"wgs_per_cu", wgs)
            d.ecamd_tune(b"exp_ch", ch)
            lay.buf.zero()
            lay.fill_splitmix(nfrags=k, stream=st)
            D.rs_encode(k, m, lay, stream=st)
            st.synchronize()
            ok = (lay.buf.download(lay.stripe_stride * 2) == ref).all()
            print(json.dumps({"check": f"exp_ch{ch}_t{threads}_w{wgs}", "bit_exact": bool(ok)}))
    reset()
    times = {n: [] for n in variants}
    for _ in range(args.rounds):
        for n, fn in variants.items():
            times[n].append(timed(fn, st))
    reset()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        for n, ts in times.items():
            med = statistics.median(ts)
            nbytes = 2 * half if n in ("d2d", "stream_copy") else algo
            rec = {"variant": n, "ms": round(med, 4), "min_ms": round(min(ts), 4),
                   "GBps": round(nbytes / med / 1e6, 1)}
            f.write(json.dumps(rec) + "\n")
            print(json.dumps(rec))


if __name__ == "__main__":
    main()
