#!/usr/bin/env python3
"""Flat-XOR kernel A/B on one GPU (development tool): xor_stream_kernel (buffer loads, unrolled
inputs) against xor_apply_kernel, at 10 inputs -> 4 outputs and the flat_xor_hd (10,6) shape, 1 MiB
fragments; output of every variant checked against the first."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main():
    d = _lib.dev()
    F, S = 1 << 20, 256
    out = open(os.path.join(ROOT, "gpurun_out", "xor_sweep.jsonl"), "w")
    for k, m in ((10, 4), (10, 6), (3, 3)):
        lay = D.Layout.alloc(k + m, F, S if k > 3 else 4 * S)
        st = D.Stream()
        lay.fill_splitmix(nfrags=k, stream=st)
        import random
        rnd = random.Random(k * 31 + m)
        masks = [rnd.randrange(1, 1 << k) for _ in range(m)]
        algo = lay.nstripes * (k + m) * F
        variants = {}
        for stream, wgs in ((0, 0), (1, 1), (1, 2), (1, 3)):
            def fn(stream=stream, wgs=wgs):
                d.ecamd_tune(b"stream", stream)
                d.ecamd_tune(b"xor_wgs", wgs)
                D.xor_apply(masks, lay, list(range(k)), list(range(k, k + m)), stream=st)
            variants[f"xor_{k}to{m}_{'old' if not stream else 'st'}_w{wgs}"] = fn
        ref = None
        for n, fn in variants.items():
            fn()
            st.synchronize()
            got = lay.buf.download(lay.stripe_stride * 2)
            if ref is None:
                ref = got
            ok = bool((got == ref).all())
            print(json.dumps({"check": n, "same_as_first": ok}), flush=True)
        a, b = D.Event(), D.Event()
        times = {n: [] for n in variants}
        for _ in range(7):
            for n, fn in variants.items():
                fn()
                a.record(st)
                for _ in range(3):
                    fn()
                b.record(st)
                times[n].append(a.elapsed_ms(b) / 3)
        for n, ts in times.items():
            med = statistics.median(ts)
            r = {"variant": n, "ms": round(med, 4), "GBps": round(algo / med / 1e6, 1)}
            out.write(json.dumps(r) + "\n")
            print(json.dumps(r), flush=True)
        lay.buf.free()
    d.ecamd_tune(b"stream", 1)
    d.ecamd_tune(b"xor_wgs", 0)


if __name__ == "__main__":
    main()
