#!/usr/bin/env python3
"""Byte-split vs nibble LDS tables for the gf16 kernel at the BASELINE shapes (C2, C3, C5):
encode and the decode patterns of SURVEY §8(d), several geometries, interleaved rounds in one
process, median reported; nibble outputs are checked bit-exact against the byte-table outputs."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

CONFIGS = {"c2": (4, 2, 64 * 1024, 4096, [0, 1]),
           "c3": (10, 4, 1 << 20, 256, [0, 1, 2, 3]),
           "c5": (20, 8, 4 << 20, 32, list(range(8)))}
GEOMS = [(0, 0), (256, 8), (256, 4), (512, 4), (512, 2), (1024, 1)]


def timed(fn, stream, reps=3):
    a, b = D.Event(), D.Event()
    fn()
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    return a.elapsed_ms(b) / reps


def main():
    d = _lib.dev()
    st = D.Stream()
    rounds = int(os.environ.get("ROUNDS", "5"))

    def tune(nib, threads, wgs):
        d.ecamd_tune(b"nib", nib)
        d.ecamd_tune(b"threads", threads)
        d.ecamd_tune(b"wgs_per_cu", wgs)

    variants, algo = {}, {}
    for name, (k, m, F, S, miss) in CONFIGS.items():
        lay = D.Layout.alloc(k + m, F, S)
        lay.fill_splitmix(nfrags=k, stream=st)
        for nib in (0, 1):
            for threads, wgs in GEOMS:
                if nib == 0 and (threads, wgs) not in ((0, 0),):
                    continue
                tag = f"{name}_{'nib' if nib else 'byte'}_t{threads}_w{wgs}"

                def enc(lay=lay, k=k, m=m, nib=nib, threads=threads, wgs=wgs):
                    tune(nib, threads, wgs)
                    D.rs_encode(k, m, lay, stream=st)

                def dec(lay=lay, k=k, m=m, miss=miss, nib=nib, threads=threads, wgs=wgs):
                    tune(nib, threads, wgs)
                    D.rs_decode(k, m, miss, lay, stream=st)
                variants["enc_" + tag] = enc
                variants["dec_" + tag] = dec
                algo["enc_" + tag] = S * (k + m) * F
                algo["dec_" + tag] = S * (k + m) * F
        # bit-exactness of the nibble path on this shape
        tune(0, 0, 0)
        D.rs_encode(k, m, lay, stream=st)
        D.rs_decode(k, m, miss, lay, stream=st)
        st.synchronize()
        ref = lay.buf.download(lay.stripe_stride * 2)
        lay.buf.zero()
        lay.fill_splitmix(nfrags=k, stream=st)
        tune(1, 0, 0)
        D.rs_encode(k, m, lay, stream=st)
        D.rs_decode(k, m, miss, lay, stream=st)
        st.synchronize()
        ok = bool((lay.buf.download(lay.stripe_stride * 2) == ref).all())
        print(json.dumps({"check": name, "nib_bit_exact": ok}), flush=True)
        if not ok:
            sys.exit(1)
    times = {n: [] for n in variants}
    for r in range(rounds):
        for n, fn in variants.items():
            if r == 0:
                print(json.dumps({"start": n}), flush=True)
            times[n].append(timed(fn, st))
        print(json.dumps({"round": r}), flush=True)
    tune(0, 0, 0)
    for n, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"variant": n, "ms": round(med, 4), "GBps": round(algo[n] / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
