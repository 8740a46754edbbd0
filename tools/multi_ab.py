#!/usr/bin/env python3
"""A/B of ecamd_rs_decode_multi at the C3 shape (k=10 m=4, 1 MiB fragments): the 4 patterns of
tools/multi_bench.py over S stripes, grouped (64 consecutive stripes per pattern at S = 256) or
interleaved (stripe s has pattern s % 4), with knob multi_streams 1 / 2 / 4, beside the strided
single-pattern decode; interleaved rounds, bitsliced kernels (shipped; knob bitslice 2 for safety).
One JSON line per (round, case).  usage: python tools/multi_ab.py [rounds] [stripes]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F = 10, 4, 1 << 20
PATS = [[0, 1, 2, 3], [4, 5, 6, 7], [0, 5, 10, 13], [2, 3, 8, 9]]


def main(rounds=5, S=256, reps=10, warm=5):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    for _ in range(60):
        D.rs_encode(K, M, lay, stream=st)
    a, b = D.Event(), D.Event()
    algo = S * (K + M) * F
    grouped = [PATS[s * len(PATS) // S] for s in range(S)]
    inter = [PATS[s % len(PATS)] for s in range(S)]

    def timed(fn):
        for _ in range(warm):
            fn()
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        st.synchronize()
        return a.elapsed_ms(b) / reps

    cases = [("strided_0123", 1, lambda: D.rs_decode(K, M, PATS[0], lay, stream=st))]
    for streams in (1, 2, 4):
        cases.append((f"grouped_s{streams}", streams, lambda: D.rs_decode_multi(K, M, grouped, lay, stream=st)))
        cases.append((f"interleaved_s{streams}", streams, lambda: D.rs_decode_multi(K, M, inter, lay, stream=st)))
    for rnd in range(rounds):
        for name, streams, fn in cases:
            d.ecamd_tune(b"multi_streams", streams)
            ms = timed(fn)
            print(json.dumps({"round": rnd, "stripes": S, "case": name, "ms": round(ms, 4),
                              "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
    d.ecamd_tune(b"multi_streams", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5, int(sys.argv[2]) if len(sys.argv) > 2 else 256)
