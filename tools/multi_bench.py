#!/usr/bin/env python3
"""Heterogeneous batch decode (ecamd_rs_decode_multi: one pointer-table launch per distinct erasure
pattern) at the C3 shape, stream kernel vs first version (development tool)."""
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
    k, m, F, S = 10, 4, 1 << 20, 256
    lay = D.Layout.alloc(k + m, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=k, stream=st)
    D.rs_encode(k, m, lay, stream=st)
    pats = [[0, 1, 2, 3], [4, 5, 6, 7], [0, 5, 10, 13], [2, 3, 8, 9]]
    per = [pats[s % len(pats)] for s in range(S)]
    algo = S * (k + m) * F
    a, b = D.Event(), D.Event()
    res = {}
    for stream in (1, 0, 1, 0):
        d.ecamd_tune(b"stream", stream)
        ts = []
        for _ in range(5):
            D.rs_decode_multi(k, m, per, lay, stream=st)
            a.record(st)
            for _ in range(3):
                D.rs_decode_multi(k, m, per, lay, stream=st)
            b.record(st)
            ts.append(a.elapsed_ms(b) / 3)
        res.setdefault(stream, []).append(statistics.median(ts))
    d.ecamd_tune(b"stream", 1)
    for stream, ts in res.items():
        ms = min(ts)
        print(json.dumps({"decode_multi": "stream" if stream else "first_version", "patterns": len(pats),
                          "ms": round(ms, 4), "GBps": round(algo / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
