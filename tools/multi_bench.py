#!/usr/bin/env python3
"""Heterogeneous batch decode (ecamd_rs_decode_multi: one launch per distinct erasure pattern) at
the C3 shape: stripe-list stream launches, pointer-table stream kernel, first-version pointer kernel,
and a single-pattern strided decode for reference (development tool)."""
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
    algo = S * (k + m) * F
    a, b = D.Event(), D.Event()
    allpats = [[0, 1, 2, 3], [4, 5, 6, 7], [0, 5, 10, 13], [2, 3, 8, 9]]

    def timed(fn):
        ts = []
        for _ in range(7):
            fn()
            a.record(st)
            for _ in range(3):
                fn()
            b.record(st)
            ts.append(a.elapsed_ms(b) / 3)
        return statistics.median(ts)

    for npat in (1, 2, 4):
        pats = allpats[:npat]
        per = [pats[s % len(pats)] for s in range(S)]
        res = {}
        names = {(1, 1): "stripe_list", (1, 0): "ptrs_stream", (0, 0): "first_version"}
        for _ in range(2):
            for key in names:
                d.ecamd_tune(b"stream", key[0])
                d.ecamd_tune(b"multi_list", key[1])
                res.setdefault(key, []).append(timed(lambda: D.rs_decode_multi(k, m, per, lay, stream=st)))
        d.ecamd_tune(b"stream", 1)
        d.ecamd_tune(b"multi_list", 1)
        for key, ts in res.items():
            ms = min(ts)
            print(json.dumps({"decode_multi": names[key], "patterns": npat,
                              "ms": round(ms, 4), "GBps": round(algo / ms / 1e6, 1)}), flush=True)
    ms = timed(lambda: D.rs_decode(k, m, allpats[0], lay, stream=st))
    print(json.dumps({"decode_strided": allpats[0], "ms": round(ms, 4), "GBps": round(algo / ms / 1e6, 1)}))
    lay.buf.free()

    # flat_xor_hd (10, 6, 4): encode, single-pattern decode and a 4-pattern batch (stripe lists);
    # bytes = the fragments each launch reads and writes (read set differs per pattern: the sum
    # over the launch's plan inputs + outputs, counted per stripe)
    xk, xm, hd = 10, 6, 4
    lay = D.Layout.alloc(xk + xm, F, S)
    lay.fill_splitmix(nfrags=xk, stream=st)
    D.xor_encode(xk, xm, hd, lay, stream=st)
    xpats = [[0, 1, 2], [3, 7, 12], [4, 5, 6], [0, 9, 15]]
    per = [xpats[s % len(xpats)] for s in range(S)]
    for name, fn in (("xor_encode", lambda: D.xor_encode(xk, xm, hd, lay, stream=st)),
                     ("xor_decode_1pattern", lambda: D.xor_decode(xk, xm, hd, xpats[0], lay, stream=st)),
                     ("xor_decode_multi_4patterns", lambda: D.xor_decode_multi(xk, xm, hd, per, lay, stream=st))):
        ms = timed(fn)
        print(json.dumps({name: [xk, xm, hd], "ms": round(ms, 4),
                          "GiBps_object": round(S * xk * F / ms / 1e6 / 1.073741824, 1)}), flush=True)


if __name__ == "__main__":
    main()
