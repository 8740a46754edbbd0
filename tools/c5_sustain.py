#!/usr/bin/env python3
"""Sustained C5 launches (k=20, m=8, 4 MiB, 32 stripes): per-launch HIP-event times of 40
back-to-back encodes / decodes of 8 lost fragments, bitsliced vs LDS-table kernel, to see clock /
power behaviour over time rather than a short burst."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 20, 8, 4 << 20, 32


def main(n=40):
    d = _lib.dev()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    D.rs_encode(K, M, lay, stream=st)
    algo = S * (K + M) * F
    for mode in (2, 0, 2, 0):
        d.ecamd_tune(b"bitslice", mode)
        for op, fn in (("encode", lambda: D.rs_encode(K, M, lay, stream=st)),
                       ("decode", lambda: D.rs_decode(K, M, list(range(8)), lay, stream=st))):
            fn()
            st.synchronize()
            ev = [D.Event() for _ in range(n + 1)]
            ev[0].record(st)
            for i in range(n):
                fn()
                ev[i + 1].record(st)
            st.synchronize()
            ms = [ev[i].elapsed_ms(ev[i + 1]) for i in range(n)]
            print(json.dumps({"kernel": "bitslice" if mode else "lds", "op": op,
                              "first5_TBps": [round(algo / x / 1e9, 2) for x in ms[:5]],
                              "last5_TBps": [round(algo / x / 1e9, 2) for x in ms[-5:]],
                              "mean_TBps": round(algo * n / sum(ms) / 1e9, 3)}), flush=True)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
