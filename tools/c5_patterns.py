#!/usr/bin/env python3
"""Rebuild-8 rate by erasure pattern at C5 (k=20 m=8, 4 MiB, 32 stripes), bitsliced kernels: which
patterns run slower than others at the same network size, and whether the fragment layout
(interleaved reads and writes) explains it.  Interleaved rounds, steady launches only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 20, 8, 4 << 20, 32
PATTERNS = {
    "data_0_7": list(range(8)),
    "data_12_19": list(range(12, 20)),
    "mixed_even": [0, 2, 4, 6, 20, 22, 24, 26],
    "data_even": [0, 2, 4, 6, 8, 10, 12, 14],
    "data_4_parity_4": [0, 1, 2, 3, 24, 25, 26, 27],
    "mixed_odd": [1, 3, 5, 7, 21, 23, 25, 27],
}


def main(n=30, skip=10, rounds=2):
    d = _lib.dev()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    d.ecamd_tune(b"bitslice", 2)
    D.rs_encode(K, M, lay, stream=st)
    for p in PATTERNS.values():
        D.rs_decode(K, M, p, lay, stream=st)
    st.synchronize()
    for _ in range(25):
        D.rs_encode(K, M, lay, stream=st)
    algo = S * (K + M) * F
    for rnd in range(rounds):
        for name, p in PATTERNS.items():
            ev = [D.Event() for _ in range(n + 1)]
            ev[0].record(st)
            for i in range(n):
                D.rs_decode(K, M, p, lay, stream=st)
                ev[i + 1].record(st)
            st.synchronize()
            ms = [ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n)]
            avg = sum(ms) / len(ms)
            print(json.dumps({"round": rnd, "pattern": name, "lost": p, "steady_ms": round(avg, 4),
                              "frac": round(algo / avg / 1e9 / 8, 4)}), flush=True)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
