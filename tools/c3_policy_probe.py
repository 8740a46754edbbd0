#!/usr/bin/env python3
"""Cache-policy probe at the C3 codec's launch shape (round 6): the 10-read / 4-write stream of a C3 pass
(k=10 m=4, 1 MiB fragments, 256 stripes) with no compute, one ONE-wave workgroup per 4 KiB tile (4 chunks of
16 B per lane, 1 KiB apart: ecamd_bs_kernel's one-wave form), 7 resident per CU (its cap), for every
(load, store) cache-policy pair instantiated (ECAMD_MIX_POLICIES; gfx950 cpol bits 1 sc0, 2 nt, 16 sc1).
The codec uses (2, 2).  Interleaved rounds; one JSON line per (round, pattern, policy).

usage: python tools/c3_policy_probe.py [rounds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 10, 4, 1 << 20, 256
POLICIES = [(0, 0), (0, 2), (0, 16), (0, 18), (0, 1), (2, 0), (2, 2), (2, 16), (2, 18), (2, 1), (1, 0), (1, 2),
            (16, 2), (18, 2), (3, 2), (18, 18)]
PATTERNS = {"encode": list(range(K + M)), "mixed": [1, 2, 3, 4, 6, 7, 8, 9, 11, 12, 0, 5, 10, 13]}


def main(rounds=3, reps=20, warm=10):
    p = _lib.probe()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    a, b = D.Event(), D.Event()
    algo = S * (K + M) * F

    def timed(fn):
        for _ in range(warm):
            fn()
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        st.synchronize()
        return a.elapsed_ms(b) / reps

    for rnd in range(rounds):
        for name, order in PATTERNS.items():
            frag = _lib.ints(order)
            for lp, sp in POLICIES:
                ms = timed(lambda: _lib.check(p.ecamd_probe_mix4(lp, sp, 4, 64, 0, 7, 1, lay.buf.ptr, F, K, M, S, frag,
                                                                 st.handle), "mix4"))
                print(json.dumps({"round": rnd, "pattern": name, "policy": f"{lp}_{sp}", "ms": round(ms, 4),
                                  "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
