#!/usr/bin/env python3
"""C5's real ceiling: the 20-read / 8-write stream of a C5 pass (k=20 m=8, 4 MiB
fragments, 32 stripes) with no compute, in the codec's own launch shapes -- one workgroup per tile
(ecamd_probe_mix4 with wgs_per_cu 0) under per-CU residency caps (dynamic LDS share, as the codec's
cap_lds) -- beside the bitsliced codec's passes of the same patterns at its default and at its 16 KiB
tile caps (knob bs_tile_per_cu).  Interleaved rounds; one JSON line per (round, shape, pattern).

usage: python tools/c5_ceiling.py [rounds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 20, 8, 4 << 20, 32
PATTERNS = {"encode": None, "data_0_7": list(range(8)), "mixed": [0, 2, 4, 6, 20, 22, 24, 26]}
# (threads, wave_contig, caps): 16 KiB four-wave tiles (the C5 codec's), 8 KiB two-wave and 4 KiB one-wave tiles,
# 4 chunks of 16 B per lane as the bitsliced kernel's transposes need; cap 0 = resident as registers allow
SHAPES = [(256, 1, [0, 1, 2, 3, 4]), (256, 0, [0, 2]), (128, 1, [0, 2, 3, 4, 6, 8]),
          (64, 1, [0, 4, 6, 7, 8, 10, 12, 16])]


def main(rounds=3, reps=20, warm=10):
    d, p = _lib.dev(), _lib.probe()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    d.ecamd_tune(b"bitslice", 2)
    D.rs_encode(K, M, lay, stream=st)
    algo = S * (K + M) * F
    a, b = D.Event(), D.Event()

    def timed(fn):
        for _ in range(warm):
            fn()
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        st.synchronize()
        return a.elapsed_ms(b) / reps

    def frac(ms):
        return round(algo / (ms * 1e-3) / 8e12, 4)

    def codec(lost):
        if lost is None:
            D.rs_encode(K, M, lay, stream=st)
        else:
            D.rs_decode(K, M, lost, lay, stream=st)

    for _ in range(25):  # clock settle
        codec(None)
    for rnd in range(rounds):
        for name, lost in PATTERNS.items():
            if lost is None:
                order = list(range(K + M))
            else:
                order = [f for f in range(K + M) if f not in lost][:K] + sorted(lost)
            frag = _lib.ints(order)
            for threads, wc, caps in SHAPES:
                for cap in caps:
                    ms = timed(lambda: _lib.check(p.ecamd_probe_mix4(2, 2, 4, threads, 0, cap, wc, lay.buf.ptr, F, K,
                                                                     M, S, frag, st.handle), "mix4"))
                    print(json.dumps({"round": rnd, "pattern": name, "probe": f"t{threads}_wc{wc}_cap{cap}",
                                      "ms": round(ms, 4), "frac": frac(ms)}), flush=True)
            for cap in (-1, 1, 2, 3):  # the codec: default, then 16 KiB tiles capped at 1 / 2 / 3 per CU
                d.ecamd_tune(b"bs_tile_per_cu", cap)
                ms = timed(lambda: codec(lost))
                print(json.dumps({"round": rnd, "pattern": name, "codec": f"tile_per_cu{cap}",
                                  "ms": round(ms, 4), "frac": frac(ms)}), flush=True)
            d.ecamd_tune(b"bs_tile_per_cu", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
