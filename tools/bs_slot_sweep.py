#!/usr/bin/env python3
"""Launch length of bitsliced 8-output passes (knob bs_tiles_per_slot: the most 16 KiB tiles per
resident workgroup in one launch, 0 = one launch per pass): C5 shape (k=20 m=8, 4 MiB) encode and
rebuild of 8 data fragments at 32 / 64 / 128 stripes, interleaved rounds, median; outputs of
every variant checked against the one-launch pass."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F = 20, 8, 4 << 20
LOST = list(range(8))
LIMITS = [0, 8, 16, 32, 64]


def main():
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)  # wait for the compile
    st = D.Stream()
    for S in (32, 64, 128):
        lay = D.Layout.alloc(K + M, F, S)
        lay.fill_splitmix(nfrags=K, stream=st)
        D.rs_encode(K, M, lay, stream=st)
        D.rs_decode(K, M, LOST, lay, stream=st)
        st.synchronize()
        ref = lay.download_stripes()
        for lim in LIMITS:
            d.ecamd_tune(b"bs_tiles_per_slot", lim)
            D.rs_encode(K, M, lay, stream=st)
            D.rs_decode(K, M, LOST, lay, stream=st)
            st.synchronize()
            assert (lay.download_stripes() == ref).all(), (S, lim)
        times = {}
        for _ in range(3):
            for lim in LIMITS:
                d.ecamd_tune(b"bs_tiles_per_slot", lim)
                for op, fn in (("enc", lambda: D.rs_encode(K, M, lay, stream=st)),
                               ("dec8", lambda: D.rs_decode(K, M, LOST, lay, stream=st))):
                    ev = [D.Event() for _ in range(13)]
                    ev[0].record(st)
                    for i in range(12):
                        fn()
                        ev[i + 1].record(st)
                    st.synchronize()
                    times.setdefault((lim, op), []).append(
                        statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(3, 12)))
        for (lim, op), ts in sorted(times.items()):
            med = statistics.median(ts)
            algo = S * (K + (M if op == "enc" else 8)) * F
            print(json.dumps({"S": S, "bs_tiles_per_slot": lim, "op": op, "ms": round(med, 4),
                              "frac": round(algo / (med * 1e-3) / 8e12, 4)}), flush=True)
        lay.buf.free()
    d.ecamd_tune(b"bs_tiles_per_slot", 16)  # the library default
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
