#!/usr/bin/env python3
"""Launch length of flat-XOR stream passes (knob xor_tiles_per_slot: the most 4 KiB tiles per
resident workgroup in one launch, 0 = one launch per pass): 10 -> 4 and flat_xor_hd (10,6) at 1 MiB
x 256 stripes, (3,3) at 1 MiB x 1024 stripes; interleaved rounds, median; every variant's
output checked against the one-launch pass."""
import json
import os
import random
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

LIMITS = [0, 16, 32, 64, 128]


def main():
    d = _lib.dev()
    F = 1 << 20
    st = D.Stream()
    for k, m, S in ((10, 4, 256), (10, 6, 256), (3, 3, 1024)):
        lay = D.Layout.alloc(k + m, F, S)
        lay.fill_splitmix(nfrags=k, stream=st)
        rnd = random.Random(k * 31 + m)
        masks = [rnd.randrange(1, 1 << k) for _ in range(m)]
        algo = S * (k + m) * F

        def fn():
            D.xor_apply(masks, lay, list(range(k)), list(range(k, k + m)), stream=st)

        ref = None
        for lim in LIMITS:
            d.ecamd_tune(b"xor_tiles_per_slot", lim)
            lay.buf.zero()
            lay.fill_splitmix(nfrags=k, stream=st)
            fn()
            st.synchronize()
            got = lay.download_stripes()
            if ref is None:
                ref = got
            assert (got == ref).all(), lim
        times = {lim: [] for lim in LIMITS}
        for _ in range(3):
            for lim in LIMITS:
                d.ecamd_tune(b"xor_tiles_per_slot", lim)
                ev = [D.Event() for _ in range(13)]
                ev[0].record(st)
                for i in range(12):
                    fn()
                    ev[i + 1].record(st)
                st.synchronize()
                times[lim].append(statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(3, 12)))
        for lim, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"shape": f"{k}to{m}", "S": S, "xor_tiles_per_slot": lim, "ms": round(med, 4),
                              "TBps": round(algo / med / 1e9, 3)}), flush=True)
        lay.buf.free()
    d.ecamd_tune(b"xor_tiles_per_slot", -1)  # the library default


if __name__ == "__main__":
    main()
