#!/usr/bin/env python3
"""Launch-shape ceiling of the codec's access patterns (development tool): the codec-shaped streaming
probe (ecamd_probe_mix3: K fragment reads + R writes per tile, no table work) as a grid-stride launch
over 4 resident workgroups per CU against one workgroup per tile (grid = tiles; the dispatcher hands
each freed slot the next tile), for tile widths of 4 / 8 / 16 / 32 KiB per fragment and 1 or 2
launches per pass; shapes C3 (10+4, 1 MiB, 256 stripes), flat-XOR (10+6) and C5 (20+8, 4 MiB, 32
stripes). Median of interleaved rounds, TB/s of the algorithmic bytes."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

SHAPES = [("c3", 10, 4, 1 << 20, 256), ("xor_10_6", 10, 6, 1 << 20, 256), ("c5", 20, 8, 4 << 20, 32)]
# (name, threads, ch, wgs_per_cu); wgs_per_cu 0 = one workgroup per tile
GEOMS = [("stride_4k", 256, 1, 4), ("stride_4k_x2", 256, 1, 8), ("tile_4k", 256, 1, 0), ("tile_8k", 256, 2, 0),
         ("tile_16k", 1024, 1, 0), ("tile_32k", 1024, 2, 0)]


def main(rounds=3, reps=10):
    p = _lib.probe()
    st = D.Stream()
    for name, K, R, F, S in SHAPES:
        lay = D.Layout.alloc(K + R, F, S)
        lay.fill_splitmix(nfrags=K, stream=st)
        ss = lay.stripe_stride

        def mk(threads, ch, wgs, nl):
            per = S // nl
            w = wgs if wgs else 1 << 20

            def fn():
                for i in range(nl):
                    _lib.check(p.ecamd_probe_mix3(2, 2, ch, threads, w, 0, 0, lay.buf.ptr + i * per * ss, F, K, R,
                                                  per, None, st.handle), "mix3")
            return fn
        variants = {f"{g}_{nl}l": mk(t, c, w, nl) for g, t, c, w in GEOMS for nl in (1, 2)}
        for _ in range(30):
            variants["stride_4k_2l"]()
        times = {}
        for _ in range(rounds):
            for vn, fn in variants.items():
                fn()
                a, b = D.Event(), D.Event()
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                st.synchronize()
                times.setdefault(vn, []).append(a.elapsed_ms(b) / reps)
        algo = S * (K + R) * F
        for vn, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"shape": name, "variant": vn, "ms": round(med, 4),
                              "TBps": round(algo / (med * 1e-3) / 1e12, 3),
                              "frac": round(algo / (med * 1e-3) / 8e12, 4)}), flush=True)
        lay.buf.free()


if __name__ == "__main__":
    main()
