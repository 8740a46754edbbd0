#!/usr/bin/env python3
"""LDS-table stream kernel launch shape A/B (development tool): grid-stride over the resident slots
(default) against a grid of one workgroup per `stream_chunk` consecutive 4 KiB tiles, the dispatcher
handing freed slots the next range (knob stream_chunk), each with the default launch length and as
one launch per pass; C3 encode and decode of data {0,1,2,3} (k=10 m=4, 1 MiB, 256 stripes) and C2
encode (k=4 m=2, 64 KiB, 4096 stripes). Interleaved rounds after a clock-settling warm-up, median per
pass (HIP events); every variant's outputs checked equal to the first's."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

CHUNKS = [int(x) for x in os.environ.get("CHUNKS", "0,1,2,4,8,16").split(",")]
SLOTS = [int(x) for x in os.environ.get("SLOTS", "0,1048576").split(",")]
SHAPES = [("c3", 10, 4, 1 << 20, 256), ("c2", 4, 2, 64 << 10, 4096)]


def main(rounds=3, reps=10):
    d = _lib.dev()
    st = D.Stream()
    for name, K, M, F, S in SHAPES:
        lay = D.Layout.alloc(K + M, F, S)
        lay.fill_splitmix(nfrags=K, stream=st)
        lost = list(range(min(M, 4)))
        ops = {"encode": lambda: D.rs_encode(K, M, lay, stream=st)}
        if name == "c3":
            ops["decode"] = lambda: D.rs_decode(K, M, lost, lay, stream=st)
        variants = [(c, t) for c in CHUNKS for t in SLOTS]
        ref = None
        for c, t in variants:
            d.ecamd_tune(b"stream_chunk", c)
            d.ecamd_tune(b"tiles_per_slot", t)
            for fn in ops.values():
                fn()
            st.synchronize()
            got = lay.download_stripes()
            if ref is None:
                ref = got
            assert bool((got == ref).all()), (name, c, t)
        d.ecamd_tune(b"stream_chunk", 0)
        d.ecamd_tune(b"tiles_per_slot", 0)
        for _ in range(60):
            ops["encode"]()
        times = {}
        for _ in range(rounds):
            for c, t in variants:
                d.ecamd_tune(b"stream_chunk", c)
                d.ecamd_tune(b"tiles_per_slot", t)
                for op, fn in ops.items():
                    fn()
                    a, b = D.Event(), D.Event()
                    a.record(st)
                    for _ in range(reps):
                        fn()
                    b.record(st)
                    st.synchronize()
                    times.setdefault((op, c, t), []).append(a.elapsed_ms(b) / reps)
        algo = S * (K + M) * F
        for (op, c, t), ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"shape": name, "op": op, "stream_chunk": c, "tiles_per_slot": t, "ms": round(med, 4),
                              "frac": round(algo / (med * 1e-3) / 8e12, 4)}), flush=True)
        d.ecamd_tune(b"stream_chunk", -1)
        d.ecamd_tune(b"tiles_per_slot", 0)
        lay.buf.free()


if __name__ == "__main__":
    main()
