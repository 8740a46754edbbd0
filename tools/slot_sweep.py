#!/usr/bin/env python3
"""Launch length of stream passes (knob tiles_per_slot: the most tiles per resident workgroup in
one launch; longer batches run as several launches): C3 encode / decode at 256 and 2048 stripes
and C2 at 4096 stripes, 16 ... 4096 tiles per slot, interleaved rounds, median of steady passes
(HIP events over the whole pass)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

CASES = [("c3", 10, 4, 1 << 20, 256, [0, 1, 2, 3]), ("c3", 10, 4, 1 << 20, 2048, [0, 1, 2, 3]),
         ("c2", 4, 2, 64 << 10, 4096, [0, 1])]
SLOTS = [16, 32, 48, 64, 128, 4096]


def timed(fn, st, n=16, skip=4):
    ev = [D.Event() for _ in range(n + 1)]
    ev[0].record(st)
    for i in range(n):
        fn()
        ev[i + 1].record(st)
    st.synchronize()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n))


def main():
    d = _lib.dev()
    st = D.Stream()
    for cfg, k, m, F, S, lost in CASES:
        lay = D.Layout.alloc(k + m, F, S)
        lay.fill_splitmix(nfrags=k, stream=st)
        res = {}
        for rnd in range(3):
            for tps in SLOTS:
                d.ecamd_tune(b"tiles_per_slot", tps)
                for op, fn in (("enc", lambda: D.rs_encode(k, m, lay, stream=st)),
                               ("dec", lambda: D.rs_decode(k, m, lost, lay, stream=st))):
                    res.setdefault((tps, op), []).append(timed(fn, st))
        for (tps, op), ms in sorted(res.items()):
            med = statistics.median(ms)
            print(json.dumps({"cfg": cfg, "S": S, "tiles_per_slot": tps, "op": op, "ms": round(med, 4),
                              "TBps": round(S * (k + m) * F / (med * 1e-3) / 1e12, 3)}), flush=True)
        lay.buf.free()
    d.ecamd_tune(b"tiles_per_slot", 0)


if __name__ == "__main__":
    main()
