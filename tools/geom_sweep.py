#!/usr/bin/env python3
"""Workgroup shape of the C3 stream kernel at 16 waves per CU -- 4 x 256, 2 x 512, 1 x 1024 threads
(knobs threads / wgs_per_cu) -- each with launches of 16 / 32 / 64 / 128 tiles per resident
workgroup (knob tiles_per_slot; a tile is threads x 16 B of every fragment): C3 encode / decode of
256 stripes, interleaved rounds, median; outputs checked against the default's."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 10, 4, 1 << 20, 256
LOST = [0, 1, 2, 3]
SHAPES = [(256, 4), (512, 2), (1024, 1)]
LIMITS = [16, 32, 64, 128]


def setv(d, thr, wgs, lim):
    d.ecamd_tune(b"threads", thr)
    d.ecamd_tune(b"wgs_per_cu", wgs)
    d.ecamd_tune(b"tiles_per_slot", lim)


def main():
    d = _lib.dev()
    st = D.Stream()
    lay = D.Layout.alloc(K + M, F, S)
    lay.fill_splitmix(nfrags=K, stream=st)
    D.rs_encode(K, M, lay, stream=st)
    st.synchronize()
    ref = lay.download_stripes()
    variants = [(t, w, l) for t, w in SHAPES for l in LIMITS]
    host = ref.copy()
    host[:, K:] = 0
    for v in variants:
        setv(d, *v)
        lay.upload_stripes(host)
        D.rs_encode(K, M, lay, stream=st)
        st.synchronize()
        assert (lay.download_stripes() == ref).all(), v
    times = {}
    for _ in range(3):
        for v in variants:
            setv(d, *v)
            for op, fn in (("enc", lambda: D.rs_encode(K, M, lay, stream=st)),
                           ("dec", lambda: D.rs_decode(K, M, LOST, lay, stream=st))):
                ev = [D.Event() for _ in range(15)]
                ev[0].record(st)
                for i in range(14):
                    fn()
                    ev[i + 1].record(st)
                st.synchronize()
                times.setdefault(v + (op,), []).append(
                    statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(4, 14)))
    for key, ts in sorted(times.items()):
        med = statistics.median(ts)
        print(json.dumps({"threads": key[0], "wgs_per_cu": key[1], "tiles_per_slot": key[2], "op": key[3],
                          "ms": round(med, 4), "TBps": round(S * (K + M) * F / (med * 1e-3) / 1e12, 3)}),
              flush=True)
    setv(d, 0, 0, 0)
    lay.buf.free()


if __name__ == "__main__":
    main()
