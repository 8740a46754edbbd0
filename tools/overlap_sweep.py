#!/usr/bin/env python3
"""Overlapped launches within a stream pass (knob stream_overlap: odd launches of a split pass on a
second stream, forked from / joined into the caller's) against in-order launches, at 8 ... 64
tiles per resident workgroup per launch (knob tiles_per_slot): C3 encode / decode at 256 and 2048
stripes, interleaved rounds, median of steady passes; outputs checked against the defaults'.

Measured and rejected (profiles/r02_overlap_sweep.log): overlapping loses 1-13% except at 8 tiles
per slot, where the launch boundaries dominate -- a boundary's value is that it starts every
workgroup in step again, which overlap gives up.  The knob was removed from libecamd again; against
the current library this script times the in-order variants twice."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F = 10, 4, 1 << 20
LOST = [0, 1, 2, 3]
VARIANTS = [(ov, lim) for ov in (0, 1) for lim in (8, 16, 32, 64)]


def main():
    d = _lib.dev()
    st = D.Stream()
    for S in (256, 2048):
        lay = D.Layout.alloc(K + M, F, S)
        lay.fill_splitmix(nfrags=K, stream=st)
        D.rs_encode(K, M, lay, stream=st)
        st.synchronize()
        if S <= 256:
            ref = lay.download_stripes()
            host = ref.copy()
            host[:, K:] = 0
            for ov, lim in VARIANTS:
                d.ecamd_tune(b"stream_overlap", ov)
                d.ecamd_tune(b"tiles_per_slot", lim)
                lay.upload_stripes(host)
                D.rs_encode(K, M, lay, stream=st)
                st.synchronize()
                assert (lay.download_stripes() == ref).all(), (ov, lim)
        times = {}
        for _ in range(3):
            for v in VARIANTS:
                d.ecamd_tune(b"stream_overlap", v[0])
                d.ecamd_tune(b"tiles_per_slot", v[1])
                for op, fn in (("enc", lambda: D.rs_encode(K, M, lay, stream=st)),
                               ("dec", lambda: D.rs_decode(K, M, LOST, lay, stream=st))):
                    ev = [D.Event() for _ in range(13)]
                    ev[0].record(st)
                    for i in range(12):
                        fn()
                        ev[i + 1].record(st)
                    st.synchronize()
                    times.setdefault(v + (op,), []).append(
                        statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(3, 12)))
        for key, ts in sorted(times.items()):
            med = statistics.median(ts)
            print(json.dumps({"S": S, "overlap": key[0], "tiles_per_slot": key[1], "op": key[2],
                              "ms": round(med, 4), "TBps": round(S * (K + M) * F / (med * 1e-3) / 1e12, 3)}),
                  flush=True)
        lay.buf.free()
    d.ecamd_tune(b"stream_overlap", 0)
    d.ecamd_tune(b"tiles_per_slot", 0)


if __name__ == "__main__":
    main()
