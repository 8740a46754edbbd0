#!/usr/bin/env python3
"""Fixed vs per-stripe cost of the C3 stream kernel: encode / decode({0,1,2,3}) launch time at
S = 64 ... 1024 stripes (k=10 m=4, 1 MiB fragments), grid_mult 1 and 2 and the default policy (0), HIP events on the launch
stream, median of steady launches.  A straight-line fit t(S) = a + b*S separates the per-launch
ramp + tail (a) from the streaming rate (b) -- how much a better end-of-launch balance could win."""
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


def timed(fn, st, n=24, skip=6):
    ev = [D.Event() for _ in range(n + 1)]
    ev[0].record(st)
    for i in range(n):
        fn()
        ev[i + 1].record(st)
    st.synchronize()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n))


def main():
    d = _lib.dev()
    sizes = [int(x) for x in (sys.argv[1:] or ["64", "128", "256", "512", "1024"])]
    st = D.Stream()
    big = D.Layout.alloc(K + M, F, max(sizes))
    big.fill_splitmix(nfrags=K, stream=st)
    rows = []
    for rnd in range(2):
        for S in sizes:
            lay = D.Layout(big.buf, K + M, F, S, big.frag_stride, big.stripe_stride)
            for gm in (0, 1, 2):  # 0: the library's default policy
                d.ecamd_tune(b"grid_mult", gm)
                for op, fn in (("encode", lambda: D.rs_encode(K, M, lay, stream=st)),
                               ("decode", lambda: D.rs_decode(K, M, LOST, lay, stream=st))):
                    ms = timed(fn, st)
                    r = {"round": rnd, "S": S, "grid_mult": gm, "op": op, "ms": round(ms, 4),
                         "TBps": round(S * (K + M) * F / (ms * 1e-3) / 1e12, 3)}
                    rows.append(r)
                    print(json.dumps(r), flush=True)
    d.ecamd_tune(b"grid_mult", 0)
    for gm in (0, 1, 2):
        for op in ("encode", "decode"):
            pts = [(r["S"], r["ms"]) for r in rows if r["grid_mult"] == gm and r["op"] == op]
            n = len(pts)
            sx = sum(p[0] for p in pts)
            sy = sum(p[1] for p in pts)
            sxx = sum(p[0] ** 2 for p in pts)
            sxy = sum(p[0] * p[1] for p in pts)
            b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
            a = (sy - b * sx) / n
            print(json.dumps({"fit": op, "grid_mult": gm, "fixed_us": round(a * 1e3, 2),
                              "per_stripe_us": round(b * 1e3, 4),
                              "stream_TBps": round((K + M) * F / (b * 1e-3) / 1e12, 3)}), flush=True)
    big.buf.free()


if __name__ == "__main__":
    main()
