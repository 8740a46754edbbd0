#!/usr/bin/env python3
"""Why does the C3 stream kernel's rate drift down with the batch (tools/c3_size_sweep.py)?
Separates the address span a launch sweeps from the work in it, single pass (grid_mult 1):
  * compact   -- S stripes back to back (stripe stride 14 MiB);
  * spread    -- 256 stripes placed 8 stripe slots apart (the span of 2048 stripes, the work of 256);
  * split8    -- 2048 stripes as 8 launches of 256 back to back (the work of 2048, spans of 256).
Median of steady launches (HIP events), TB/s of algorithmic bytes."""
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


def timed(fns, st, n=16, skip=4):
    ev = [D.Event() for _ in range(n + 1)]
    ev[0].record(st)
    for i in range(n):
        for fn in fns:
            fn()
        ev[i + 1].record(st)
    st.synchronize()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n))


def main():
    d = _lib.dev()
    d.ecamd_tune(b"grid_mult", 1)
    st = D.Stream()
    big = D.Layout.alloc(K + M, F, 2048)
    big.fill_splitmix(nfrags=K, stream=st)
    fs, ss = big.frag_stride, big.stripe_stride

    def mk(S, stride=ss, first=0):
        L = D.Layout(big.buf, K + M, F, S, fs, stride)
        L.base = big.buf.ptr + first * ss
        return L

    def enc(L):
        return lambda: _lib.check(d.ecamd_rs_encode(K, M, L.base, L.stripe_stride, L.frag_stride,
                                                    F, L.nstripes, st.handle), "encode")

    cases = [("compact_256", [mk(256)], 256), ("spread_256x8", [mk(256, 8 * ss)], 256),
             ("compact_2048", [mk(2048)], 2048),
             ("split8_2048", [mk(256, ss, 256 * i) for i in range(8)], 2048),
             ("compact_512", [mk(512)], 512), ("spread_256x2", [mk(256, 2 * ss)], 256)]
    for rnd in range(2):
        for name, lays, S in cases:
            ms = timed([enc(L) for L in lays], st)
            print(json.dumps({"round": rnd, "case": name, "ms": round(ms, 4),
                              "TBps": round(S * (K + M) * F / (ms * 1e-3) / 1e12, 3)}), flush=True)
    d.ecamd_tune(b"grid_mult", 0)
    big.buf.free()


if __name__ == "__main__":
    main()
