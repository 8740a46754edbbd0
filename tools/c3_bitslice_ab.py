#!/usr/bin/env python3
"""A/B at C3 (k=10 m=4, 1 MiB, 256 stripes): the LDS-table stream kernel (default for <= 4 outputs)
against the bitsliced kernel built for 4 waves per SIMD (knob bitslice_min_rows 4), encode and
decode of data {0,1,2,3} and of the mixed {0,5,10,13}, interleaved rounds after a clock-settling warm-up, steady launches (HIP
events). The bitsliced kernel runs both launch shapes (knob bs_grid: 1 = one workgroup per tile,
0 = grid-stride over the resident slots)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 10, 4, 1 << 20, 256
LOST = [0, 1, 2, 3]
MIXED = [0, 5, 10, 13]  # SURVEY §8d's second C3 pattern: data and parity lost, writes interleaved


def main(rounds=3, n=30, skip=10):
    d = _lib.dev()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    d.ecamd_tune(b"bitslice", 2)
    d.ecamd_tune(b"bitslice_min_rows", 4)
    D.rs_encode(K, M, lay, stream=st)
    D.rs_decode(K, M, LOST, lay, stream=st)
    D.rs_decode(K, M, MIXED, lay, stream=st)
    ref = lay.download_stripes()
    d.ecamd_tune(b"bitslice_min_rows", 0)
    D.rs_encode(K, M, lay, stream=st)
    D.rs_decode(K, M, LOST, lay, stream=st)
    D.rs_decode(K, M, MIXED, lay, stream=st)
    assert (lay.download_stripes() == ref).all()
    d.ecamd_tune(b"bitslice_min_rows", 4)
    d.ecamd_tune(b"bs_grid", 0)
    D.rs_encode(K, M, lay, stream=st)
    D.rs_decode(K, M, LOST, lay, stream=st)
    D.rs_decode(K, M, MIXED, lay, stream=st)
    assert (lay.download_stripes() == ref).all()
    d.ecamd_tune(b"bs_grid", 1)
    for _ in range(60):  # settle the clocks
        D.rs_encode(K, M, lay, stream=st)
    st.synchronize()
    algo = S * (K + M) * F
    for rnd in range(rounds):
        for name, rows, grid in (("lds", 0, 1), ("bitslice_wg_per_tile", 4, 1), ("bitslice_slots", 4, 0)):
            d.ecamd_tune(b"bitslice_min_rows", rows)
            d.ecamd_tune(b"bs_grid", grid)
            for op, fn in (("encode", lambda: D.rs_encode(K, M, lay, stream=st)),
                           ("decode", lambda: D.rs_decode(K, M, LOST, lay, stream=st)),
                           ("decode_mixed", lambda: D.rs_decode(K, M, MIXED, lay, stream=st))):
                ev = [D.Event() for _ in range(n + 1)]
                ev[0].record(st)
                for i in range(n):
                    fn()
                    ev[i + 1].record(st)
                st.synchronize()
                ms = [ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n)]
                avg = sum(ms) / len(ms)
                print(json.dumps({"round": rnd, "kernel": name, "op": op, "ms": round(avg, 4),
                                  "frac": round(algo / (avg * 1e-3) / 8e12, 4)}), flush=True)
    d.ecamd_tune(b"bitslice_min_rows", 0)
    d.ecamd_tune(b"bs_grid", 1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
