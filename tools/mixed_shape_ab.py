#!/usr/bin/env python3
"""Launch shape of the LDS-table stream kernel for the C3 mixed decode {0,5,10,13} (development tool,
round 3): knobs tiles_per_slot (launch length) x grid_mult (resident workgroups per slot), beside the
contiguous decode {0,1,2,3} and the encode, interleaved rounds, median of steady passes (HIP
events), fraction of 8 TB/s of the algorithmic 14 MiB per stripe.  Every variant's bytes are
checked against the default's."""
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
OPS = {"encode": None, "decode_0123": [0, 1, 2, 3], "decode_mixed": [0, 5, 10, 13]}
SHAPES = [(tps, gm) for tps in (8, 16, 32, 64) for gm in (1, 2, 3)]


def timed(fn, st, n=16, skip=4):
    ev = [D.Event() for _ in range(n + 1)]
    ev[0].record(st)
    for i in range(n):
        fn()
        ev[i + 1].record(st)
    st.synchronize()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n))


def main(rounds=3):
    d = _lib.dev()
    st = D.Stream()
    lay = D.Layout.alloc(K + M, F, S)
    lay.fill_splitmix(nfrags=K, stream=st)

    def run(op):
        if OPS[op] is None:
            D.rs_encode(K, M, lay, stream=st)
        else:
            D.rs_decode(K, M, OPS[op], lay, stream=st)
    for op in OPS:
        run(op)
    ref = lay.download_stripes()
    for tps, gm in SHAPES:
        d.ecamd_tune(b"tiles_per_slot", tps)
        d.ecamd_tune(b"grid_mult", gm)
        for op in OPS:
            run(op)
        assert (lay.download_stripes() == ref).all(), (tps, gm)
    for _ in range(60):
        run("encode")
    algo = S * (K + M) * F
    res = {}
    for _ in range(rounds):
        for tps, gm in SHAPES:
            d.ecamd_tune(b"tiles_per_slot", tps)
            d.ecamd_tune(b"grid_mult", gm)
            for op in OPS:
                res.setdefault((tps, gm, op), []).append(timed(lambda: run(op), st))
    for (tps, gm, op), ts in res.items():
        ms = statistics.median(ts)
        print(json.dumps({"tiles_per_slot": tps, "grid_mult": gm, "op": op, "ms": round(ms, 4),
                          "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
    d.ecamd_tune(b"tiles_per_slot", 0)
    d.ecamd_tune(b"grid_mult", 0)


if __name__ == "__main__":
    main()
