#!/usr/bin/env python3
"""Flat-XOR tile width (round 3): xor_stream_kernel with one workgroup per tile of 256 / 128 / 64
threads (4 / 2 / 1 KiB of every fragment; knob xor_threads) -- the codec-shaped probe ran the C3
pattern at 0.73 / 0.76 with 4 KiB / 1 KiB one-wave tiles (profiles/r03_geom_probe3.log).  Encode and
decode of (10,6,4) and (10,5,3) at 1 MiB x 256 stripes and (3,3,3) at 4 KiB x 131072 stripes,
interleaved rounds, median; every variant's bytes checked equal to the default's.
Round 5: `xor_threads_ab.py KNOB v1,v2,...` A/Bs any knob the same way (e.g. xor_per_cu 0,7,8,12:
resident workgroups per CU)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

SHAPES = [(10, 6, 4, 1 << 20, 256, [0, 1, 2]), (10, 5, 3, 1 << 20, 256, [0, 1]), (3, 3, 3, 4096, 131072, [0, 1]),
          (3, 3, 3, 1 << 20, 1024, [0, 1]), (10, 6, 4, 64 << 10, 4096, [0, 1, 2]), (10, 6, 4, 16 << 10, 16384, [0, 1, 2])]
KNOB = sys.argv[1].encode() if len(sys.argv) > 2 else b"xor_threads"
THREADS = ([int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2
           else [256, 128, 64, 0])  # xor_threads 0: the library default (by fragment size)


def timed(fn, st, n=14, skip=4):
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
    for k, m, hd, F, S, lost in SHAPES:
        lay = D.Layout.alloc(k + m, F, S)
        lay.fill_splitmix(nfrags=k, stream=st)
        ops = {"encode": (lambda: D.xor_encode(k, m, hd, lay, stream=st), S * (k + m) * F),
               "decode": (lambda: D.xor_decode(k, m, hd, lost, lay, stream=st), None)}
        refs = {}
        for t in THREADS:
            d.ecamd_tune(KNOB, t)
            for op, (fn, _) in ops.items():
                fn()
                st.synchronize()
                got = lay.download_stripes()
                if op not in refs:
                    refs[op] = got
                assert (got == refs[op]).all(), (k, m, op, t)
        del refs
        for _ in range(30):
            ops["encode"][0]()
        res = {}
        for _ in range(rounds):
            for t in THREADS:
                d.ecamd_tune(KNOB, t)
                for op, (fn, _) in ops.items():
                    res.setdefault((t, op), []).append(timed(fn, st))
        for (t, op), ts in res.items():
            ms = statistics.median(ts)
            algo = ops[op][1]
            print(json.dumps({"code": f"({k},{m},{hd})", "F": F, "stripes": S, "op": op,
                              KNOB.decode(): t, "ms": round(ms, 4),
                              "frac": round(algo / (ms * 1e-3) / 8e12, 4) if algo else None}), flush=True)
        lay.buf.free()
    d.ecamd_tune(KNOB, 0)


if __name__ == "__main__":
    main()
