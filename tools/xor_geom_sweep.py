#!/usr/bin/env python3
"""Flat-XOR launch geometry sweep (development tool): xor_wgs (256-thread workgroups per CU) x
xor_tiles_per_slot over the flat_xor_hd encode / decode shapes, interleaved rounds in one process,
median per variant; every variant's output checked equal to the first's."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

SHAPES = [  # k, m, hd, fragment bytes, stripes, decode erasures
    (10, 6, 4, 1 << 20, 256, [0, 1, 2]),
    (10, 5, 3, 1 << 20, 256, [0, 1]),
    (3, 3, 3, 4096, 131072, [0, 1]),
    (3, 3, 3, 1 << 20, 1024, [0, 1]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--wgs", default="2,3,4")
    ap.add_argument("--slots", default="64,32,0")
    ap.add_argument("--grid", default="0", help="xor_grid values (1: one workgroup per tile)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "xor_geom_sweep.jsonl"))
    args = ap.parse_args()
    d = _lib.dev()
    out = open(args.out, "w")
    for k, m, hd, F, S, lost in SHAPES:
        lay = D.Layout.alloc(k + m, F, S)
        st = D.Stream()
        lay.fill_splitmix(nfrags=k, stream=st)
        for op in ("encode", "decode"):
            if op == "encode":
                fn0 = lambda: D.xor_encode(k, m, hd, lay, stream=st)  # noqa: E731
                algo = S * (k + m) * F
            else:
                fn0 = lambda: D.xor_decode(k, m, hd, lost, lay, stream=st)  # noqa: E731
                algo = None
            variants = {}
            for gr in [int(x) for x in args.grid.split(",")]:
                for w in [int(x) for x in args.wgs.split(",")]:
                    for t in [int(x) for x in args.slots.split(",")]:
                        def fn(w=w, t=t, gr=gr):
                            d.ecamd_tune(b"xor_grid", gr)
                            d.ecamd_tune(b"xor_wgs", w)
                            d.ecamd_tune(b"xor_tiles_per_slot", t)
                            fn0()
                        variants[f"g{gr}_w{w}_t{t}"] = fn
            ref = None
            for n, fn in variants.items():
                fn()
                st.synchronize()
                got = lay.buf.download(lay.stripe_stride * 2)
                if ref is None:
                    ref = got
                assert bool((got == ref).all()), n
            a, b = D.Event(), D.Event()
            times = {n: [] for n in variants}
            for _ in range(args.rounds):
                for n, fn in variants.items():
                    fn()
                    a.record(st)
                    for _ in range(4):
                        fn()
                    b.record(st)
                    st.synchronize()
                    times[n].append(a.elapsed_ms(b) / 4)
            for n, ts in times.items():
                med = statistics.median(ts)
                r = {"shape": [k, m, hd, F, S], "op": op, "variant": n, "ms": round(med, 4),
                     "min_ms": round(min(ts), 4)}
                if algo:
                    r["GBps"] = round(algo / med / 1e6, 1)
                    r["frac"] = round(algo / med / 1e6 / 8000, 4)
                out.write(json.dumps(r) + "\n")
                print(json.dumps(r), flush=True)
        lay.buf.free()
    d.ecamd_tune(b"xor_wgs", 0)
    d.ecamd_tune(b"xor_grid", 1)
    d.ecamd_tune(b"xor_tiles_per_slot", -1)


if __name__ == "__main__":
    main()
