#!/usr/bin/env python3
"""Grid oversubscription A/B of the stream kernel on one GPU (development tool): `grid_mult`
workgroups per resident slot let the hardware dispatcher balance the end of the launch, at the
price of one LDS table load per extra workgroup.  Interleaved rounds, median, C2 / C3 / C5."""
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

CFGS = {"c3": (10, 4, 1 << 20, 256, [0, 1, 2, 3]),
        "c2": (4, 2, 64 << 10, 4096, [0, 1]),
        "c5": (20, 8, 4 << 20, 32, list(range(8)))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="c3,c5,c2")
    ap.add_argument("--mults", default="1,2,4,8")
    ap.add_argument("--rounds", type=int, default=9)
    args = ap.parse_args()
    d = _lib.dev()
    st = D.Stream()
    a, b = D.Event(), D.Event()
    for cfg in args.cfg.split(","):
        k, m, F, S, miss = CFGS[cfg]
        lay = D.Layout.alloc(k + m, F, S)
        lay.fill_splitmix(nfrags=k, stream=st)
        algo = S * (k + m) * F
        times = {}
        for _ in range(args.rounds):
            for gm in (int(x) for x in args.mults.split(",")):
                d.ecamd_tune(b"grid_mult", gm)
                for op in ("enc", "dec"):
                    def fn():
                        if op == "enc":
                            D.rs_encode(k, m, lay, stream=st)
                        else:
                            D.rs_decode(k, m, miss, lay, stream=st)
                    fn()
                    a.record(st)
                    for _ in range(3):
                        fn()
                    b.record(st)
                    times.setdefault((op, gm), []).append(a.elapsed_ms(b) / 3)
        d.ecamd_tune(b"grid_mult", 0)
        for (op, gm), ts in sorted(times.items()):
            med = statistics.median(ts)
            print(json.dumps({"cfg": cfg, "op": op, "grid_mult": gm, "ms": round(med, 4),
                              "TBps": round(algo / med / 1e9, 3)}), flush=True)
        lay.buf.free()


if __name__ == "__main__":
    main()
