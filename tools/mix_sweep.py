#!/usr/bin/env python3
"""Cache-policy / geometry sweep of the codec's HBM access pattern (development tool).

mix_probe_kernel streams the gf16 kernel's exact pattern -- K fragment reads, R fragment writes per
tile of the strided [S][K+R][F] layout -- without the table work, with the buffer-load and store
cache policy as a parameter (gfx950 cpol: 1 sc0, 2 nt, 16 sc1).  Interleaved rounds in one process,
median reported, the codec encode on the same layout timed alongside.
"""
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

POLICIES = [(0, 0), (0, 2), (0, 16), (0, 18), (0, 1), (2, 0), (2, 2), (2, 16), (2, 18), (2, 1),
            (1, 0), (1, 2), (16, 2), (18, 2), (3, 2), (18, 18)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--F", type=int, default=1 << 20)
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--geoms", default="256x4,512x2,1024x1")
    ap.add_argument("--policies", default="")
    ap.add_argument("--layouts", default="0x0", help="order x wave_contig pairs")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "mix_sweep.jsonl"))
    args = ap.parse_args()
    k, m, F, S = args.k, args.m, args.F, args.S
    C = _lib.C
    d = _lib.dev()
    p = _lib.probe()
    lay = D.Layout.alloc(k + m, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=k, stream=st)
    algo = S * (k + m) * F

    variants = {}
    geoms = [tuple(int(x) for x in g.split("x")) for g in args.geoms.split(",")]
    pols = POLICIES if not args.policies else [tuple(int(x) for x in p.split("/"))
                                               for p in args.policies.split(",")]
    lays = [tuple(int(x) for x in p.split("x")) for p in args.layouts.split(",")]
    for lp, sp in pols:
        for ch in (1, 2):
            for threads, wgs in geoms:
                for order, wc in lays:
                    def fn(lp=lp, sp=sp, ch=ch, threads=threads, wgs=wgs, order=order, wc=wc):
                        _lib.check(p.ecamd_probe_mix2(lp, sp, ch, threads, wgs, order, wc,
                                                            lay.buf.ptr, F, k, m, S, st.handle),
                                   "mix probe")
                    variants[f"mix_l{lp}_s{sp}_ch{ch}_t{threads}_w{wgs}_o{order}_wc{wc}"] = fn

    def enc():
        D.rs_encode(k, m, lay, stream=st)
    variants["codec_encode"] = enc

    a, b = D.Event(), D.Event()
    times = {n: [] for n in variants}
    for _ in range(args.rounds):
        for n, fn in variants.items():
            fn()
            a.record(st)
            for _ in range(3):
                fn()
            b.record(st)
            times[n].append(a.elapsed_ms(b) / 3)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    recs = []
    for n, ts in times.items():
        med = statistics.median(ts)
        recs.append({"variant": n, "ms": round(med, 4), "GBps": round(algo / med / 1e6, 1)})
    recs.sort(key=lambda r: -r["GBps"])
    with open(args.out, "w") as f:
        for r in recs:
            f.write(json.dumps(r) + "\n")
            print(json.dumps(r))


if __name__ == "__main__":
    main()
