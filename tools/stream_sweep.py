#!/usr/bin/env python3
"""A/B of the gf16 kernels on one GPU (development tool): the streaming kernel (buffer loads,
pipelined groups; chunks per lane, store policy, launch geometry) against the previous
gf16_apply_kernel, for encode and decode at C2 / C3 / C5.  Interleaved rounds in one process,
median reported; every variant's output is checked against the reference variant's first."""
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


# (stream, ch, pf, nib, order, hybrid)
VARIANTS = [(0, 1, 0, 0, 0, 0), (1, 1, 0, 0, 0, 1), (1, 1, 0, 0, 1, 1), (1, 1, 0, 0, 2, 1), (1, 1, 0, 0, 3, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="c3,c5,c2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--geoms", default="0x0")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "stream_sweep.jsonl"))
    args = ap.parse_args()
    d = _lib.dev()
    out = open(args.out, "w")
    geoms = [tuple(int(x) for x in g.split("x")) for g in args.geoms.split(",")]
    for cfg in args.cfg.split(","):
        k, m, F, S, miss = CFGS[cfg]
        lay = D.Layout.alloc(k + m, F, S)
        st = D.Stream()
        lay.fill_splitmix(nfrags=k, stream=st)
        algo = S * (k + m) * F

        def setk(stream, ch, pf, nib, order, hyb, threads, wgs):
            d.ecamd_tune(b"stream_order", order)
            d.ecamd_tune(b"stream_hybrid", hyb)
            d.ecamd_tune(b"stream", stream)
            d.ecamd_tune(b"stream_nib", nib)
            d.ecamd_tune(b"stream_ch", ch)
            d.ecamd_tune(b"stream_pf", pf)
            d.ecamd_tune(b"threads", threads)
            d.ecamd_tune(b"wgs_per_cu", wgs)

        variants = {}
        for (threads, wgs) in geoms:
            for (stream, ch, pf, nib, order, hyb) in VARIANTS:
                if stream == 0 and (threads, wgs) != (0, 0):
                    continue
                tag = f"{cfg}_{'old' if not stream else f'st_ch{ch}_pf{pf}_nib{nib}_o{order}_h{hyb}'}_t{threads}_w{wgs}"
                for op in ("enc", "dec"):
                    def fn(op=op, a=(stream, ch, pf, nib, order, hyb, threads, wgs)):
                        setk(*a)
                        if op == "enc":
                            D.rs_encode(k, m, lay, stream=st)
                        else:
                            D.rs_decode(k, m, miss, lay, stream=st)
                    variants[f"{op}_{tag}"] = fn
        # correctness: every variant reproduces the old kernel's encode and decode output
        setk(0, 1, 0, 0, 0, 0, 0, 0)
        D.rs_encode(k, m, lay, stream=st)
        st.synchronize()
        ref = lay.buf.download(lay.stripe_stride * min(S, 4))
        bad = []
        for name, fn in variants.items():
            lay.buf.zero()
            lay.fill_splitmix(nfrags=k, stream=st)
            if name.startswith("dec"):
                setk(0, 1, 0, 0, 0, 0, 0, 0)
                D.rs_encode(k, m, lay, stream=st)
            fn()
            st.synchronize()
            if not (lay.buf.download(lay.stripe_stride * min(S, 4)) == ref).all():
                bad.append(name)
        print(json.dumps({"cfg": cfg, "mismatch": bad}), flush=True)
        out.write(json.dumps({"cfg": cfg, "mismatch": bad}) + "\n")
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
        recs = []
        for n, ts in times.items():
            med = statistics.median(ts)
            recs.append({"variant": n, "ms": round(med, 4), "GBps": round(algo / med / 1e6, 1)})
        recs.sort(key=lambda r: -r["GBps"])
        for r in recs:
            out.write(json.dumps(r) + "\n")
            print(json.dumps(r), flush=True)
        lay.buf.free()
        setk(1, 1, 0, 0, 0, 1, 0, 0)


if __name__ == "__main__":
    main()
