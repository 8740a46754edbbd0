#!/usr/bin/env python3
"""Fragment / stripe pitch A/B at C3 on one GPU (development tool): does padding the fragment stride
(so the k + m fragments of a stripe do not sit exactly 1 MiB apart) change the HBM rate of the
stream kernel?  Interleaved rounds, median; each layout's encode output is checked against the
unpadded layout's."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pads", default="0,256,1024,4096,65536,4352")
    ap.add_argument("--spads", default="0")
    ap.add_argument("--offs", default="0", help="base offsets (e.g. 80: payloads behind 80-byte headers)")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--cfg", default="10,4,1048576,256")
    args = ap.parse_args()
    k, m, F, S = (int(x) for x in args.cfg.split(","))
    st = D.Stream()
    lays = {}
    class Shifted:  # a view of a device buffer starting `off` bytes in
        def __init__(self, buf, off):
            self.buf, self.ptr = buf, buf.ptr + off

        def download(self, n):
            return self.buf.download(n + (self.ptr - self.buf.ptr))[self.ptr - self.buf.ptr:]

    for pad in (int(p) for p in args.pads.split(",")):
        for spad in (int(p) for p in args.spads.split(",")):
            for off in (int(p) for p in args.offs.split(",")):
                fs = F + pad
                ss = fs * (k + m) + spad
                buf = D.DeviceBuffer(ss * S + 256)
                lay = D.Layout(Shifted(buf, off), k + m, F, S, fs, ss)
                lay.fill_splitmix(nfrags=k, stream=st)
                lays[(pad, spad, off)] = lay
    ref = None
    for key, lay in lays.items():
        D.rs_encode(k, m, lay, stream=st)
        st.synchronize()
        got = lay.download_stripes()[:4]
        if ref is None:
            ref = got
        assert (got == ref).all(), key
    algo = S * (k + m) * F
    a, b = D.Event(), D.Event()
    times = {}
    for _ in range(args.rounds):
        for key, lay in lays.items():
            for op in ("enc", "dec"):
                def fn():
                    if op == "enc":
                        D.rs_encode(k, m, lay, stream=st)
                    else:
                        D.rs_decode(k, m, list(range(m)), lay, stream=st)
                fn()
                a.record(st)
                for _ in range(3):
                    fn()
                b.record(st)
                times.setdefault((op,) + key, []).append(a.elapsed_ms(b) / 3)
    for key, ts in sorted(times.items(), key=lambda kv: statistics.median(kv[1])):
        med = statistics.median(ts)
        print(json.dumps({"op": key[0], "frag_pad": key[1], "stripe_pad": key[2], "base_off": key[3],
                          "ms": round(med, 4),
                          "TBps": round(algo / med / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
