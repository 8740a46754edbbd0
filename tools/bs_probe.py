#!/usr/bin/env python3
"""Bitsliced C5 encode (libecamd_probe.so, tools/gen_bitslice.py) against the product kernel:
bit-exact check of the parity and per-launch times on the same box, interleaved."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 20, 8, 4 << 20, 32


def main(reps=8):
    p = _lib.probe()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    D.rs_encode(K, M, lay, stream=st)
    st.synchronize()
    want = lay.buf.download(lay.stripe_stride * 2)
    algo = S * (K + M) * F
    for wpc in (2, 4):
        # clear the parity of stripes 0-1, run the bitsliced encode, compare
        zero = want.copy()
        zero[K * F:(K + M) * F] = 0
        zero[lay.stripe_stride + K * F:lay.stripe_stride + (K + M) * F] = 0
        lay.buf.upload(zero)
        _lib.check(p.ecamd_probe_bs_c5_encode(lay.buf.ptr, lay.stripe_stride, lay.frag_stride, F, S, wpc,
                                              st.handle), "bs")
        st.synchronize()
        got = lay.buf.download(lay.stripe_stride * 2)
        exact = bool((got == want).all())
        res = {"wgs_per_cu": wpc, "exact": exact}
        for name, fn in (("bitslice", lambda: p.ecamd_probe_bs_c5_encode(lay.buf.ptr, lay.stripe_stride,
                                                                          lay.frag_stride, F, S, wpc, st.handle)),
                         ("product", lambda: D.rs_encode(K, M, lay, stream=st))):
            ts = []
            for _ in range(3):
                fn()
                a, b = D.Event(), D.Event()
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                st.synchronize()
                ts.append(a.elapsed_ms(b) / reps)
            ms = min(ts)
            res[f"{name}_ms"] = round(ms, 4)
            res[f"{name}_TBps"] = round(algo / ms / 1e9, 3)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
