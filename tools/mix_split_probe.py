#!/usr/bin/env python3
"""Is the HBM ceiling of the C3 access pattern itself higher when a pass is split into shorter
launches?  The codec-shaped streaming probe (ecamd_probe_mix3: 10 fragment reads + 4 writes per
tile, grid-stride order, 4 x 256 threads per CU, no table work) over 256 C3 stripes as 1 / 2 / 4
launches, beside the codec's encode at its default (2 launches) and forced to one launch; median
of interleaved rounds, TB/s of the 14 MiB per stripe."""
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


def main():
    d, p = _lib.dev(), _lib.probe()
    st = D.Stream()
    lay = D.Layout.alloc(K + M, F, S)
    lay.fill_splitmix(nfrags=K, stream=st)
    ss = lay.stripe_stride

    def mix(nl, lp=2, sp=2):
        per = S // nl

        def fn():
            for i in range(nl):
                _lib.check(p.ecamd_probe_mix3(lp, sp, 1, 256, 4, 0, 0, lay.buf.ptr + i * per * ss, F, K, M,
                                              per, None, st.handle), "mix3")
        return fn

    def enc(tps):
        def fn():
            d.ecamd_tune(b"tiles_per_slot", tps)
            D.rs_encode(K, M, lay, stream=st)
        return fn

    variants = {"mix_1launch": mix(1), "mix_2launch": mix(2), "mix_4launch": mix(4),
                "mix_1launch_l0s0": mix(1, 0, 0), "mix_2launch_l0s0": mix(2, 0, 0),
                "codec_enc_default": enc(0), "codec_enc_1launch": enc(1 << 20)}
    times = {}
    for _ in range(4):
        for name, fn in variants.items():
            fn()
            ev = [D.Event() for _ in range(11)]
            ev[0].record(st)
            for i in range(10):
                fn()
                ev[i + 1].record(st)
            st.synchronize()
            times.setdefault(name, []).append(statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(2, 10)))
    d.ecamd_tune(b"tiles_per_slot", 0)
    for name, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"variant": name, "ms": round(med, 4), "TBps": round(S * (K + M) * F / (med * 1e-3) / 1e12, 3),
                          "rounds": [round(t, 4) for t in ts]}), flush=True)
    lay.buf.free()


if __name__ == "__main__":
    main()
