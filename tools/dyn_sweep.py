#!/usr/bin/env python3
"""Static grid-stride tile order (grid_mult 1 / 2) against the dynamic one-wave-tile order
(knob stream_dyn, runs of stream_grab tiles from a per-stream counter) for the LDS-table stream
kernel: C3 (k=10 m=4, 1 MiB) at several batch sizes and C2 (k=4 m=2, 64 KiB), encode and decode,
interleaved rounds, median of steady launches (HIP events).  Every variant's outputs are checked
byte-equal to the static order's first.

Measured and rejected (profiles/r02_dyn_sweep_1ctr.log: one counter; r02_dyn_sweep_8ctr.log: one
counter per XCD): the dynamic order ran 0.52-0.83x the static one at C3 / C2 and its knobs were
removed from libecamd again; against the current library this script times the static variants
only (ecamd_tune refuses the unknown keys)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

SHAPES = {"c3": (10, 4, 1 << 20, [0, 1, 2, 3]), "c2": (4, 2, 64 << 10, [0, 1])}
VARIANTS = [("static_gm1", 0, 1, 0), ("static_gm2", 0, 2, 0), ("dyn_g2", 1, 0, 2),
            ("dyn_g4", 1, 0, 4), ("dyn_g8", 1, 0, 8), ("dyn_g16", 1, 0, 16)]


def set_variant(d, dyn, gm, grab):
    d.ecamd_tune(b"stream_dyn", dyn)
    d.ecamd_tune(b"grid_mult", gm)
    d.ecamd_tune(b"stream_grab", grab)


def timed(fn, st, n=20, skip=5):
    ev = [D.Event() for _ in range(n + 1)]
    ev[0].record(st)
    for i in range(n):
        fn()
        ev[i + 1].record(st)
    st.synchronize()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n))


def main():
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 0)
    cases = [("c3", 128), ("c3", 256), ("c3", 512), ("c3", 1024), ("c2", 4096)]
    if len(sys.argv) > 1:
        cases = [(c.split(":")[0], int(c.split(":")[1])) for c in sys.argv[1:]]
    st = D.Stream()
    for cfg, S in cases:
        k, m, F, lost = SHAPES[cfg]
        lay = D.Layout.alloc(k + m, F, S)
        lay.fill_splitmix(nfrags=k, stream=st)
        set_variant(d, 0, 2, 0)
        D.rs_encode(k, m, lay, stream=st)
        st.synchronize()
        ref = lay.download_stripes()
        if S * (k + m) * F <= (4 << 30):  # exactness: outputs cleared before every launch
            enc_in = ref.copy()
            enc_in[:, k:] = 0
            dec_in = ref.copy()
            dec_in[:, lost] = 0
            for name, dyn, gm, grab in VARIANTS:
                set_variant(d, dyn, gm, grab)
                for rep in range(2):  # the second launch reuses the stream's counter
                    for src, fn in ((enc_in, lambda: D.rs_encode(k, m, lay, stream=st)),
                                    (dec_in, lambda: D.rs_decode(k, m, lost, lay, stream=st))):
                        lay.upload_stripes(src)
                        fn()
                        st.synchronize()
                        if not (lay.download_stripes() == ref).all():
                            print(json.dumps({"cfg": cfg, "S": S, "variant": name, "rep": rep,
                                              "EXACT": False}), flush=True)
                            sys.exit(1)
            print(json.dumps({"cfg": cfg, "S": S, "exact": True}), flush=True)
        algo = S * (k + m) * F
        res = {}
        for rnd in range(3):
            for name, dyn, gm, grab in VARIANTS:
                set_variant(d, dyn, gm, grab)
                for op, fn in (("enc", lambda: D.rs_encode(k, m, lay, stream=st)),
                               ("dec", lambda: D.rs_decode(k, m, lost, lay, stream=st))):
                    res.setdefault((name, op), []).append(timed(fn, st))
        for (name, op), ms in res.items():
            med = statistics.median(ms)
            print(json.dumps({"cfg": cfg, "S": S, "variant": name, "op": op, "ms": round(med, 4),
                              "TBps": round(algo / (med * 1e-3) / 1e12, 3),
                              "rounds": [round(x, 4) for x in ms]}), flush=True)
        lay.buf.free()
    set_variant(d, 0, 0, 0)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
