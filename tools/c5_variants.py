#!/usr/bin/env python3
"""C5 (k=20, m=8, 4 MiB fragments, 32 stripes) lookup-engine variants for rocprofv3 PMC passes
(tools/gpu_prof_c5.sh): the 8-output GF(2^16) pass of encode and of decode {0..7} under each
ecamd_tune setting, a fixed number of launches each, every variant checked bit-exact against the
default.  Prints one JSON line per variant with HIP-event per-launch times."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M = 20, 8
F = int(os.environ.get("C5_F", 4 << 20))
S = int(os.environ.get("C5_S", 32))
LOST = list(range(8))
DEFAULTS = {"stream_hybrid": 1, "stream_nib": 0, "stream_deep": 0, "stream_ch": 1, "stream_pf": 0,
            "bitslice": 0}
VARIANTS = {
    "bitslice": {"bitslice": 2},
    "hybrid": {},
    "byte": {"stream_hybrid": 0},
}
for extra in sys.argv[1:]:  # name=key:val,key:val
    name, kv = extra.split("=", 1)
    VARIANTS[name] = {k: int(v) for k, v in (p.split(":") for p in kv.split(","))}


def setv(d, v):
    for key, val in DEFAULTS.items():
        d.ecamd_tune(key.encode(), v.get(key, val))


def main(reps=8, rounds=3):
    d = _lib.dev()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    setv(d, {})
    D.rs_encode(K, M, lay, stream=st)
    st.synchronize()
    want = lay.buf.download(lay.stripe_stride * 2)
    algo = S * (K + M) * F
    for rnd, (name, v) in [(r, nv) for r in range(rounds) for nv in VARIANTS.items()]:
        setv(d, v)
        res = {"round": rnd, "variant": name, "knobs": v}
        for op, fn in (("encode", lambda: D.rs_encode(K, M, lay, stream=st)),
                       ("decode", lambda: D.rs_decode(K, M, LOST, lay, stream=st))):
            fn()
            st.synchronize()
            res[f"{op}_exact"] = bool((lay.buf.download(lay.stripe_stride * 2) == want).all())
            a, b = D.Event(), D.Event()
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            st.synchronize()
            ms = a.elapsed_ms(b) / reps
            res[f"{op}_ms"] = round(ms, 4)
            res[f"{op}_TBps"] = round(algo / ms / 1e9, 3)
        print(json.dumps(res), flush=True)
    setv(d, {})


if __name__ == "__main__":
    main()
