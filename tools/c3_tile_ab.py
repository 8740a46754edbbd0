#!/usr/bin/env python3
"""C3 on the LDS-table stream kernel in the one-wave-tile shape (round 3): the one-wave 1 KiB tile
copies at 0.86 of 8 TB/s and streams the codec's pattern at 0.76 (profiles/r03_geom_probe3.log),
but a one-wave workgroup must stage its own tables -- 40 KiB of byte tables at C3, 5 KiB of nibble
tables (knob stream_nib).  Variants (threads per workgroup, workgroups per tile run, nibble tables,
tiles per slot per launch): the default, one-wave 1 KiB tiles with nibble / byte tables, 4-wave
4 KiB tiles with nibble tables, and the default geometry on nibble tables.  Encode and decode of
{0,1,2,3} and {0,5,10,13}, interleaved rounds, median; bytes checked equal to the default's."""
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
OPS = {"encode": None, "decode_0123": [0, 1, 2, 3], "decode_mixed": [0, 5, 10, 13]}
if len(sys.argv) > 1 and sys.argv[1] == "c2":  # C2: k=4 m=2, 64 KiB x 4096 stripes (1 KiB nibble image)
    K, M, F, S = 4, 2, 64 << 10, 4096
    OPS = {"encode": None, "decode_01": [0, 1], "decode_mixed": [0, 4]}
# label: (threads, stream_chunk, stream_nib, tiles_per_slot)
VARIANTS = {"default": (0, -1, 0, 0), "wave1k_nib": (64, 1, 1, 128), "wave1k_bytes": (64, 1, 0, 128),
            "wg4k_nib": (256, 1, 1, 32), "default_nib": (0, -1, 1, 0), "wave1k_nib_tps512": (64, 1, 1, 512)}
if len(sys.argv) > 2 and sys.argv[2] == "chunk":  # one workgroup per 1 / 2 / 4 tiles only, more rounds
    VARIANTS = {"default": (0, -1, 0, 0), "chunk1": (0, 1, 0, 0), "chunk2": (0, 2, 0, 0), "chunk4": (0, 4, 0, 0)}
elif len(sys.argv) > 1 and sys.argv[1] == "c2":
    VARIANTS = {"default": (0, -1, 0, 0), "wave1k_nib": (64, 1, 1, 0), "wave1k_bytes": (64, 1, 0, 0),
                "wave2k_bytes": (128, 1, 0, 0), "wg4k_bytes": (256, 1, 0, 0), "default_nib": (0, -1, 1, 0)}


def set_variant(d, v):
    t, chunk, nib, tps = v
    for key, val in ((b"threads", t), (b"stream_chunk", chunk), (b"stream_nib", nib), (b"tiles_per_slot", tps)):
        _lib.check(d.ecamd_tune(key, val), "tune")


def timed(fn, st, n=14, skip=4):
    ev = [D.Event() for _ in range(n + 1)]
    ev[0].record(st)
    for i in range(n):
        fn()
        ev[i + 1].record(st)
    st.synchronize()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n))


def main(rounds=5 if len(sys.argv) > 2 else 3):
    d = _lib.dev()
    st = D.Stream()
    lay = D.Layout.alloc(K + M, F, S)
    lay.fill_splitmix(nfrags=K, stream=st)

    def run(op):
        if OPS[op] is None:
            D.rs_encode(K, M, lay, stream=st)
        else:
            D.rs_decode(K, M, OPS[op], lay, stream=st)
    ref = {}
    for name, v in VARIANTS.items():
        set_variant(d, v)
        for op in OPS:
            run(op)
            st.synchronize()
            got = lay.download_stripes()
            if op not in ref:
                ref[op] = got
            assert (got == ref[op]).all(), (name, op)
    del ref
    set_variant(d, VARIANTS["default"])
    for _ in range(60):
        run("encode")
    algo = S * (K + M) * F
    res = {}
    for _ in range(rounds):
        for name, v in VARIANTS.items():
            set_variant(d, v)
            for op in OPS:
                res.setdefault((name, op), []).append(timed(lambda: run(op), st))
    for (name, op), ts in res.items():
        ms = statistics.median(ts)
        print(json.dumps({"shape": f"k{K}m{M}", "variant": name, "op": op, "ms": round(ms, 4),
                          "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
    set_variant(d, (0, -1, 0, 0))


if __name__ == "__main__":
    main()
