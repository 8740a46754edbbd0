#!/usr/bin/env python3
"""Rebuild traffic's maps in a COLD process, at the C3 shape (k=10 m=4, 1 MiB
fragments, 256 stripes in HBM), knob bitslice at its default (1: never waits for a compile):

  phase "reconstruct": liberasurecode_reconstruct_fragment's map for every destination d of (10, 4)
    with d lost (ecamd_rs_reconstruct, missing [d]): the bitsliced launches of its FIRST call (the
    launch counter) and the steady rate over `reps` more calls; algorithmic bytes (k + 1) x F per stripe;
  phase "multi": ecamd_rs_decode_multi with the 4 patterns of tools/multi_bench.py (64 stripes each,
    one launch per pattern) and, for reference, the strided decode of {0,1,2,3}; (k + 4) x F per stripe.

Run with an empty $ECAMD_JIT_CACHE so only lib/jit's shipped objects can serve.  One JSON line per
case with the HIP-event rate; under `rocprofv3 --kernel-trace` the dispatch order is: 1 + SETTLE
encodes, then per destination 1 + reps reconstructs, then 1 + reps decode_multi calls of 4 launches,
for each multi_streams setting (1, 2, 4), then 1 + reps strided decodes -- tools/rebuild_prof_trace.py turns the trace into the same table.

usage: python tools/rebuild_prof.py [reps]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 10, 4, 1 << 20, 256
SETTLE = 60
PATS = [[0, 1, 2, 3], [4, 5, 6, 7], [0, 5, 10, 13], [2, 3, 8, 9]]
MULTI_STREAMS = (1, 2, 4)


def main(reps=20):
    d = _lib.dev()
    cnt = d.ecamd_bitslice_launches
    cnt.restype = ctypes.c_longlong
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    for _ in range(1 + SETTLE):
        D.rs_encode(K, M, lay, stream=st)
    st.synchronize()
    a, b = D.Event(), D.Event()

    def run(name, fn, algo, extra=None):
        n0 = cnt()
        fn()  # the first call: which kernel served it
        st.synchronize()
        first_bs = cnt() - n0
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        st.synchronize()
        ms = a.elapsed_ms(b) / reps
        out = {"case": name, "first_call_bitsliced_launches": first_bs, "ms": round(ms, 4),
               "frac": round(algo / (ms * 1e-3) / 8e12, 4)}
        out.update(extra or {})
        print(json.dumps(out), flush=True)

    for dest in range(K + M):
        run(f"reconstruct_{dest}", lambda: D.rs_reconstruct(K, M, [dest], dest, lay, stream=st), S * (K + 1) * F,
            {"form": d.ecamd_rs_kernel_form(K, M, _lib.ints([dest, -1]), dest, 0, F)})
    per = [PATS[s * len(PATS) // S] for s in range(S)]  # 4 groups of 64 consecutive stripes
    per2 = [PATS[s % len(PATS)] for s in range(S)]  # the same groups interleaved through the batch
    for streams in MULTI_STREAMS:  # knob multi_streams: the 4 launches on 1 .. 4 streams
        d.ecamd_tune(b"multi_streams", streams)
        sfx = "" if streams == 1 else f"_streams{streams}"
        run("decode_multi_4patterns" + sfx, lambda: D.rs_decode_multi(K, M, per, lay, stream=st), S * (K + 4) * F)
        run("decode_multi_4patterns_interleaved" + sfx, lambda: D.rs_decode_multi(K, M, per2, lay, stream=st),
            S * (K + 4) * F)
    d.ecamd_tune(b"multi_streams", -1)
    run("decode_strided_0123", lambda: D.rs_decode(K, M, PATS[0], lay, stream=st), S * (K + 4) * F)
    lay.buf.free()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
