#!/usr/bin/env python3
"""C5 workload for rocprofv3 (tools/gpu_prof_c5.sh): k=20 m=8, 4 MiB fragments, 32 stripes in HBM.
With the bitsliced kernels (knob bitslice = 2: compile on first use, then always taken), in this
order: 25 untimed warm-up encodes, 30 encodes, 30 rebuilds of data {0..7}, 30 rebuilds of the
mixed pattern {0,2,4,6,20,22,24,26}; then the same 115 launches on the LDS-table kernels
(bitslice = 0).  Each run of 30 is one kernel (ecamd_bs_kernel / gf16_hybrid_kernel<5>) in
dispatch order, so the summary takes launches 10..29 of each run as the steady state (the clock
settles over the first ~20 launches of a VALU-dense kernel): ecamd_bs_kernel dispatches 38, 68, 98
(after 3 compile-time launches), gf16_hybrid_kernel 36, 66, 96 (after 1).  Prints the HIP-event rate of each steady window too.
C5_MODES="2:0,2:4,0:0" picks other (bitslice, bitslice_depth) sequences, e.g. for A/B runs;
C5_K / C5_M / C5_S other shapes (m = 8).
PROF_CFG=c3: the same sequence at C3 (k=10 m=4, 1 MiB, 256 stripes) with the decodes of data
{0,1,2,3} and of the mixed {0,5,10,13} -- every pass on the one-wave bitsliced kernel, then on the
LDS-table stream kernel (gf16_stream_kernel): the same dispatch indices (tools/gpu_prof_c3ops.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M = int(os.environ.get("C5_K", 20)), int(os.environ.get("C5_M", 8))  # other shapes: A/B only
F, S = 4 << 20, int(os.environ.get("C5_S", 32))
WARM = 25
PATTERNS = {"rebuild8_data": list(range(8)), "rebuild8_mixed": [0, 2, 4, 6, K, K + 2, K + 4, K + 6]}
if os.environ.get("PROF_CFG") == "c3":
    K, M, F, S = 10, 4, 1 << 20, 256
    PATTERNS = {"decode_0123": [0, 1, 2, 3], "decode_mixed": [0, 5, 10, 13]}


def main(n=30, skip=10):
    modes = [tuple(int(x) for x in m.split(":")) for m in os.environ.get("C5_MODES", "").split(",") if m]
    d = _lib.dev()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    d.ecamd_tune(b"bitslice", 0)
    D.rs_encode(K, M, lay, stream=st)
    # compile every bitsliced network before the profiled launches
    d.ecamd_tune(b"bitslice", 2)
    for _, depth in modes:
        d.ecamd_tune(b"bitslice_depth", depth)
        D.rs_encode(K, M, lay, stream=st)
        for pat in PATTERNS.values():
            D.rs_decode(K, M, pat, lay, stream=st)
    D.rs_encode(K, M, lay, stream=st)
    for pat in PATTERNS.values():
        D.rs_decode(K, M, pat, lay, stream=st)
    st.synchronize()
    assert d.ecamd_bitslice_wait() == 0
    algo = S * (K + M) * F
    for mode, depth in modes or [(2, None), (0, None)]:
        d.ecamd_tune(b"bitslice", mode)
        if depth is not None:
            d.ecamd_tune(b"bitslice_depth", depth)
        for _ in range(WARM):
            D.rs_encode(K, M, lay, stream=st)
        ops = [("encode", lambda: D.rs_encode(K, M, lay, stream=st))]
        ops += [(name, (lambda p: lambda: D.rs_decode(K, M, p, lay, stream=st))(p)) for name, p in PATTERNS.items()]
        for name, fn in ops:
            ev = [D.Event() for _ in range(n + 1)]
            ev[0].record(st)
            for i in range(n):
                fn()
                ev[i + 1].record(st)
            st.synchronize()
            ms = [ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n)]
            avg = sum(ms) / len(ms)
            print(json.dumps({"kernel": "bitslice" if mode else "lds", "depth": depth, "op": name,
                              "steady_ms": round(avg, 4), "TBps": round(algo / avg / 1e9, 3),
                              "frac": round(algo / avg / 1e9 / 8, 4)}), flush=True)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
