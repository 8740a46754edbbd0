#!/usr/bin/env python3
"""C5 bitsliced launch-grid A/B (development tool): k=20 m=8, 4 MiB fragments, 32 stripes;
encode, rebuild of {0..7} and of the mixed {0,2,4,6,20,22,24,26}, under (bs_grid, bs_tiles_per_slot)
variants -- resident-slot grid-stride launches against one workgroup per tile -- interleaved
rounds after a clock-settling warm-up, median per launch, fraction of 8 TB/s of the algorithmic
(20 read + 8 written) fragments; every variant's outputs checked equal to the first's."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

VARIANTS = [(0, 16), (1, 0), (1, 16), (0, 8)]


def main(rounds=5, reps=10):
    d = _lib.dev()
    k, m, F = 20, 8, 4 << 20
    S = int(os.environ.get("C5_S", 32))
    lay = D.Layout.alloc(k + m, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=k, stream=st)
    d.ecamd_tune(b"bitslice", 2)
    ops = {"encode": lambda: D.rs_encode(k, m, lay, stream=st),
           "rebuild_0_7": lambda: D.rs_decode(k, m, list(range(8)), lay, stream=st),
           "rebuild_mixed": lambda: D.rs_decode(k, m, [0, 2, 4, 6, 20, 22, 24, 26], lay, stream=st)}
    for fn in ops.values():
        fn()
    st.synchronize()
    ref = None
    for g, t in VARIANTS:
        d.ecamd_tune(b"bs_grid", g)
        d.ecamd_tune(b"bs_tiles_per_slot", t)
        ops["encode"]()
        ops["rebuild_0_7"]()
        st.synchronize()
        got = lay.buf.download(lay.stripe_stride)
        if ref is None:
            ref = got
        assert bool((got == ref).all()), (g, t)
    for _ in range(40):  # settle the clocks on this kernel mix
        ops["encode"]()
    algo = S * (k + 8) * F
    times = {(n, v): [] for n in ops for v in VARIANTS}
    a, b = D.Event(), D.Event()
    for _ in range(rounds):
        for v in VARIANTS:
            d.ecamd_tune(b"bs_grid", v[0])
            d.ecamd_tune(b"bs_tiles_per_slot", v[1])
            for n, fn in ops.items():
                fn()
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                st.synchronize()
                times[(n, v)].append(a.elapsed_ms(b) / reps)
    for (n, v), ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"op": n, "stripes": S, "bs_grid": v[0], "bs_tiles_per_slot": v[1], "ms": round(med, 4),
                          "frac": round(algo / med / 1e6 / 8000, 4)}), flush=True)
    d.ecamd_tune(b"bs_grid", -1)
    d.ecamd_tune(b"bs_tiles_per_slot", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
