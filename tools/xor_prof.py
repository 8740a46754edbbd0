#!/usr/bin/env python3
"""flat_xor_hd batch workload for rocprofv3 (tools/gpu_prof_xor.sh): ecamd_xor_encode and
ecamd_xor_decode of {0, 1} (hd 3) / {0, 1, 2} (hd 4) at C1's code (3,3,3) with 4 KiB fragments
and at (10,6,4) with 1 MiB fragments, fixed launch counts so the profile's per-launch averages are
steady-state: 2 warm-up launches then `reps` of each.  Prints one JSON line per shape with the
HIP-event per-launch times and the algorithmic bytes per launch ((k + outputs) fragments per
stripe), for comparison with the kernel trace."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import device as D  # noqa: E402

SHAPES = [  # k, m, hd, fragment bytes, stripes, decode erasures
    (3, 3, 3, 4096, 131072, [0, 1]),
    (10, 6, 4, 1 << 20, 256, [0, 1, 2]),
]


def main(reps=10):
    for k, m, hd, F, S, lost in SHAPES:
        lay = D.Layout.alloc(k + m, F, S)
        st = D.Stream()
        lay.fill_splitmix(nfrags=k, stream=st)
        res = {"code": [k, m, hd], "fragment_bytes": F, "stripes": S, "decode_missing": lost}
        for name, fn, outs in (("encode", lambda: D.xor_encode(k, m, hd, lay, stream=st), m),
                               ("decode", lambda: D.xor_decode(k, m, hd, lost, lay, stream=st),
                                None)):
            fn()
            fn()
            a, b = D.Event(), D.Event()
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            st.synchronize()
            ms = a.elapsed_ms(b) / reps
            res[f"{name}_ms"] = round(ms, 4)
            if outs is not None:
                algo = S * (k + outs) * F
                res[f"{name}_algorithmic_bytes"] = algo
                res[f"{name}_GBps"] = round(algo / ms / 1e6, 1)
        print(json.dumps(res), flush=True)
        lay.buf.free()


if __name__ == "__main__":
    main()
