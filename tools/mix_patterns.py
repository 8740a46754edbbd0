#!/usr/bin/env python3
"""Is the rebuild-rate spread across erasure patterns (tools/c5_patterns.py) a memory-system effect?
mix_probe_kernel streams exactly the reads and writes of each C5 rebuild -- the 20 surviving
fragments read, the 8 lost ones written, per 4 MiB tile row of 32 stripes -- with no compute
(ecamd_probe_mix3, best cache policy / geometry of tools/mix_sweep.py), beside the bitsliced
decode of the same pattern.  Interleaved rounds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from c5_patterns import PATTERNS, K, M, F, S  # noqa: E402


def main(rounds=2, reps=20, warm=10):
    d, p = _lib.dev(), _lib.probe()
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    d.ecamd_tune(b"bitslice", 2)
    D.rs_encode(K, M, lay, stream=st)
    algo = S * (K + M) * F
    a, b = D.Event(), D.Event()

    def timed(fn):
        for _ in range(warm):
            fn()
        a.record(st)
        for _ in range(reps):
            fn()
        b.record(st)
        st.synchronize()
        return a.elapsed_ms(b) / reps

    for rnd in range(rounds):
        for name, lost in PATTERNS.items():
            surv = [f for f in range(K + M) if f not in lost][:K]
            frag = _lib.ints(surv + sorted(lost))
            probe_ms = timed(lambda: _lib.check(p.ecamd_probe_mix3(2, 2, 2, 512, 2, 0, 0, lay.buf.ptr, F, K, M, S,
                                                                   frag, st.handle), "mix3"))
            dec_ms = timed(lambda: D.rs_decode(K, M, lost, lay, stream=st))
            print(json.dumps({"round": rnd, "pattern": name, "probe_frac": round(algo / (probe_ms * 1e-3) / 8e12, 4),
                              "decode_frac": round(algo / (dec_ms * 1e-3) / 8e12, 4)}), flush=True)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
