#!/usr/bin/env python3
"""HBM ceilings on this MI355X: copy / read-only / write-only probes over 2 GiB, several
unroll depths and occupancies (interleaved rounds in one process, median reported)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main():
    d = _lib.dev()
    p = _lib.probe()
    half = 2 << 30
    buf = D.DeviceBuffer(2 * half)
    buf.zero()
    st = D.Stream()
    variants = [(kind, u, w) for kind in (0, 1, 2) for u in (1, 4, 8) for w in (2, 4, 8)]
    times = {v: [] for v in variants}
    a, b = D.Event(), D.Event()
    for _ in range(3):
        for v in variants:
            kind, u, w = v
            _lib.check(p.ecamd_probe_bw(kind, u, w, buf.ptr + half, buf.ptr, half, st.handle), "probe")
            a.record(st)
            for _ in range(3):
                p.ecamd_probe_bw(kind, u, w, buf.ptr + half, buf.ptr, half, st.handle)
            b.record(st)
            times[v].append(a.elapsed_ms(b) / 3)
    best = {}
    for (kind, u, w), ts in times.items():
        moved = half * (2 if kind == 0 else 1)
        gbs = moved / statistics.median(ts) / 1e6
        name = ["copy", "read", "write"][kind]
        print(json.dumps({"probe": name, "unroll": u, "wgs_per_cu": w, "GBps": round(gbs, 1)}))
        best[name] = max(best.get(name, 0), gbs)
    print(json.dumps({"best_GBps": {k: round(v, 1) for k, v in best.items()}}))


if __name__ == "__main__":
    main()
