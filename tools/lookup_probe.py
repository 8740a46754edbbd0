#!/usr/bin/env python3
"""Lookup engines on one MI355X (development tool): random 16-byte table lookups per clock per CU
from LDS, from global memory through the vector L1, and half each; 16-entry (nibble-sized) tables from each
(ecamd_probe_lookup)."""
import ctypes as C
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
    for mode in range(6):
        for wgs in (2, 4, 8):
            ts = []
            for _ in range(5):
                _lib.check(p.ecamd_probe_lookup(mode, wgs, iters, tab.ptr, st.handle), "probe")
                a.record(st)
                p.ecamd_probe_lookup(mode, wgs, iters, tab.ptr, st.handle)
                b.record(st)
                ts.append(a.elapsed_ms(b))
            ms = statistics.median(ts)
            lookups = cus * wgs * 256 * iters * 4
            per_clk_cu = lookups / (ms * 1e-3) / 2.4e9 / cus
            print(json.dumps({"mode": names[mode], "wgs_per_cu": wgs, "ms": round(ms, 3),
                              "lookups_per_clk_per_cu": round(per_clk_cu, 2),
                              "bytes_per_clk_per_cu": round(per_clk_cu * 16, 1)}), flush=True)


if __name__ == "__main__":
    main()
