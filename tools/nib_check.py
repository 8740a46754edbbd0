#!/usr/bin/env python3
"""Bit-exactness probe of the nibble-table gf16 path vs the byte-table path, per op and shape,
reporting the first mismatching (stripe, fragment, offset)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def run(k, m, F, S, op, miss, nib):
    d = _lib.dev()
    d.ecamd_tune(b"nib", nib)
    lay = D.Layout.alloc(k + m, F, S)
    lay.fill_splitmix()
    if op == "enc":
        D.rs_encode(k, m, lay)
    else:
        D.rs_decode(k, m, miss, lay)
    D.synchronize()
    d.ecamd_tune(b"nib", 0)
    return lay.download_stripes()


def main():
    for (k, m, F, S, miss) in [(4, 2, 4096, 4, [0, 1]), (10, 4, 4096, 4, [0, 1, 2, 3]),
                               (6, 3, 4096, 2, [0]), (5, 4, 4096, 2, [0]), (4, 4, 4096, 2, [0]),
                               (3, 3, 4096, 2, [0]), (20, 8, 4096, 2, list(range(8))),
                               (10, 4, 1 << 20, 256, [0, 1, 2, 3]), (10, 4, 1 << 20, 8, [0, 1, 2, 3]),
                               (10, 4, 65536, 64, [0, 1, 2, 3])]:
        for op in ("enc", "dec"):
            a = run(k, m, F, S, op, miss, 0)
            b = run(k, m, F, S, op, miss, 1)
            bad = np.argwhere(a != b)
            rec = {"k": k, "m": m, "op": op, "equal": bool(len(bad) == 0)}
            if len(bad):
                s, f, o = bad[0]
                rec.update(first=[int(s), int(f), int(o)], nbad=int(len(bad)),
                           frags=sorted(set(int(x) for x in bad[:, 1])))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
