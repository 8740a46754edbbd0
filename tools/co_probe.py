#!/usr/bin/env python3
"""Concurrency experiment: the LDS-table kernel (product encode) and the bitsliced VALU kernel
(probe) on two streams over disjoint stripe ranges of one C5 batch -- do the two engines (LDS
array vs VALU) add up on one CU?  Host wall time over `reps` back-to-back rounds."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

K, M, F, S = 20, 8, 4 << 20, 32


class View:
    def __init__(self, ptr):
        self.ptr = ptr


def main(reps=10):
    p = _lib.probe()
    lay = D.Layout.alloc(K + M, F, S)
    s1, s2 = D.Stream(), D.Stream()
    lay.fill_splitmix(nfrags=K, stream=s1)
    D.rs_encode(K, M, lay, stream=s1)
    s1.synchronize()
    want = lay.buf.download()
    algo = S * (K + M) * F

    def run(a, wpc=2):
        # stripes [0, a): LDS kernel on s1; [a, S): bitslice on s2
        if a > 0:
            sub = D.Layout(View(lay.buf.ptr), K + M, F, a, lay.frag_stride, lay.stripe_stride)
            D.rs_encode(K, M, sub, stream=s1)
        if a < S:
            _lib.check(p.ecamd_probe_bs_c5_encode(lay.buf.ptr + a * lay.stripe_stride, lay.stripe_stride,
                                                  lay.frag_stride, F, S - a, wpc, s2.handle), "bs")

    for a in (32, 0, 24, 22, 20, 18, 16):
        for wpc in ((2, 1) if 0 < a < S else (2,)):
            run(a, wpc)
            s1.synchronize(); s2.synchronize()
            ok = bool((lay.buf.download() == want).all())
            best = 1e9
            for _ in range(3):
                s1.synchronize(); s2.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    run(a, wpc)
                s1.synchronize(); s2.synchronize()
                best = min(best, (time.perf_counter() - t0) / reps)
            print(json.dumps({"lds_stripes": a, "bs_wgs_per_cu": wpc, "exact": ok, "ms": round(best * 1e3, 4),
                              "TBps": round(algo / best / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
