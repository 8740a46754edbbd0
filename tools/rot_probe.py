#!/usr/bin/env python3
"""Does the order in which a tile visits its fragments matter to HBM? (development tool, round 3)
The codec-shaped streaming probe (ecamd_probe_mix3, no table work) on the C3 (10+4, 1 MiB, 256
stripes), C5 (20+8, 4 MiB, 32 stripes) and C3-mixed-decode shapes, every tile reading its fragments
in slot order (order 0, the codec's) against rotated by the tile index (order 2: neighbouring tiles
start on different fragments), grid-stride over 4 or 8 resident workgroups per CU and one workgroup
per tile, 2 launches per pass.  Median of interleaved rounds, fraction of 8 TB/s.
`rot_probe.py slots`: the C3 pattern with different sets of written slots (order 0)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

def slots(writes, n=14):
    """frag list: reads = the other slots in order, writes = `writes`."""
    return [i for i in range(n) if i not in writes] + list(writes)


SHAPES = [("c3", 10, 4, 1 << 20, 256, None), ("c5", 20, 8, 4 << 20, 32, None),
          ("c3_mixed", 10, 4, 1 << 20, 256, slots([0, 5, 10, 13]))]
GEOMS = [("stride_x4", 256, 4), ("stride_x8", 256, 8), ("tile", 256, 0)]
ORDERS = (0, 2)
if len(sys.argv) > 1 and sys.argv[1] == "slots":  # which slots of a C3 stripe are written
    SHAPES = [(f"c3_writes_{'_'.join(map(str, w))}", 10, 4, 1 << 20, 256, slots(w))
              for w in ([10, 11, 12, 13], [0, 1, 2, 3], [0, 5, 10, 13], [2, 5, 8, 11], [3, 6, 9, 12],
                        [1, 4, 7, 10], [0, 13, 6, 7])]
    GEOMS = [("stride_x8", 256, 8), ("tile", 256, 0)]
    ORDERS = (0,)
if len(sys.argv) > 1 and sys.argv[1] == "geom5":  # tile widths, C5 (20 + 8, 4 MiB) data and mixed rebuilds
    SHAPES = [("c5_rebuild_0_7", 20, 8, 4 << 20, 32, slots(list(range(8)), 28)),
              ("c5_rebuild_mixed", 20, 8, 4 << 20, 32, slots([0, 2, 4, 6, 20, 22, 24, 26], 28))]
    GEOMS = [("tile16k_4wave_ch4", 256, 0, 4), ("tile4k_1wave_ch4", 64, 0, 4), ("tile8k_2wave_ch4", 128, 0, 4),
             ("tile1k_1wave", 64, 0, 1), ("tile4k", 256, 0, 1)]
    ORDERS = (0,)
if len(sys.argv) > 1 and sys.argv[1] == "geom":  # tile widths, C3 contiguous and mixed writes
    SHAPES = [("c3", 10, 4, 1 << 20, 256, None), ("c3_mixed", 10, 4, 1 << 20, 256, slots([0, 5, 10, 13]))]
    GEOMS = [("tile4k", 256, 0, 1), ("tile1k_1wave", 64, 0, 1), ("tile16k_4wave_ch4", 256, 0, 4),
             ("tile4k_1wave_ch4", 64, 0, 4), ("tile8k_2wave_ch4", 128, 0, 4), ("tile2k_1wave", 64, 0, 2),
             ("stride16k_4wave_ch4_x2", 256, 8, 4)]
    ORDERS = (0,)


def main(rounds=5, reps=10):
    p = _lib.probe()
    st = D.Stream()
    for name, K, R, F, S, frag in SHAPES:
        lay = D.Layout.alloc(K + R, F, S)
        lay.fill_splitmix(nfrags=K, stream=st)
        ss = lay.stripe_stride
        fl = _lib.ints(frag) if frag else None

        def mk(threads, wgs, order, ch=1, nl=2):
            per = S // nl
            w = wgs if wgs else 1 << 20

            def fn():
                for i in range(nl):
                    _lib.check(p.ecamd_probe_mix3(2, 2, ch, threads, w, order, 0, lay.buf.ptr + i * per * ss, F, K,
                                                  R, per, fl, st.handle), "mix3")
            return fn
        variants = {f"{g[0]}_order{o}": mk(g[1], g[2], o, *g[3:]) for g in GEOMS for o in ORDERS}
        for _ in range(40):
            next(iter(variants.values()))()
        times = {}
        for _ in range(rounds):
            for vn, fn in variants.items():
                fn()
                a, b = D.Event(), D.Event()
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                st.synchronize()
                times.setdefault(vn, []).append(a.elapsed_ms(b) / reps)
        algo = S * (K + R) * F
        for vn, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"shape": name, "variant": vn, "ms": round(med, 4),
                              "frac": round(algo / (med * 1e-3) / 8e12, 4)}), flush=True)
        lay.buf.free()


if __name__ == "__main__":
    main()
