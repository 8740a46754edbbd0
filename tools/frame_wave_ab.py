#!/usr/bin/env python3
"""A/B of the one-wave bitsliced kernel on the framed copy-through paths (knob bs_wave_copy, round 4;
development tool): the framed encode without checksum (one launch: objects read, payloads and parity
written) and the decode-join of data {0,1,2,3} (rebuilt data and surviving data straight into the
objects), at the C3 shape (256 x 10 MiB objects, bs = 1 MiB) and Swift's 1 MiB segments (2560 x
1 MiB, bs = 104858: unaligned object chunks, a ragged last tile).  Outputs checked equal across the
variants first; interleaved rounds, median; fraction of 8 TB/s of the algorithmic bytes (objects read
+ payloads written for the encode; payloads read + objects written for the join)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

# (bs_wave_copy, bs_prefetch): round 4, later: the next input's chunks loaded before each network and
# before the current input's copy stores
VARIANTS = {"lds_tables_stream": (0, 0), "bitsliced_wave": (1, 0), "bitsliced_wave_pf2": (1, 2),
            "bitsliced_wave_pf4": (1, 4)}
# round 5 (`frame_wave_ab.py cap`): resident one-wave workgroups per CU of the copy-through form (knob
# bs_copy_per_cu; the plain maps run best at 7, profiles/r05_ab_cap2.log), defaults otherwise
KNOBSETS = {"cap": {"copy_cap0": {"bs_copy_per_cu": 0}, "copy_cap6": {"bs_copy_per_cu": 6},
                    "copy_cap7": {"bs_copy_per_cu": 7}, "copy_cap8": {"bs_copy_per_cu": 8}},
            "cap2": {"copy_cap6": {"bs_copy_per_cu": 6, "bs_copy_realign_per_cu": 0},
                     "copy_cap5": {"bs_copy_per_cu": 5, "bs_copy_realign_per_cu": 0},
                     "realign_cap7": {"bs_copy_per_cu": 6, "bs_copy_realign_per_cu": 7},
                     "realign_cap10": {"bs_copy_per_cu": 6, "bs_copy_realign_per_cu": 10}}}
if len(sys.argv) > 1:
    VARIANTS = KNOBSETS[sys.argv[1]]


def apply(d, v):
    if isinstance(v, dict):
        for key, val in v.items():
            d.ecamd_tune(key.encode(), val)
    else:
        d.ecamd_tune(b"bs_wave_copy", v[0])
        d.ecamd_tune(b"bs_prefetch", v[1])


def main(rounds=3, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m = 10, 4
    for tag, size, S in (("c3", 10 << 20, 256), ("swift_1MiB_segment", 1 << 20, 2560)):
        fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_NONE)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x7A, st.handle), "fill")
        out = D.DeviceBuffer(fb.obj_stride * S)
        bs = fb.blocksize
        ops = {"encode": (lambda: fb.encode(obj, stream=st), S * (size + (k + m) * bs)),
               "join_0123": (lambda: fb.decode([0, 1, 2, 3], out, stream=st), S * ((k + 4) * bs - 4 * bs + size))}
        ref = {}
        for vname, v in VARIANTS.items():
            apply(d, v)
            fb.encode(obj, stream=st)
            st.synchronize()
            frags = fb.fragments()
            fb.decode([0, 1, 2, 3], out, stream=st)
            st.synchronize()
            joined = out.download()
            if not ref:
                ref = {"f": frags, "j": joined}
            assert (frags == ref["f"]).all() and (joined == ref["j"]).all(), (tag, vname)
        del ref
        times = {}
        for _ in range(20):
            ops["encode"][0]()
        a, b = D.Event(), D.Event()
        for _ in range(rounds):
            for vname, v in VARIANTS.items():
                apply(d, v)
                for op, (fn, _) in ops.items():
                    fn()
                    a.record(st)
                    for _ in range(reps):
                        fn()
                    b.record(st)
                    st.synchronize()
                    times.setdefault((vname, op), []).append(a.elapsed_ms(b) / reps)
        for (vname, op), ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"shape": tag, "variant": vname, "op": op, "ms": round(ms, 4),
                              "frac": round(ops[op][1] / (ms * 1e-3) / 8e12, 4)}), flush=True)
        obj.free()
        out.free()
        del fb
    d.ecamd_tune(b"bs_wave_copy", -1)
    d.ecamd_tune(b"bs_prefetch", -1)
    d.ecamd_tune(b"bs_copy_per_cu", -1)
    d.ecamd_tune(b"bs_copy_realign_per_cu", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
