#!/usr/bin/env python3
"""A/B of knob frame_tail_fork (round 4; development tool): the framed encode of objects that do not
fill the payloads -- Swift's 1 MiB segments (bs = 104858) and 10 MiB + 10 B objects, RS(10,4) and
flat XOR (10,6,4), checksum none and CRC32 -- with the payloads' rest past the whole tiles on a side
stream beside the launch over the whole tiles (2: always; 1: default, without checksum and a rest of 1-4 KiB)
or after it on the caller's stream (0).  Fragments
checked equal across the variants; interleaved rounds, median ms and fraction of 8 TB/s of the
algorithmic bytes (objects read + payloads written; payloads read + objects written for the RS decode-join
of data {0,1,2,3}, whose LDS-table rest forks the same way)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

CASES = [("rs_swift_1MiB_segment", frame.RS_VAND, 10, 4, 1 << 20, 2560),
         ("rs_c3_plus_10B", frame.RS_VAND, 10, 4, (10 << 20) + 10, 256),
         ("rs_4MiB", frame.RS_VAND, 10, 4, 4 << 20, 640),
         ("xor_swift_1MiB_segment", frame.FLAT_XOR_HD, 10, 6, 1 << 20, 2560)]


def main(rounds=5, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    for tag, be, k, m, size, S in CASES:
        for ck in (frame.CHKSUM_NONE, frame.CHKSUM_CRC32):
            fb = frame.FrameBatch(be, k, m, size, S, hd=4, checksum=ck)
            obj = D.DeviceBuffer(fb.obj_stride * S)
            _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x7A, st.handle), "fill")
            nbytes = S * (size + (k + m) * fb.blocksize)
            # the decode-join of data {0,1,2,3} (RS, no checksum): the LDS-table rest of the copy-through
            # map forked the same way (map_apply_copy)
            dj = be == frame.RS_VAND and ck == frame.CHKSUM_NONE
            out = D.DeviceBuffer(fb.obj_stride * S) if dj else None
            dbytes = S * ((k + 4) * fb.blocksize - 4 * fb.blocksize + size)
            ref = None
            for v in (0, 1, 2):
                d.ecamd_tune(b"frame_tail_fork", v)
                fb.encode(obj, stream=st)
                st.synchronize()
                f = fb.fragments()
                if dj:
                    fb.decode([0, 1, 2, 3], out, stream=st)
                    st.synchronize()
                    f = (f, out.download())
                if ref is None:
                    ref = f
                if dj:
                    assert (f[0] == ref[0]).all() and (f[1] == ref[1]).all(), (tag, ck, v)
                else:
                    assert (f == ref).all(), (tag, ck, v)
            del ref, f
            for _ in range(20):
                fb.encode(obj, stream=st)
            a, b = D.Event(), D.Event()
            times = {}
            for _ in range(rounds):
                for v in (0, 1, 2):
                    d.ecamd_tune(b"frame_tail_fork", v)
                    fb.encode(obj, stream=st)
                    a.record(st)
                    for _ in range(reps):
                        fb.encode(obj, stream=st)
                    b.record(st)
                    st.synchronize()
                    times.setdefault(v, []).append(a.elapsed_ms(b) / reps)
                    if dj:
                        fb.decode([0, 1, 2, 3], out, stream=st)
                        a.record(st)
                        for _ in range(reps):
                            fb.decode([0, 1, 2, 3], out, stream=st)
                        b.record(st)
                        st.synchronize()
                        times.setdefault(("join_0123", v), []).append(a.elapsed_ms(b) / reps)
            for v, ts in times.items():
                ms = statistics.median(ts)
                op, v = (v[0], v[1]) if isinstance(v, tuple) else ("encode", v)
                nb = dbytes if op == "join_0123" else nbytes
                print(json.dumps({"shape": tag, "op": op, "checksum": ck, "frame_tail_fork": v, "ms": round(ms, 4),
                                  "frac": round(nb / (ms * 1e-3) / 8e12, 4)}), flush=True)
            obj.free()
            if out is not None:
                out.free()
            del fb
    d.ecamd_tune(b"frame_tail_fork", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
