#!/usr/bin/env python3
"""A/B of the framed CHKSUM_CRC32 encode of payloads that are not whole 16 KiB tiles (knob
frame_crc_cover, round 4; development tool): 1 = the bitsliced crc variant over each payload's whole
tiles + the codec and CRC32 of the rest + a finalize folding them (ecamd_frame_api.hip
encode_crc_cover; bs_realign 1 reads the unaligned object chunks as aligned chunks + the neighbour
lane's, realigned, 0 with unaligned loads; frame_tail_bs 1 the payloads' rest by split + plain
encode of their last tiles, 0 on the LDS-table launch), 0 = the copy-through encode + a CRC pass.  Shapes:
Swift's 1 MiB segments (2560 x 1 MiB, bs = 104858: 6 whole tiles + 6554 bytes), C3 objects 10 bytes
longer (bs = 1048578), and 4 MiB objects at k = 10 (bs = 419432).  Fragments checked equal across
the variants first; interleaved rounds, median; fraction of 8 TB/s of the algorithmic bytes (objects
read + payloads written)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

VARIANTS = {"cover_fused": (1, 1, 1), "cover_fused_lds_tail": (1, 1, 0), "codec_then_crc": (0, 1, 1)}


def main(rounds=5, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m = 10, 4
    for tag, size, S, ct in (("swift_1MiB_segment", 1 << 20, 2560, frame.CHKSUM_CRC32),
                             ("c3_plus_10B", (10 << 20) + 10, 256, frame.CHKSUM_CRC32),
                             ("obj_4MiB", 4 << 20, 640, frame.CHKSUM_CRC32),
                             ("swift_1MiB_segment_no_checksum", 1 << 20, 2560, frame.CHKSUM_NONE)):
        fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=ct)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x3C, st.handle), "fill")
        ref = None
        for v in VARIANTS.values():
            d.ecamd_tune(b"frame_crc_cover", v[0])
            d.ecamd_tune(b"bs_realign", v[1])
            d.ecamd_tune(b"frame_tail_bs", v[2])
            fb.encode(obj, stream=st)
            st.synchronize()
            got = fb.fragments()
            if ref is None:
                ref = got
            assert (got == ref).all(), (tag, v)
            del got
        del ref
        algo = S * (size + (k + m) * fb.blocksize)
        for _ in range(20):
            fb.encode(obj, stream=st)
        times = {}
        a, b = D.Event(), D.Event()
        for _ in range(rounds):
            for vname, v in VARIANTS.items():
                d.ecamd_tune(b"frame_crc_cover", v[0])
                d.ecamd_tune(b"bs_realign", v[1])
                d.ecamd_tune(b"frame_tail_bs", v[2])
                fb.encode(obj, stream=st)
                a.record(st)
                for _ in range(reps):
                    fb.encode(obj, stream=st)
                b.record(st)
                st.synchronize()
                times.setdefault(vname, []).append(a.elapsed_ms(b) / reps)
        for vname, ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"shape": tag, "variant": vname, "blocksize": fb.blocksize, "ms": round(ms, 4),
                              "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
        obj.free()
        del fb
    d.ecamd_tune(b"frame_crc_cover", 1)
    d.ecamd_tune(b"bs_realign", -1)
    d.ecamd_tune(b"frame_tail_bs", 1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
