#!/usr/bin/env python3
"""Tile shape of the framed split / join stream kernels (round 3): lanes per tile (knob
frame_copy_threads) x 16-byte chunks per lane (frame_copy_u), one workgroup per tile.  Systematic
framed decode (fragments_to_string only: the join) of 256 C3 objects (10 MiB, bs = 1 MiB) and 2560
Swift 1 MiB segments (bs = 104858), and the flat-XOR (10,6,4) framed encode of the Swift segments
(split + XOR + CRC pass).  Interleaved rounds, median; the join's objects checked equal to the
default's.  Fraction of 8 TB/s of 2 x the object bytes (join)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

SHAPES = [(256, 4, 0), (64, 4, 0), (64, 1, 0), (128, 1, 0), (256, 1, 0)]
if len(sys.argv) > 1 and sys.argv[1] == "dpp":  # round 4: knob frame_copy_dpp on the realigning path
    SHAPES = [(256, 1, 0), (256, 1, 1), (64, 1, 0), (64, 1, 1), (128, 1, 1), (256, 4, 1)]
# round 4: the copy-through flat-XOR framed encode (knob frame_xor_copy) -- mode "xorcopy": the XOR
# encode shapes only, dpp 3 marks frame_xor_copy 0 (split + XOR)
if len(sys.argv) > 1 and sys.argv[1] == "xorcopy":  # dp 4: frame_crc_cover 0 (XOR copy-through + CRC pass)
    SHAPES = [(256, 1, 1), (256, 1, 4), (256, 1, 3)]
# round 4: join tiles starting on aligned object chunks (knob frame_join_align); dpp 2 marks them
if len(sys.argv) > 1 and sys.argv[1] == "align":
    SHAPES = [(256, 1, 1), (256, 1, 2), (128, 1, 1), (128, 1, 2)]


def main(rounds=5, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)  # run-time compiled kernels ready before the timing
    st = D.Stream()
    cases = [("c3", frame.RS_VAND, 10, 4, 10 << 20, 256),
             ("swift_1MiB_segment", frame.RS_VAND, 10, 4, 1 << 20, 2560),
             ("xor_swift_encode", frame.FLAT_XOR_HD, 10, 6, 1 << 20, 2560)]
    if len(sys.argv) > 1 and sys.argv[1] == "xorcopy":
        cases = [("xor_swift_encode", frame.FLAT_XOR_HD, 10, 6, 1 << 20, 2560),
                 ("xor_c3_encode", frame.FLAT_XOR_HD, 10, 6, 10 << 20, 256)]
    elif len(sys.argv) > 1 and sys.argv[1] in ("dpp", "align"):
        cases = [("swift_1MiB_segment", frame.RS_VAND, 10, 4, 1 << 20, 2560),
                 ("c3_plus_6", frame.RS_VAND, 10, 4, (10 << 20) + 6 * 10, 256),
                 ("xor_swift_encode", frame.FLAT_XOR_HD, 10, 6, 1 << 20, 2560)]
    if len(sys.argv) > 1 and sys.argv[1] == "sizes":  # the join over payload sizes, ~2.5 GiB of objects each
        cases = [(f"join_bs_{bs}", frame.RS_VAND, 10, 4, 10 * bs, (2560 << 20) // (10 * bs))
                 for bs in (4 << 20, 1 << 20, 512 << 10, 256 << 10, 131072, 104858, 65536, 16384)]
    for tag, be, k, m, size, S in cases:
        fb = frame.FrameBatch(be, k, m, size, S, hd=4)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x5F, st.handle), "fill")
        fb.encode(obj, stream=st)
        out = D.DeviceBuffer(fb.obj_stride * S)
        enc = tag.endswith("encode")
        fn = (lambda: fb.encode(obj, stream=st)) if enc else (lambda: fb.decode([], out, stream=st))
        ref = None
        for t, u, dp in SHAPES:
            d.ecamd_tune(b"frame_copy_threads", t)
            d.ecamd_tune(b"frame_copy_u", u)
            d.ecamd_tune(b"frame_copy_dpp", 1 if dp else 0)
            d.ecamd_tune(b"frame_join_align", 1 if dp == 2 else 0)
            d.ecamd_tune(b"frame_xor_copy", 0 if dp == 3 else 1)
            d.ecamd_tune(b"frame_crc_cover", 0 if dp == 4 else 1)
            fn()
            st.synchronize()
            got = fb.fragments() if enc else out.download()
            if ref is None:
                ref = got
            assert (got == ref).all(), (tag, t, u, dp)
            del got
        del ref
        times = {sh: [] for sh in SHAPES}
        a, b = D.Event(), D.Event()
        for _ in range(20):
            fn()
        for _ in range(rounds):
            for t, u, dp in SHAPES:
                d.ecamd_tune(b"frame_copy_threads", t)
                d.ecamd_tune(b"frame_copy_u", u)
                d.ecamd_tune(b"frame_copy_dpp", 1 if dp else 0)
                d.ecamd_tune(b"frame_join_align", 1 if dp == 2 else 0)
                d.ecamd_tune(b"frame_xor_copy", 0 if dp == 3 else 1)
                d.ecamd_tune(b"frame_crc_cover", 0 if dp == 4 else 1)
                fn()
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                st.synchronize()
                times[(t, u, dp)].append(a.elapsed_ms(b) / reps)
        for (t, u, dp), ts in times.items():
            ms = statistics.median(ts)
            rec = {"op": tag, "lanes": t, "chunks_per_lane": u, "dpp": 1 if dp else 0, "aligned_tiles": dp == 2, "xor_copy": dp != 3, "crc_fused": dp not in (3, 4),
                   "tile_bytes": t * u * 16,
                   "ms": round(ms, 4)}
            if not enc:
                rec["frac"] = round(2 * S * size / (ms * 1e-3) / 8e12, 4)
            print(json.dumps(rec), flush=True)
        obj.free()
        out.free()
        del fb
    d.ecamd_tune(b"frame_copy_threads", 0)
    d.ecamd_tune(b"frame_copy_u", 0)
    d.ecamd_tune(b"frame_copy_dpp", -1)
    d.ecamd_tune(b"frame_join_align", -1)
    d.ecamd_tune(b"frame_xor_copy", 1)
    d.ecamd_tune(b"frame_crc_cover", 1)


if __name__ == "__main__":
    main()
