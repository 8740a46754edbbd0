#!/usr/bin/env python3
"""Device-resident framed path timings at the C3 shape (10 MiB objects, RS(10,4), CRC32):
CRC32 kernel alone (byte vs nibble tables), and whole framed encode / decode per stripe batch.
Prints one JSON line per measurement."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def bs_launches(d):
    import ctypes
    f = d.ecamd_bitslice_launches
    f.restype = ctypes.c_longlong
    return f()


def timed(fn, stream, reps, warm=1):
    a, b = D.Event(), D.Event()
    for _ in range(warm):  # VALU-dense kernels run slower until the clock settles
        fn()
    stream.synchronize()
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    return a.elapsed_ms(b) / reps


def systematic(d, st, fb, out, S, size, tag, reps, copy_gbs):
    """Decode with every data fragment present (src/erasurecode.c:597-607): fragments_to_string
    only -- a copy of S*size object bytes out of the payloads (read + write = 2x the bytes)."""
    for lost in ([], [fb.k, fb.k + 1]):
        for knob, grid in ((1, 0), (1, 1), (0, 0)):
            d.ecamd_tune(b"frame_copy_stream", knob)
            d.ecamd_tune(b"frame_copy_grid", grid)
            ms = timed(lambda: fb.decode(lost, out, stream=st), st, reps, warm=3)
            gbs = 2 * S * size / ms / 1e6
            print(json.dumps({"op": "frame_decode_systematic_" + tag, "lost": lost, "copy_stream": knob,
                              "copy_grid": grid,
                              "ms": round(ms, 4), "GiBps_object": round(S * size / (ms / 1e3) / 2**30, 1),
                              "copy_GBps": round(gbs, 1), "frac_of_copy_probe": round(gbs / copy_gbs, 4),
                              "frac_of_8TBps": round(gbs / 8000, 4)}), flush=True)
    d.ecamd_tune(b"frame_copy_stream", 1)
    d.ecamd_tune(b"frame_copy_grid", 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fused-sweep", action="store_true")
    ap.add_argument("--align", type=int, default=128, help="payload alignment of the fragment batch")
    ap.add_argument("--no-crc-sweep", action="store_true")
    ap.add_argument("--grid-mult", type=int, default=0, help="grid_mult tuning (0 = library default)")
    args = ap.parse_args()
    S, k, m, size = args.stripes, 10, 4, 10 * 1048576
    d = _lib.dev()
    d.ecamd_tune(b"grid_mult", args.grid_mult)
    d.ecamd_tune(b"bitslice", 2)  # run-time compiled kernels ready before any timing (steady state)
    st = D.Stream()
    import bench
    copy_gbs = bench.measured_copy_peak(D, st)[0]
    print(json.dumps({"copy_probe_GBps": round(copy_gbs, 1)}), flush=True)
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, align=args.align)
    print(json.dumps({"align": args.align, "frag_stride": fb.frag_stride, "head": fb.head}), flush=True)
    obj = D.DeviceBuffer(fb.obj_stride * S)
    lay = D.Layout(obj, 1, size, S, fb.obj_stride, fb.obj_stride)
    lay.fill_splitmix(stream=st)
    crc = D.DeviceBuffer(4 * S * (k + m))
    # Random payload bytes: the byte-table CRC lookups conflict in LDS on random data only
    # (all-zero payloads broadcast one entry and would overstate its speed).
    _lib.check(d.ecamd_fill_splitmix(fb.base + 80, fb.stripe_stride, fb.frag_stride, k + m,
                                     fb.blocksize, S, 0, 0x5EED, st.handle), "fill")
    payload_bytes = S * (k + m) * fb.blocksize
    for bits, gap, pos, span in (() if args.no_crc_sweep else
                                 ((4, 8, 0, 16), (5, 8, 1, 64), (5, 8, 1, 128), (4, 8, 1, 64), (7, 8, 1, 64),
                                  (6, 8, 1, 128), (7, 8, 1, 128), (8, 8, 1, 64), (8, 8, 1, 128))):
        for wgs in (0, 4):
            d.ecamd_tune(b"crc_span_kib", span)
            d.ecamd_tune(b"crc_pos", pos)
            d.ecamd_tune(b"crc_bits", bits)
            d.ecamd_tune(b"crc_gap_bits", gap)
            d.ecamd_tune(b"crc_wgs", wgs)
            ms = timed(lambda: _lib.check(d.ecamd_crc32(0, fb.base + 80, fb.stripe_stride,
                                                         fb.frag_stride, k + m, fb.blocksize, S,
                                                         crc.ptr, st.handle), "crc"), st, args.reps)
            print(json.dumps({"op": "crc32", "bits": bits, "gap_bits": gap, "pos": pos, "span_kib": span, "crc_wgs": wgs,
                              "ms": round(ms, 3), "GBps": round(payload_bytes / ms / 1e6, 1)}),
                  flush=True)
    for key, default in ((b"crc_bits", 0), (b"crc_gap_bits", 0), (b"crc_wgs", 0), (b"crc_pos", 1),
                         (b"crc_span_kib", 0)):
        d.ecamd_tune(key, default)
    obj_bytes = S * size
    for unfused, ct in ((0, frame.CHKSUM_NONE), (0, frame.CHKSUM_CRC32), (1, frame.CHKSUM_NONE),
                        (1, frame.CHKSUM_CRC32)):
        fb.checksum = ct
        d.ecamd_tune(b"frame_unfused", unfused)
        n0 = bs_launches(d)
        ms = timed(lambda: fb.encode(obj, stream=st), st, args.reps, warm=15)
        print(json.dumps({"op": "frame_encode", "unfused": unfused, "checksum": ct, "ms": round(ms, 3),
                          "bitsliced_launches": bs_launches(d) - n0,
                          "GiBps_object": round(obj_bytes / (ms / 1e3) / 2**30, 1),
                          "min_traffic_GBps": round((obj_bytes + payload_bytes) / ms / 1e6, 1)}),
              flush=True)
    d.ecamd_tune(b"frame_unfused", 0)
    if args.fused_sweep:  # fused CRC encode: codec tables (byte / nibble) x workgroups per CU x units per CU
        fb.checksum = frame.CHKSUM_CRC32
        # (bitsliced crc variant, its position sets, workgroups per CU (0: one per unit), units per CU);
        # bitsliced 0 = the LDS-table fused kernel (byte tables, 2 workgroups per CU)
        # (..., lane-shift fold)
        variants = [(0, 1, 2, 4, 0), (1, 2, 0, 64, 0), (1, 2, 0, 64, 1), (1, 1, 0, 64, 0), (1, 1, 0, 64, 1),
                    (1, 2, 0, 32, 1), (1, 1, 0, 32, 1), (1, 1, 0, 16, 1)]
        d.ecamd_tune(b"bitslice", 2)
        for bsv, pos, wgs, units, lane in variants:  # compile the crc variants outside the timing
            d.ecamd_tune(b"frame_crc_bs", bsv)
            d.ecamd_tune(b"frame_crc_pos", pos)
            d.ecamd_tune(b"frame_crc_lane", lane)
            fb.encode(obj, stream=st)
        st.synchronize()
        res = {v: [] for v in variants}
        for _ in range(3):
            for bsv, pos, wgs, units, lane in variants:
                d.ecamd_tune(b"frame_crc_bs", bsv)
                d.ecamd_tune(b"frame_crc_pos", pos)
                d.ecamd_tune(b"frame_crc_lane", lane)
                d.ecamd_tune(b"frame_crc_wgs", wgs if not bsv else 0)
                d.ecamd_tune(b"frame_crc_bs_wgs", wgs)
                d.ecamd_tune(b"frame_crc_units", units)
                res[(bsv, pos, wgs, units, lane)].append(timed(lambda: fb.encode(obj, stream=st), st, args.reps, warm=5))
        import statistics
        for (bsv, pos, wgs, units, lane), ts in res.items():
            ms = statistics.median(ts)
            print(json.dumps({"op": "frame_encode_fused_crc", "bitsliced_crc": bsv, "crc_pos": pos, "lane_fold": lane,
                              "wgs": wgs,
                              "units_per_cu": units, "ms": round(ms, 4),
                              "frac": round((obj_bytes + payload_bytes) / ms / 1e6 / 8000, 4)}), flush=True)
        d.ecamd_tune(b"frame_crc_pos", -1)
        d.ecamd_tune(b"frame_crc_lane", -1)
        d.ecamd_tune(b"frame_crc_bs", -1)
        d.ecamd_tune(b"frame_crc_bs_wgs", 0)
        d.ecamd_tune(b"bitslice", 1)
        d.ecamd_tune(b"frame_crc_mb", 0)
        d.ecamd_tune(b"frame_crc_nib", -1)
        d.ecamd_tune(b"frame_crc_wgs", 0)
        d.ecamd_tune(b"frame_crc_units", 0)
    # objects that do not fill the payloads: Swift's default 1 MiB EC segments (bs = 104858) and a
    # C3 object 6 bytes short -- copy-through with zero padding vs split + encode
    # (and two shapes that isolate its costs: aligned payloads that fill exactly, with a partial last
    # 4 KiB tile -- bs = 104864 -- and with none -- bs = 26 x 4096)
    for size2, S2, tag in (((1 << 20), 2560, "swift_1MiB_segment"), (k * (1 << 20) - 6, S, "c3_minus_6B"),
                           (k * 104864, 2560, "swift_aligned_fill"), (k * 26 * 4096, 2560, "swift_tile_multiple")):
        fb2 = frame.FrameBatch(6, k, m, size2, S2, align=args.align)
        obj2 = D.DeviceBuffer(fb2.obj_stride * S2)
        _lib.check(d.ecamd_fill_splitmix(obj2.ptr, fb2.obj_stride, 0, 1, size2, S2, 0, 0xB0B, st.handle), "fill")
        for padded, ct in ((1, frame.CHKSUM_NONE), (0, frame.CHKSUM_NONE), (1, frame.CHKSUM_CRC32),
                           (0, frame.CHKSUM_CRC32)):
            fb2.checksum = ct
            d.ecamd_tune(b"frame_copy_padded", padded)
            ms = timed(lambda: fb2.encode(obj2, stream=st), st, args.reps, warm=3)
            print(json.dumps({"op": "frame_encode_" + tag, "copy_padded": padded, "checksum": ct,
                              "ms": round(ms, 3), "GiBps_object": round(S2 * size2 / (ms / 1e3) / 2**30, 1)}),
                  flush=True)
        out2 = D.DeviceBuffer(fb2.obj_stride * S2)
        fb2.encode(obj2, stream=st)
        systematic(d, st, fb2, out2, S2, size2, tag, args.reps, copy_gbs)
        for padded in (1, 0):
            d.ecamd_tune(b"frame_copy_padded", padded)
            ms = timed(lambda: fb2.decode([0, 1, 2, 3], out2, stream=st), st, args.reps)
            print(json.dumps({"op": "frame_decode_4data_" + tag, "copy_padded": padded, "ms": round(ms, 3),
                              "GiBps_object": round(S2 * size2 / (ms / 1e3) / 2**30, 1)}), flush=True)
        d.ecamd_tune(b"frame_copy_padded", 1)
        out2.free()
        obj2.free()
        fb2.buf.free()
    out = D.DeviceBuffer(fb.obj_stride * S)
    fb.checksum = frame.CHKSUM_NONE
    fb.encode(obj, stream=st)
    systematic(d, st, fb, out, S, size, "c3", args.reps, copy_gbs)
    ms = timed(lambda: fb.decode([0, 1, 2, 3], out, stream=st), st, args.reps)
    print(json.dumps({"op": "frame_decode_4data", "ms": round(ms, 3),
                      "GiBps_object": round(obj_bytes / (ms / 1e3) / 2**30, 1)}), flush=True)
    ms = timed(lambda: fb.verify(stream=st), st, args.reps)
    print(json.dumps({"op": "frame_verify", "ms": round(ms, 3),
                      "GBps": round(payload_bytes / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
