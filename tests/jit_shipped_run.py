"""Child process of tests/test_gpu_jit_shipped.py: one fresh process, knob "bitslice" at its default
(1: never waits for a compile).  Reports which kernel form C3 encode and a decode take at their FIRST
launch (ecamd_rs_kernel_form + the bitsliced launch counter) and whether the bytes equal the oracle's,
and whether a CHKSUM_CRC32 framed encode runs its bitsliced kernel at the first call.
Environment: LIBERASURECODE_AMD_LIBDIR (which library copy), ECAMD_JIT_CACHE (an empty directory)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import torch  # noqa: E402,F401

import oracle_lib as orc  # noqa: E402
from ecdata import stripe_fragments  # noqa: E402
from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main():
    d = _lib.dev()
    k, m, bs, S = 10, 4, 1 << 17, 4  # above small_chunks (4096 chunks = 64 KiB) for one stripe too
    out = {"available": d.ecamd_bitslice_available()}
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=5)
    want = [list(stripe_fragments(5 + s, k, bs)) + list(orc.encode(k, m, stripe_fragments(5 + s, k, bs)))
            for s in range(S)]
    # "decode_other": a map no build ships -- the reconstruct of destination 2 with {1, 2, 3, 4} lost
    # (prebuild ships every <= 4-loss DECODE of (10, 4), single-loss reconstructs only)
    for name, miss in (("encode", None), ("decode_shipped", [0, 1, 2, 3]), ("decode_other", [1, 2, 3, 4])):
        arr = _lib.ints(miss + [-1]) if miss else None
        other = name == "decode_other"
        out[name + "_form"] = d.ecamd_rs_kernel_form(k, m, arr, 2 if other else -1, 0 if other else 1, bs)
        if miss:
            host = lay.download_stripes()
            host[:, [2] if other else miss] = 0xEE
            lay.upload_stripes(host)
        n0 = d.ecamd_bitslice_launches()
        if other:
            D.rs_reconstruct(k, m, miss, 2, lay)
        elif miss:
            D.rs_decode(k, m, miss, lay)
        else:
            D.rs_encode(k, m, lay)
        got = lay.download_stripes()
        out[name + "_bitsliced_launches"] = d.ecamd_bitslice_launches() - n0
        out[name + "_exact"] = all((got[s, f] == want[s][f]).all() for s in range(S) for f in range(k + m))
    # maps of real rebuild traffic that the bench never times (prebuild.rebuild_ops): a single-destination
    # reconstruct of data fragment 6 with it lost, and a 2-loss decode {2, 7} -- shipped, so bitsliced at
    # their first launch in this fresh process
    for name, miss, dest in (("reconstruct6", [6], 6), ("decode_2_7", [2, 7], -1)):
        arr = _lib.ints(miss + [-1])
        out[name + "_form"] = d.ecamd_rs_kernel_form(k, m, arr, dest, 1 if dest < 0 else 0, bs)
        host = lay.download_stripes()
        host[:, miss] = 0xEE
        lay.upload_stripes(host)
        n0 = d.ecamd_bitslice_launches()
        if dest < 0:
            D.rs_decode(k, m, miss, lay)
        else:
            D.rs_reconstruct(k, m, miss, dest, lay)
        got = lay.download_stripes()
        out[name + "_bitsliced_launches"] = d.ecamd_bitslice_launches() - n0
        out[name + "_exact"] = all((got[s, f] == want[s][f]).all() for s in range(S) for f in range(k + m))
    # one stripe of 16 KiB fragments takes gf16_small_kernel: the form says TABLES and nothing bitsliced
    # runs (ecamd_rs_kernel_form follows launch_gf16's small-launch test)
    out["small16k_form"] = d.ecamd_rs_kernel_form(k, m, None, -1, 1, 16384)
    small = D.Layout.alloc(k + m, 16384, 1)
    small.fill_splitmix(nfrags=k, stripe0=3)
    n0 = d.ecamd_bitslice_launches()
    D.rs_encode(k, m, small)
    out["small16k_bitsliced_launches"] = d.ecamd_bitslice_launches() - n0
    got = small.download_stripes()
    data = stripe_fragments(3, k, 16384)
    out["small16k_exact"] = bool((got[0, :k] == data).all() and (got[0, k:] == orc.encode(k, m, data)).all())
    small.buf.free()
    # the CHKSUM_CRC32 framed encode (ecamd_frame_prebuild ships its kernel): bitsliced at the first
    # call or not, and byte-equal to the LDS-table fused kernel's fragments (knob frame_crc_bs 0)
    from liberasurecode_amd import frame
    size = k * (1 << 16) - 6  # object chunks at offsets that are not multiples of 16
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S)
    obj = D.DeviceBuffer(fb.obj_stride * S)
    _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x77, None), "fill")
    n0 = d.ecamd_bitslice_launches()
    fb.encode(obj)
    out["frame_bitsliced_launches"] = d.ecamd_bitslice_launches() - n0
    first = fb.fragments()
    d.ecamd_tune(b"frame_crc_bs", 0)
    fb.encode(obj)
    d.ecamd_tune(b"frame_crc_bs", -1)
    out["frame_exact"] = bool((fb.fragments() == first).all())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
