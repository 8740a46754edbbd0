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
    k, m, bs, S = 10, 4, 1 << 16, 4
    out = {"available": d.ecamd_bitslice_available()}
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=5)
    want = [list(stripe_fragments(5 + s, k, bs)) + list(orc.encode(k, m, stripe_fragments(5 + s, k, bs)))
            for s in range(S)]
    for name, miss in (("encode", None), ("decode_shipped", [0, 1, 2, 3]), ("decode_other", [1, 2, 3, 4])):
        arr = _lib.ints(miss + [-1]) if miss else None
        out[name + "_form"] = d.ecamd_rs_kernel_form(k, m, arr, -1, 1, bs)
        if miss:
            host = lay.download_stripes()
            host[:, miss] = 0xEE
            lay.upload_stripes(host)
        n0 = d.ecamd_bitslice_launches()
        if miss:
            D.rs_decode(k, m, miss, lay)
        else:
            D.rs_encode(k, m, lay)
        got = lay.download_stripes()
        out[name + "_bitsliced_launches"] = d.ecamd_bitslice_launches() - n0
        out[name + "_exact"] = all((got[s, f] == want[s][f]).all() for s in range(S) for f in range(k + m))
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
