#!/usr/bin/env python3
"""Issue cost of the VALU forms the GF(2^16) kernels use (libecamd_probe.so ecamd_probe_valu):
ns per wave-instruction per SIMD, and the same relative to v_xor_b32 (a VOP2 op, 4 cycles per
wave64 instruction per the MI355X guide), which calibrates the clock."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

NAMES = ["v_xor_b32", "v_bitop3_b32", "v_lshlrev_b32_sdwa", "v_bfe_u32", "v_and_b32", "v_perm_b32",
         "v_lshl_or_b32", "ds_read_b128+wait", "v_bfi_b32", "v_lshrrev_b32", "v_bitop3_b32 0xca",
         "v_alignbit_b32"]


def main(iters=4096):
    p = _lib.probe()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    st = D.Stream()
    a, b = D.Event(), D.Event()
    base = None
    for wpc in (2, 4, 8):
        for op, name in enumerate(NAMES):
            _lib.check(p.ecamd_probe_valu(op, wpc, iters, st.handle), "probe")
            a.record(st)
            for _ in range(3):
                p.ecamd_probe_valu(op, wpc, iters, st.handle)
            b.record(st)
            ms = a.elapsed_ms(b) / 3
            waves_per_simd = wpc  # wpc workgroups of 4 waves on 4 SIMDs
            ns = ms * 1e6 / (iters * 8 * waves_per_simd)
            if op == 0:
                base = ns
            print(json.dumps({"op": name, "waves_per_simd": waves_per_simd, "ns_per_inst": round(ns, 4),
                              "cycles_if_xor_is_4": round(4 * ns / base, 2), "cus": cus}), flush=True)


if __name__ == "__main__":
    main()
