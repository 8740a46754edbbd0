#!/usr/bin/env python3
"""What a device-to-device copy reaches on this MI355X, by several means (2 GiB, bytes counted =
read + write): torch's copy_ (its own copy kernel), hipMemcpyAsync D2D through torch's
untyped-storage copy, and libecamd_probe's non-temporal grid-stride copy (bw_probe_kernel) at the
bench's setting.  The denominators DESIGN.md §4 compares the codec kernels against."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(5):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps)
    return statistics.median(out)


def main():
    n = 2 << 30
    a = torch.empty(n, dtype=torch.uint8, device="cuda")
    b = torch.empty(n, dtype=torch.uint8, device="cuda")
    a.fill_(1)
    res = {}
    res["torch_copy_u8"] = timed(lambda: b.copy_(a))
    a4, b4 = a.view(torch.int32), b.view(torch.int32)
    res["torch_copy_i32"] = timed(lambda: b4.copy_(a4))
    sa, sb = a.untyped_storage(), b.untyped_storage()
    res["storage_copy"] = timed(lambda: sb.copy_(sa))
    p = _lib.probe()
    h = torch.cuda.current_stream().cuda_stream
    for u, w in ((4, 2), (8, 2), (4, 4), (1, 8)):
        res[f"probe_nt_copy_u{u}_w{w}"] = timed(lambda: p.ecamd_probe_bw(0, u, w, b.data_ptr(), a.data_ptr(), n, h))
    for k, ms in res.items():
        print(json.dumps({"copy": k, "ms": round(ms, 4), "GBps": round(2 * n / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
