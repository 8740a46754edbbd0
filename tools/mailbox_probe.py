#!/usr/bin/env python3
"""Host -> GPU -> host round trip through a mailbox in coherent pinned memory (round 6; the resident-
server question of DESIGN.md §10): one wave polls for requests the host posts and acks each
(libecamd_probe ecamd_probe_mailbox).  Against it: the per-call path's launch + completion flag.
One JSON line per (round, payload).

usage: python tools/mailbox_probe.py [rounds]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402


def main(rounds=3):
    p = _lib.probe()
    out = (ctypes.c_double * 4)()
    for rnd in range(rounds):
        for payload in (0, 256):
            rc = p.ecamd_probe_mailbox(2000, payload, 20000, out)
            if rc:
                raise SystemExit(f"mailbox probe rc={rc}: {p.ecamd_probe_last_error().decode()}")
            print(json.dumps({"round": rnd, "payload": payload, "mean_us": round(out[0], 2), "min_us": round(out[1], 2),
                              "p50_us": round(out[2], 2), "p90_us": round(out[3], 2)}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
