#!/usr/bin/env python3
"""A/B of per-call latency settings: tools/latency_bench.py --codec own in child processes,
interleaved rounds -- the copy helpers' batch threshold (ECAMD_COPY_MIN_KIB, default 2048) at 256 KiB
and 1 MiB, and the helpers off.  Earlier forms of this tool compared the round-2 host path, the
recycled buffers and polling the staging streams (profiles/r03_latency_ab1..4.log).
One JSON line per (setting, round, checksum, size) with the median encode / decode latency.
usage: latency_ab.py [rounds] [set: copy | zc | crc | flag | r06 | server | ocrc] [latency_bench.py args]"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SETS = {
    "copy": {"default": {},
             "copy_min_256k": {"ECAMD_COPY_MIN_KIB": "256"},
             "copy_min_1m": {"ECAMD_COPY_MIN_KIB": "1024"},
             "no-helpers": {"ECAMD_COPY_THREADS": "0"}},
    # round 6: inputs read from the pinned slab by the kernel (ZEROCOPY_MODE 3, no H2D DMA), with the
    # small kernel's inputs staged into LDS by 16-byte loads (small_stage 1) or read in place (0)
    "zc": {"default": {},
           "mode3_staged": {"ECAMD_PERCALL_ZEROCOPY_MODE": "3"},
           "mode3_inplace": {"ECAMD_PERCALL_ZEROCOPY_MODE": "3", "ECAMD_TUNE": "small_stage=0"},
           "mode2_inplace": {"ECAMD_TUNE": "small_stage=0"}},
    # round 6: the CRC32 encode's checksums folded into the small-launch kernel (default) or the
    # separate two-launch ecamd_crc32 pass / host zlib (FUSE_CRC 0); round 5's defaults for reference
    "crc": {"default": {},
            "no_fuse": {"ECAMD_PERCALL_FUSE_CRC": "0"},
            "r05_defaults": {"ECAMD_PERCALL_FUSE_CRC": "0", "ECAMD_PERCALL_ZEROCOPY_IN_KIB": "0",
                             "ECAMD_PERCALL_DONE_FLAG": "0"}},
    # round 6: the small kernel's completion flag polled (default) or the stream synchronized
    "flag": {"default": {}, "stream_sync": {"ECAMD_PERCALL_DONE_FLAG": "0"}},
    # round 6, both changes of the per-call path at once against round 5's (inputs by DMA, stream synchronised)
    "r06": {"default": {}, "r05_path": {"ECAMD_PERCALL_ZEROCOPY_IN_KIB": "0", "ECAMD_PERCALL_DONE_FLAG": "0",
                                        "ECAMD_PERCALL_FUSE_CRC": "0"}},
    # round 6: one-launch calls posted to the resident small server (default) or launched
    "server": {"default": {}, "launch": {"ECAMD_PERCALL_SERVER": "0"}},
    # round 6: a small CRC32 call's input checksums taken on the host while the kernel runs (default)
    "ocrc": {"default": {}, "no_overlap": {"ECAMD_PERCALL_OVERLAP_CRC": "0"}},
}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    SETTINGS = SETS[sys.argv[2] if len(sys.argv) > 2 else "copy"]
    extra = sys.argv[3:]  # passed to latency_bench.py (e.g. --max-size 262144)
    for rnd in range(rounds):
        names = list(SETTINGS)
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:  # rotated every round
            env = SETTINGS[name]
            r = subprocess.run([sys.executable, os.path.join(HERE, "latency_bench.py"), "--codec", "own",
                                "--reps", "25"] + extra, capture_output=True, text=True, timeout=600,
                               env=dict(os.environ, **env))
            if r.returncode != 0:
                sys.stderr.write(r.stderr[-2000:])
                raise SystemExit(r.returncode)
            for line in r.stdout.splitlines():
                if line.startswith("{"):
                    rec = json.loads(line)
                    print(json.dumps({"setting": name, "round": rnd, "ct": rec["ct"], "size": rec["size"],
                                      "encode_us": rec["encode_us"], "decode_4lost_us": rec["decode_4lost_us"],
                                      "encode_p90_us": rec["encode_p90_us"],
                                      "decode_4lost_p90_us": rec["decode_4lost_p90_us"]}), flush=True)


if __name__ == "__main__":
    main()
