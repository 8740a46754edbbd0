#!/usr/bin/env python3
"""A/B of the per-call host path (round 3): tools/e2e_bench.py --per-call-only in child processes,
interleaved rounds, 1 and 8 caller threads, three settings --
  ref-zeroing   ECAMD_FRONTEND_ZERO_ALL=1 ECAMD_COPY_THREADS=0  (the frontend zeroes every buffer in
                full as the reference does; every copy on the caller's thread)
  lean          ECAMD_FRONTEND_ZERO_ALL=0 ECAMD_COPY_THREADS=0  (only uncovered bytes zeroed)
  lean+helpers  ECAMD_FRONTEND_ZERO_ALL=0 ECAMD_COPY_THREADS=4  (default: copies of a call shared
                with the helper threads of host/copy_pool.cpp)
  lean+helpers+pool  ... and the frontend's recycled fragment / object buffers (ECAMD_FRONTEND_POOL_MIB,
                default 256; the others run with 0)
  lean+helpers+pool+direct  ... and decode straight into the object (round 4, frontend.cpp
                decode_direct, ECAMD_FRONTEND_DECODE_DIRECT; the default -- the others run without)
(the staging chunk, ECAMD_PERCALL_CHUNK_KIB, measured at 2 and 4 MiB against the default 8 MiB in round 3:
no gain, profiles/r03_percall_ab1.log).  The order of the settings rotates every round.
One JSON line per run."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SETTINGS = {"ref-zeroing": {"ECAMD_FRONTEND_ZERO_ALL": "1", "ECAMD_COPY_THREADS": "0",
                            "ECAMD_FRONTEND_POOL_MIB": "0"},
            "lean": {"ECAMD_FRONTEND_ZERO_ALL": "0", "ECAMD_COPY_THREADS": "0", "ECAMD_FRONTEND_POOL_MIB": "0"},
            "lean+helpers": {"ECAMD_FRONTEND_ZERO_ALL": "0", "ECAMD_COPY_THREADS": "4",
                             "ECAMD_FRONTEND_POOL_MIB": "0"},
            "lean+helpers+pool": {"ECAMD_FRONTEND_ZERO_ALL": "0", "ECAMD_COPY_THREADS": "4",
                                  "ECAMD_FRONTEND_POOL_MIB": "256", "ECAMD_FRONTEND_DECODE_DIRECT": "0"},
            "lean+helpers+pool+direct": {"ECAMD_FRONTEND_ZERO_ALL": "0", "ECAMD_COPY_THREADS": "4",
                                         "ECAMD_FRONTEND_POOL_MIB": "256", "ECAMD_FRONTEND_DECODE_DIRECT": "1"}}


def run(setting, threads, objects):
    env = dict(os.environ, **SETTINGS[setting])
    env.setdefault("ECAMD_FRONTEND_DECODE_DIRECT", "0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "e2e_bench.py"), "--per-call-only",
                        "--threads", str(threads), "--objects", str(objects)],
                       capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-2000:])
        raise SystemExit(r.returncode)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["setting"] = setting
    return out


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for rnd in range(rounds):
        for threads, objects in ((1, 48), (8, 256)):
            names = list(SETTINGS)
            for setting in names[rnd % len(names):] + names[:rnd % len(names)]:
                res = run(setting, threads, objects)
                res["round"] = rnd
                print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
