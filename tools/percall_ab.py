#!/usr/bin/env python3
"""A/B of the per-call host path: tools/e2e_bench.py --per-call-only in child processes,
interleaved rounds, 1 and 8 caller threads, settings --
  ref-zeroing  the frontend zeroes every buffer in full as the reference does, every copy on the
               caller's thread, no recycled buffers, the reference's decode order
  r03-default  round 3's defaults: lean zeroing, 4 copy helpers (host/copy_pool.cpp), recycled
               fragment / object buffers (ECAMD_FRONTEND_POOL_MIB 256)
  direct       + decode straight into the object (round 4, frontend.cpp decode_direct,
               ECAMD_FRONTEND_DECODE_DIRECT)
  direct+tee   + the object <-> data payload copies riding on the codec's staging pack (round 4,
               TeeCopies / ecamd_percall_tee_arm, ECAMD_FRONTEND_TEE) -- the default
Each run reports encode / decode GiB/s without and with the caller's own read of the outputs
(GIL-free memmove, e2e_bench.py per_call).  The order of the settings rotates every round.
One JSON line per run."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SETTINGS = {"ref-zeroing": {"ECAMD_FRONTEND_ZERO_ALL": "1", "ECAMD_COPY_THREADS": "0",
                            "ECAMD_FRONTEND_POOL_MIB": "0", "ECAMD_FRONTEND_DECODE_DIRECT": "0",
                            "ECAMD_FRONTEND_TEE": "0"},
            "r03-default": {"ECAMD_FRONTEND_ZERO_ALL": "0", "ECAMD_COPY_THREADS": "4",
                            "ECAMD_FRONTEND_POOL_MIB": "256", "ECAMD_FRONTEND_DECODE_DIRECT": "0",
                            "ECAMD_FRONTEND_TEE": "0"},
            "direct": {"ECAMD_FRONTEND_ZERO_ALL": "0", "ECAMD_COPY_THREADS": "4",
                       "ECAMD_FRONTEND_POOL_MIB": "256", "ECAMD_FRONTEND_DECODE_DIRECT": "1",
                       "ECAMD_FRONTEND_TEE": "0"},
            "direct+tee": {"ECAMD_FRONTEND_ZERO_ALL": "0", "ECAMD_COPY_THREADS": "4",
                           "ECAMD_FRONTEND_POOL_MIB": "256", "ECAMD_FRONTEND_DECODE_DIRECT": "1",
                           "ECAMD_FRONTEND_TEE": "1"}}


def run(setting, threads, objects):
    env = dict(os.environ, **SETTINGS[setting])
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
