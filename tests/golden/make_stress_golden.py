#!/usr/bin/env python3
"""Generate tests/golden/rs_stress.json: the digests of tests/ref_api_stress.py (the reference's
liberasure_rs_isal_stress_test.c restated for liberasurecode_rs_vand) run over the REFERENCE codec.

Build container only: oracle/_ref/liberasurecode_rs_vand.so.1 is compiled from /root/reference's own
sources (`make -C oracle ref`); tests/ref_api_stress_run.py runs in a child whose LD_LIBRARY_PATH puts
it first, so this repo's frontend (liberasurecode.so.1) drives the reference codec on the CPU.  The
JSON holds data only: per code the SHA-256 of every encoded fragment, decoded object and rebuilt
fragment in call order, and the pattern / call counts."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
ROOT = os.path.dirname(TESTS)
REF = os.path.join(ROOT, "oracle", "_ref")


def main():
    if not os.path.exists(os.path.join(REF, "liberasurecode_rs_vand.so.1")):
        raise SystemExit("oracle/_ref not built (make -C oracle ref)")
    env = dict(os.environ, LD_LIBRARY_PATH=REF + (":" + os.environ["LD_LIBRARY_PATH"]
                                                  if os.environ.get("LD_LIBRARY_PATH") else ""))
    r = subprocess.run([sys.executable, os.path.join(TESTS, "ref_api_stress_run.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=1800, check=True)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for code, v in res.items():
        if not isinstance(v, dict):
            raise SystemExit(f"{code}: {v}")
    out = {"source": "tests/ref_api_stress.py over oracle/_ref/liberasurecode_rs_vand.so.1 (reference sources, CPU)",
           "codes": res}
    with open(os.path.join(HERE, "rs_stress.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
