"""Runner (a subprocess of tests/test_ref_api_stress.py and tests/golden/make_stress_golden.py):
tests/ref_api_stress.py for (10, 4) and (20, 8) against this repo's liberasurecode.so.1; prints one
JSON line {"k_m": digests | failure text}.  Started with LD_LIBRARY_PATH=oracle/_ref the frontend
drives the REFERENCE liberasurecode_rs_vand codec on the CPU (test infrastructure only; the product
never links it).  Optional argv[1]: a pattern limit per code (quick runs)."""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ref_api_stress as S  # noqa: E402


def main():
    limit = int(sys.argv[1]) if len(sys.argv) > 1 else None
    out = {}
    for k, m in S.CODES:
        try:
            out[f"{k}_{m}"] = S.stress(k, m, limit=limit)
        except Exception:  # report every failure, keep going
            out[f"{k}_{m}"] = traceback.format_exc()[-1500:]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
