"""Runner (a subprocess of tests/test_ref_api_slap.py): tests/ref_api_slap.py for every code against
this repo's liberasurecode.so.1; prints one JSON line {"k_m_hd": "ok" | failure text}.  Started with
LD_LIBRARY_PATH=oracle/_ref the frontend drives the REFERENCE libXorcode on the CPU (test
infrastructure only; the product never links it)."""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ref_api_slap as S  # noqa: E402


def main():
    out = {}
    for k, m, hd in S.CODES:
        try:
            S.slap(k, m, hd)
            out[f"{k}_{m}_{hd}"] = "ok"
        except Exception:  # report every failure, keep going
            out[f"{k}_{m}_{hd}"] = traceback.format_exc()[-1500:]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
