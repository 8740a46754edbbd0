"""Runner (a subprocess of tests/test_ref_api_invalid.py): runs tests/ref_api_invalid.py's suite
for one backend against this repo's liberasurecode.so.1 and prints one JSON line
{test name: "ok" | failure text}.  Started with LD_LIBRARY_PATH=oracle/_ref the frontend drives the
REFERENCE codec libraries on the CPU (test infrastructure only; the product never links them).

usage: ref_api_invalid_run.py rs|xor"""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ref_api_invalid as R  # noqa: E402


def main():
    a = R.BACKENDS[sys.argv[1]]
    out = {}
    for fn in R.SUITE:
        try:
            fn(a)
            out[fn.__name__] = "ok"
        except Exception:  # report every failure, keep going
            out[fn.__name__] = traceback.format_exc()[-1500:]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
