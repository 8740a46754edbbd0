"""Runner (a subprocess of tests/test_gpu_frontend.py::test_frontend_on_dirty_heap): drives
liberasurecode.so.1 with glibc filling every fresh allocation with garbage (MALLOC_PERTURB_, and
MALLOC_MMAP_THRESHOLD_ so even the 1-4 MiB fragments come from the perturbed heap).

The frontend skips the reference's zeroing passes where this repo's codec overwrites the bytes
anyway (frontend.cpp: lean encode buffers, assemble without a full memset); on a dirty heap any
byte those passes were still needed for -- fragment padding, the object tail -- shows up here as a
mismatch against the restated framing (tests/test_gpu_frontend.py expected()).

Prints one JSON line: {"perturbed": bool, "cases": n, "failures": [...]}."""
import ctypes as C
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import ec_api as E  # noqa: E402
from test_gpu_frontend import expected, make  # noqa: E402

CODES = [("rs", 10, 4), ("rs", 4, 2), ("xor", 3, 3, 3), ("xor", 10, 6, 4)]
SIZES = [1, 1000, 65536 + 3, 300001, (4 << 20) + 7]


def heap_is_dirty():
    libc = C.CDLL(None)
    libc.malloc.restype = C.c_void_p
    libc.free.argtypes = [C.c_void_p]
    p = libc.malloc(1 << 20)
    head = C.string_at(p, 64)
    libc.free(p)
    return head != bytes(64)


def main():
    out = {"perturbed": heap_is_dirty(), "cases": 0, "failures": []}
    for code in CODES:
        for ct in (E.CHKSUM_NONE, E.CHKSUM_CRC32):
            desc, k, m, hd = make(code, ct)
            for size in SIZES:
                data = random.Random(size * 7 + k).randbytes(size)
                rc, dp, pp, flen = E.encode(desc, data)
                frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
                E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
                want = expected(code, k, m, hd, data, ct)
                tag = f"{code} ct={ct} size={size}"
                out["cases"] += 1
                if rc != 0 or frags != want:
                    bad = [i for i in range(len(want)) if i >= len(frags) or frags[i] != want[i]]
                    out["failures"].append(f"encode {tag} rc={rc} fragments {bad}")
                    continue
                lost = [0] if code[0] == "xor" else list(range(min(m, k)))
                for miss in ([], lost, [k]):  # systematic, data lost, one parity lost
                    avail = [f for i, f in enumerate(frags) if i not in miss]
                    rc, obj = E.decode(desc, avail, flen)
                    out["cases"] += 1
                    if rc != 0 or obj != data:
                        out["failures"].append(f"decode {tag} lost={miss} rc={rc}")
                rc, fr = E.reconstruct(desc, frags[1:], flen, 0)
                out["cases"] += 1
                if rc != 0 or fr != frags[0]:
                    out["failures"].append(f"reconstruct {tag} rc={rc}")
            E.lib().liberasurecode_instance_destroy(desc)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
