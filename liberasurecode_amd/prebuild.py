"""Build-time compile of the bitsliced kernels the BASELINE configurations run (no GPU needed).

The bitsliced GF(2^16) kernel is generated per coefficient matrix (csrc/host/bitslice.cpp) and is
normally compiled at run time by the `ecamd_jitc` child process; until a compile lands, a process
runs that map on the LDS-table kernels.  `build()` calls `prebuild()` so that the
maps of C2 / C3 / C5 -- encode, the decodes the bench times, single-destination reconstructs -- are
already in `lib/jit/`, which libecamd searches before the per-user cache: a fresh process takes the
bitsliced kernel at their first launch, with or without `ecamd_jitc` / libhiprtc on the machine.
The CHKSUM_CRC32 framed encode's kernels (one per code, ecamd_frame_prebuild) ship the same way.
Every object is named by the run time's own key (request text, target, generator fingerprint), so
a map whose knobs or generator differ simply is not found there and compiles as before.

usage: python -m liberasurecode_amd.prebuild [--arch gfx950] [--jobs N]"""
import argparse
import ctypes as C
import os
import stat
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
JIT_DIR = os.path.join(HERE, "lib", "jit")

# (k, m, missing or None, dest, rebuild_parity): the operations of BASELINE.json configs[1..4] that
# bench.py times, plus __graft_entry__.smoke()'s (rs_vand, k = 10, m = 4) ...
C3_LOST = [[0, 1, 2, 3], [0, 5, 10, 13]]
C5_LOST = [list(range(8)), [0, 2, 4, 6, 20, 22, 24, 26]]
BENCH_OPS = (
    [(4, 2, None, -1, 1), (4, 2, [0, 1], -1, 1), (4, 2, [0, 4], -1, 1)]  # C2
    + [(10, 4, None, -1, 1)] + [(10, 4, p, -1, 1) for p in C3_LOST]  # C3 (and C4's shards)
    + [(10, 4, [d], d, 0) for d in (3, 12)] + [(10, 4, [0, 5, 10, 13], 13, 0)]  # C3 reconstruct, smoke
    + [(20, 8, None, -1, 1)] + [(20, 8, p, -1, 1) for p in C5_LOST]  # C5
    + [(20, 8, C5_LOST[0], d, 0) for d in C5_LOST[0]]  # C5: 8 single-destination reconstructs
    + [(10, 4, p, -1, 1) for p in ([4, 5, 6, 7], [2, 3, 8, 9])]  # tools/multi_bench.py's other patterns
)


# ... and the maps real rebuild traffic uses: for each BASELINE code, every single-loss
# decode (the API's liberasurecode_decode asks rebuild_parity 1, frontend.cpp rs_decode) and every
# single-destination reconstruct with that one fragment lost (Swift's reconstructor,
# liberasurecode_reconstruct_fragment); for Swift's default (10, 4) every 2-, 3- and 4-loss decode as
# well -- all 1,470 erasure patterns (≈3 min on 8 cores, ≈39 MB of code objects; DESIGN.md §4 "Shipped
# kernels").  ECAMD_PREBUILD_FULL=0 stops at the 2-loss decodes (≈25 s, ≈3 MB).  Maps that take the LDS
# tables by shape (k = 4's 1-2-output maps) build nothing.
def rebuild_ops(full=False):
    from itertools import combinations
    ops = []
    for k, m in ((10, 4), (4, 2), (20, 8)):
        n = k + m
        ops += [(k, m, [f], -1, 1) for f in range(n)]
        ops += [(k, m, [f], f, 0) for f in range(n)]
    ops += [(10, 4, list(c), -1, 1) for c in combinations(range(14), 2)]
    if full:
        ops += [(10, 4, list(c), -1, 1) for r in (3, 4) for c in combinations(range(14), r)]
    return ops


def all_ops(full=None):
    if full is None:
        full = os.environ.get("ECAMD_PREBUILD_FULL", "1") != "0"
    seen, out = set(), []
    for op in list(BENCH_OPS) + rebuild_ops(full):
        key = (op[0], op[1], tuple(op[2]) if op[2] is not None else None, op[3], op[4])
        if key not in seen:
            seen.add(key)
            out.append(op)
    return out

# (backend, k, m, hd): the CHKSUM_CRC32 framed encode's codec-and-checksum kernel, one per code whatever
# the object size -- Swift's default rs_vand (10, 4) (whole objects and 1 MiB segments alike), the
# other BASELINE codes, and flat_xor_hd (3, 3, 3)
FRAME_CODES = [(6, 10, 4, 0), (6, 4, 2, 0), (6, 20, 8, 0), (3, 3, 3, 3)]


def _ints(v):
    return (C.c_int * (len(v) + 1))(*(list(v) + [-1]))


def prebuild(arch="gfx950", jobs=8, verbose=False, full=None):
    lib = C.CDLL(os.path.join(HERE, "lib", "libecamd.so"))
    lib.ecamd_bitslice_prebuild.restype = C.c_int
    lib.ecamd_bitslice_prebuild.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_char_p]
    lib.ecamd_frame_prebuild.restype = C.c_int
    lib.ecamd_frame_prebuild.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_char_p]
    lib.ecamd_last_error.restype = C.c_char_p
    os.makedirs(JIT_DIR, exist_ok=True)
    for name in os.listdir(JIT_DIR):  # objects of an earlier generator or knob set are never looked up
        if name.startswith("bs_"):
            os.remove(os.path.join(JIT_DIR, name))
    # the run time uses this directory only if nobody but its owner can write it
    os.chmod(JIT_DIR, stat.S_IRWXU | stat.S_IRGRP | stat.S_IXGRP | stat.S_IROTH | stat.S_IXOTH)

    def one(op):
        if op[0] == "frame":
            _, backend, k, m, hd = op
            return op, lib.ecamd_frame_prebuild(backend, k, m, hd, arch.encode(), JIT_DIR.encode())
        k, m, miss, dest, rebuild = op
        arr = _ints(miss) if miss is not None else None
        rc = lib.ecamd_bitslice_prebuild(k, m, C.cast(arr, C.c_void_p) if arr is not None else None, dest, rebuild,
                                         arch.encode(), JIT_DIR.encode())
        return op, rc

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        results = list(ex.map(one, all_ops(full) + [("frame",) + c for c in FRAME_CODES]))
    bad = [(op, rc) for op, rc in results if rc < 0]
    if verbose:
        for op, rc in results:
            print("prebuild", op, rc)
    if bad:
        raise RuntimeError(f"bitsliced prebuild failed: {bad} ({lib.ecamd_last_error().decode()})")
    return sum(rc for _, rc in results)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="gfx950")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    n = prebuild(a.arch, a.jobs, verbose=True)
    print(f"{n} code objects in {JIT_DIR}")
    sys.exit(0)
