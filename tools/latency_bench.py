#!/usr/bin/env python3
"""Per-call latency of the drop-in API, one thread, RS(10,4): liberasurecode_encode / _decode
(4 data fragments lost) through this repo's liberasurecode.so.1, with

  own: this repo's codec liberasurecode_rs_vand.so.1 -> libecamd -> the MI355X, and
  ref: the REFERENCE codec (oracle/_ref/liberasurecode_rs_vand.so.1, compiled from /root/reference
       sources) first on LD_LIBRARY_PATH, run in a child process -- the CPU codec the drop-in
       replaces, behind the same frontend, on the same host,

object sizes 4 KiB .. 16 MiB, median / p10 / p90 of N calls, and the crossover: the largest size
at which the CPU codec is still faster per call.  One JSON line per (codec, checksum, size), then
a summary line.  (The reference frontend itself is unbuildable here -- DESIGN.md §2.)"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
SIZES = [4096, 16384, 65536, 262144, 1 << 20, 4 << 20, 16 << 20]


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


BACKEND = {"rs": None, "xor": None}  # set in main: (backend id, k, m, hd)


def measure(codec, reps, repeat=False):
    import ec_api
    be, k, m, hd = BACKEND["cur"]
    out = []
    for ct in (ec_api.CHKSUM_NONE, ec_api.CHKSUM_CRC32):
        desc = ec_api.create(be, k, m, hd=hd, ct=ct)
        assert desc > 0, desc
        for size in SIZES:
            data = os.urandom(size)
            n = reps if size <= (4 << 20) else max(8, reps // 3)
            enc, dec = [], []
            if repeat:  # one operation repeated (a caller encoding, or decoding, object after object)
                for it in range(n + 3):
                    t0 = time.perf_counter()
                    rc, d, p, flen = ec_api.encode(desc, data)
                    t1 = time.perf_counter()
                    assert rc == 0
                    frags = ec_api.fragments(d, k, flen) + ec_api.fragments(p, m, flen)
                    ec_api.lib().liberasurecode_encode_cleanup(desc, d, p)
                    if it >= 3:
                        enc.append(t1 - t0)
                avail = frags[min(m, hd - 1 if hd else m):]
                for it in range(n + 3):
                    t1b = time.perf_counter()
                    rc, got = ec_api.decode(desc, avail, flen)
                    t2 = time.perf_counter()
                    assert rc == 0 and got == data
                    if it >= 3:
                        dec.append(t2 - t1b)
            for it in range(0 if repeat else n + 3):
                t0 = time.perf_counter()
                rc, d, p, flen = ec_api.encode(desc, data)
                t1 = time.perf_counter()
                assert rc == 0
                frags = ec_api.fragments(d, k, flen) + ec_api.fragments(p, m, flen)
                ec_api.lib().liberasurecode_encode_cleanup(desc, d, p)
                avail = frags[min(m, hd - 1 if hd else m):]
                t1b = time.perf_counter()
                rc, got = ec_api.decode(desc, avail, flen)
                t2 = time.perf_counter()
                assert rc == 0 and got == data
                if it >= 3:  # first calls: pool / map set-up
                    enc.append(t1 - t0)
                    dec.append(t2 - t1b)  # includes the ctypes copy-out of the decoded object
            rec = {"codec": codec, "ct": ct, "size": size, "calls": n, "order": "repeat" if repeat else "alternate"}
            for name, xs in (("encode", enc), ("decode_4lost", dec)):
                med = statistics.median(xs)
                rec[f"{name}_us"] = round(med * 1e6, 1)
                rec[f"{name}_p10_us"] = round(pct(xs, 0.1) * 1e6, 1)
                rec[f"{name}_p90_us"] = round(pct(xs, 0.9) * 1e6, 1)
                rec[f"{name}_GiBps"] = round(size / med / 2**30, 3)
            out.append(rec)
            print(json.dumps(rec), flush=True)
        ec_api.lib().liberasurecode_instance_destroy(desc)
    return out


def crossover(own, ref, op):
    """Largest size where the reference CPU codec is faster per call (None: never)."""
    best = None
    for ct in sorted({r["ct"] for r in own}):
        o = {r["size"]: r[f"{op}_us"] for r in own if r["ct"] == ct}
        f = {r["size"]: r[f"{op}_us"] for r in ref if r["ct"] == ct}
        slower = [s for s in SIZES if s in o and s in f and f[s] < o[s]]
        best = max(slower) if slower and (best is None or max(slower) > best) else best
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=25)
    ap.add_argument("--codec", default="both", choices=["both", "own", "ref"])
    ap.add_argument("--max-size", type=int, default=0, help="skip object sizes above this (0: all)")
    ap.add_argument("--backend", default="rs", choices=["rs", "xor"],
                    help="rs: liberasurecode_rs_vand (10, 4); xor: flat_xor_hd (10, 6, 4), hd - 1 = 3 data lost")
    ap.add_argument("--repeat", action="store_true",
                    help="time N encodes in a row, then N decodes (default: encode and decode alternate)")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ec_api
    BACKEND["cur"] = ((ec_api.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, 0) if args.backend == "rs"
                      else (ec_api.EC_BACKEND_FLAT_XOR_HD, 10, 6, 4))
    if args.max_size:
        SIZES[:] = [x for x in SIZES if x <= args.max_size]
    if args.codec in ("own", "ref"):
        measure(args.codec, args.reps, args.repeat)
        return
    ref_dir = os.path.join(ROOT, "oracle", "_ref")
    env = dict(os.environ, LD_LIBRARY_PATH=ref_dir + (":" + os.environ["LD_LIBRARY_PATH"]
                                                      if os.environ.get("LD_LIBRARY_PATH") else ""))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--codec", "ref", "--reps",
                        str(args.reps), "--backend", args.backend, "--max-size", str(args.max_size)] +
                       (["--repeat"] if args.repeat else []), env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    ref = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    for x in ref:
        print(json.dumps(x), flush=True)
    own = measure("own", args.reps, args.repeat)
    print(json.dumps({"summary": "per-call crossover (1 thread, RS 10+4): largest object size where "
                                 "the reference CPU codec is faster than the GPU drop-in",
                      "encode_crossover_bytes": crossover(own, ref, "encode"),
                      "decode_crossover_bytes": crossover(own, ref, "decode_4lost")}), flush=True)


if __name__ == "__main__":
    main()
