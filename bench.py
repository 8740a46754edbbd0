#!/usr/bin/env python3
"""bench.py -- device-resident encode+decode GiB/s of liberasurecode_rs_vand on MI355X.

One step = one pass of the hot path over one batch: RS(k=10, m=4) encode of S stripes of 1 MiB
fragments (BASELINE.json configs[2], "C3"), then decode of the same S stripes with data fragments
{0,1,2,3} erased (every rebuilt fragment needs a full 10-term GF(2^16) dot product).  Inputs are
resident in HBM before the timed region.  value = object bytes (2 * S * k * F per step per GPU,
summed over GPUs) / wall time of the K timed steps (max over ranks), in GiB/s.

Multi-GPU: one process per GPU (torch.distributed.run); stripes are independent, each rank owns
its own S stripes (weak scaling) and there is no data-path collective -- the process group is used
for the start barrier and the max-over-ranks of the elapsed time only.

Extra fields: "roofline" (gf16_stream_kernel, HIP-event timed per launch on the launch stream; peak =
8 TB/s spec, plus a copy peak measured live) and "cpu_baseline" (the reference codec compiled from
its sources -- or the oracle restatement when that build is absent -- on the host cores; rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (before libecamd: one HIP runtime per process)

from liberasurecode_amd import device as D  # noqa: E402
from liberasurecode_amd.shard import Coordinator, stripe_range  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
# second decode pattern per config, data and parity mixed
MIXED_PATTERNS = {"c3": [0, 5, 10, 13], "c2": [0, 4], "c5": [0, 2, 4, 6, 20, 22, 24, 26]}
GIB = float(1 << 30)

CONFIGS = {
    # name: (k, m, fragment bytes, stripes per GPU, decode erasures, description)
    "c3": (10, 4, 1 << 20, 256, [0, 1, 2, 3],
           "C3 liberasurecode_rs_vand k=10 m=4, 1 MiB fragments, encode + decode(4 data missing)"),
    "c2": (4, 2, 64 << 10, 4096, [0, 1],
           "C2 liberasurecode_rs_vand k=4 m=2, 64 KiB fragments, encode + decode(2 data missing)"),
    "c5": (20, 8, 4 << 20, 32, list(range(8)),
           "C5 liberasurecode_rs_vand k=20 m=8, 4 MiB fragments, encode + decode(8 data missing)"),
}


def cpu_baseline(k, m, F, missing, threads, stripes):
    """Host-CPU baseline of the same hot path on this machine.

    Uses the REFERENCE codec itself (oracle/_ref/liberasurecode_rs_vand.so.1, compiled from the
    reference sources by oracle/Makefile, kind "reference") when it is present, else the oracle
    restatement (oracle/ec_oracle.c, same log/antilog algorithm, kind "port").  One stripe per task,
    `threads` threads (ctypes releases the GIL), and separately one thread."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as orc
    from ecdata import stripe_fragments

    ref_path = os.path.join(ROOT, "oracle", "_ref", "liberasurecode_rs_vand.so.1")
    IP = C.POINTER(C.c_int)
    if os.path.exists(ref_path):
        lib = C.CDLL(ref_path)
        lib.make_systematic_matrix.restype = IP
        lib.make_systematic_matrix.argtypes = [C.c_int, C.c_int]
        lib.liberasurecode_rs_vand_encode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                                      C.c_int]
        lib.liberasurecode_rs_vand_decode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                                      IP, C.c_int, C.c_int]
        lib.init_liberasurecode_rs_vand(k, m)
        G = lib.make_systematic_matrix(k, m)
        enc, dec, kind = lib.liberasurecode_rs_vand_encode, lib.liberasurecode_rs_vand_decode, "reference"
        what = "reference liberasurecode_rs_vand.so.1 built from /root/reference sources, gcc -O2"
    else:
        lib = orc.lib()
        G = orc.ints(orc.generator(k, m))
        enc, dec, kind = lib.orc_rs_encode, lib.orc_rs_decode, "port"
        what = "oracle/ec_oracle.c (log/antilog tables as the reference), gcc -O2"
    miss = orc.ints(list(missing) + [-1])

    def job(t, count):
        data = stripe_fragments(t, k, F)
        frags = [np.array(x) for x in data] + [np.zeros(F, np.uint8) for _ in range(m)]
        dp, pp = orc.ptr_array(frags[:k]), orc.ptr_array(frags[k:])
        t0 = time.perf_counter()
        for _ in range(count):
            enc(G, dp, pp, k, m, F)
            dec(G, dp, pp, k, m, miss, F, 1)
        return count, time.perf_counter() - t0

    def run(nthreads, per):
        with ThreadPoolExecutor(nthreads) as ex:
            list(ex.map(job, range(nthreads), [1] * nthreads))  # warm (allocations, page faults)
            t0 = time.perf_counter()
            res = list(ex.map(job, range(nthreads), [per] * nthreads))
            wall = time.perf_counter() - t0
        total = sum(n for n, _ in res)
        return 2 * total * k * F / GIB / wall, total, sum(t for _, t in res)

    value, total, cpu_s = run(threads, stripes)
    one, one_total, one_s = run(1, max(2, stripes // 4))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(value, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1core": round(one, 4),
            "sample": f"{total} stripes x (encode + decode {list(missing)}) of k={k} m={m} F={F} on "
                      f"{threads} threads, plus {one_total} on 1 thread; {what}",
            "cpu_seconds": round(cpu_s + one_s, 2), "cpu_model": model,
            "host_cpus_visible": os.cpu_count()}


def measured_copy_peak(stream, nbytes=1 << 30):
    """Second roofline denominator: non-temporal 16 B/lane copy of 1 GiB on this GPU (GB/s)."""
    import ctypes as C

    from liberasurecode_amd import _lib
    d = _lib.dev()
    d.ecamd_debug_bw_probe.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                       C.c_int64, C.c_void_p]
    buf = D.DeviceBuffer(2 * nbytes)
    a, b = D.Event(), D.Event()
    best = 0.0
    for _ in range(3):
        _lib.check(d.ecamd_debug_bw_probe(0, 4, 2, buf.ptr + nbytes, buf.ptr, nbytes,
                                          stream.handle), "copy probe")
        a.record(stream)
        for _ in range(4):
            d.ecamd_debug_bw_probe(0, 4, 2, buf.ptr + nbytes, buf.ptr, nbytes, stream.handle)
        b.record(stream)
        best = max(best, 2 * nbytes * 4 / (a.elapsed_ms(b) * 1e-3) / 1e9)
    buf.free()
    return best


def pmc_traffic(cfg, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this same
    command (profiles/<round>_<cfg>_summary.json, built by tools/summarize_prof.py from separate
    FETCH_SIZE / WRITE_SIZE passes with the gfx950 FETCH_SIZE x2 correction)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{cfg}_summary.json")),
                       reverse=True):
        try:
            summ = json.load(open(path))
        except Exception:
            continue
        for name, d in summ.get("kernels", {}).items():
            if kernel in name and "hbm_bytes_per_launch" in d:
                return int(d["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=0, help="override stripes per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-stripes", type=int, default=32, help="stripes per CPU thread")
    args = ap.parse_args()

    co = Coordinator()  # one process per GPU; RCCL only for the barrier and time reductions
    world, rank = co.world, co.rank

    k, m, F, S, missing, desc = CONFIGS[args.config]
    if args.stripes:
        S = args.stripes
    assert D.available(), "no HIP device"
    first, S = stripe_range(rank, world, S)  # this rank's shard of independent stripes
    lay = D.Layout.alloc(k + m, F, S)
    stream = D.Stream()
    lay.fill_splitmix(nfrags=k, stripe0=first, stream=stream)
    D.rs_encode(k, m, lay, stream=stream)
    stream.synchronize()

    ev = [(D.Event(), D.Event(), D.Event()) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        D.rs_encode(k, m, lay, stream=stream)
        if i is not None:
            ev[i][1].record(stream)
        D.rs_decode(k, m, missing, lay, stream=stream)
        if i is not None:
            ev[i][2].record(stream)

    for _ in range(args.warmup):
        step()
    stream.synchronize()

    def sync_all():
        D.synchronize()
        torch.cuda.synchronize()

    sync_all()
    co.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    sync_all()
    elapsed = time.perf_counter() - t0
    elapsed = co.reduce([elapsed], op="max")[0]
    co.barrier()

    enc_ms = [a.elapsed_ms(b) for a, b, _ in ev]
    dec_ms = [b.elapsed_ms(c) for _, b, c in ev]
    obj_bytes = S * k * F  # object bytes per stripe batch per GPU
    value = 2 * obj_bytes * args.steps * world / GIB / elapsed
    # dominant kernel: the stream kernel (C3 encode and decode: 10 in, 4 out per launch)
    launch_ms = (sum(enc_ms) + sum(dec_ms)) / (2 * args.steps)
    # algorithmic HBM bytes per launch: k inputs read + outputs written, per stripe
    algo_bytes = S * (2 * k + m + len(missing)) * F // 2
    achieved = algo_bytes / (launch_ms * 1e-3) / 1e9
    width = 2 if max(m, len(missing)) <= 2 else (4 if max(m, len(missing)) <= 4 else 8)
    # <W outputs per pass, KG groups of 4 inputs, CH chunks per lane, PF prefetch, NIB nibble tables>;
    # 8-output passes run its hybrid LDS + L1 lookup form <KG>
    kernel = (f"gf16_hybrid_kernel<{(k + 3) // 4}>" if width == 8 else
              f"gf16_stream_kernel<{width}, {(k + 3) // 4}, 1, false, false>")
    traffic, traffic_src = pmc_traffic(args.config, kernel)
    if traffic is not None and S != CONFIGS[args.config][3]:
        traffic = int(traffic * S / CONFIGS[args.config][3])  # profile ran at the default S

    copy_gbs = measured_copy_peak(stream)

    # The survey's second decode pattern per config, outside the timed steps:
    # erasures mixing data and parity (fewer full dot products than all-data erasures).
    mixed = MIXED_PATTERNS.get(args.config)
    mixed_gibs = None
    if mixed is not None:
        a, b = D.Event(), D.Event()
        D.rs_decode(k, m, mixed, lay, stream=stream)
        a.record(stream)
        for _ in range(5):
            D.rs_decode(k, m, mixed, lay, stream=stream)
        b.record(stream)
        mixed_gibs = round(obj_bytes / GIB / (a.elapsed_ms(b) / 5 / 1e3), 3)

    if rank == 0:
        out = {
            "metric": "device-resident encode+decode GiB/s (RS k=10 m=4, 1 MiB frags), 1/2/4/8 GPU"
            if args.config == "c3" else f"device-resident encode+decode GiB/s ({desc})",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16 (GF(2^16) words)",
            "data": "synthetic (splitmix64 fragments generated in HBM)",
            "config": {"workload": desc, "k": k, "m": m, "fragment_bytes": F,
                       "stripes_per_gpu": S, "decode_missing": missing,
                       "parallelism": f"stripe-sharded x{world} (no data-path collective)"},
            "encode_gibs_per_gpu": round(obj_bytes / GIB / (sum(enc_ms) / len(enc_ms) / 1e3), 3),
            "decode_gibs_per_gpu": round(obj_bytes / GIB / (sum(dec_ms) / len(dec_ms) / 1e3), 3),
            "decode_mixed_pattern": mixed,
            "decode_mixed_gibs_per_gpu": mixed_gibs,
            "roofline": {"bound": "hbm", "kernel": kernel,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "launch_ms": round(launch_ms, 4),
                         "copy_peak_measured": round(copy_gbs, 1),
                         "frac_of_measured_copy": round(achieved / copy_gbs, 4),
                         "algorithmic_bytes_per_launch": algo_bytes},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(k, m, F, missing, args.cpu_threads,
                                               args.cpu_stripes)
        print(json.dumps(out), flush=True)
    co.close()


if __name__ == "__main__":
    main()
