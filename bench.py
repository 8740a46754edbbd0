#!/usr/bin/env python3
"""bench.py -- device-resident encode+decode GiB/s of liberasurecode_rs_vand on MI355X.

One step = one pass of the hot path over one batch: RS(k=10, m=4) encode of S stripes of 1 MiB
fragments (BASELINE.json configs[2], "C3"), then decode of the same S stripes with data fragments
{0,1,2,3} erased (every rebuilt fragment needs a full 10-term GF(2^16) dot product).  Inputs are
resident in HBM before the timed region.  value = object bytes (2 * S * k * F per step, summed
over ranks) / wall time of the K timed steps (max over ranks), in GiB/s.

Multi-GPU (C4): one process per GPU.  Stripes are independent (src/erasurecode.c:383-477), so each
rank owns its own stripes -- S per GPU (--scaling weak, default) or an even split of a fixed total
(--scaling strong, 2048 stripes) -- and there is no data-path collective: the process group
carries the start barrier, the max-over-ranks of the elapsed time and the per-rank rates only.
Ranks come from torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*), or, when
`--gpus N` > 1 is given without them, bench.py starts the N rank processes itself before anything
touches the GPU (fresh child processes, no exec) and relays rank 0's line.

Extra fields: "roofline" (the dominant kernel, per launch from the HIP event pair around the timed
steps on their launch stream -- gaps between launches count; the encode / decode split comes from
PASS_SPLIT_STEPS untimed steps after the region, whose extra events would perturb it; peak =
8 TB/s spec, plus a live copy probe; "trace" = the same figure from the committed rocprofv3 kernel
trace of this command), "cpu_baseline" (the reference codec compiled from its sources -- or the
oracle restatement when that build is absent -- on the host's usable cores; at every N, timed by
rank 0 after all GPU work while the other ranks wait on a gloo barrier), and "c5" (BASELINE
configs[4], k=20 m=8 4 MiB: rebuild of 8 lost fragments, outside the timed steps, on every rank at
once with per-rank figures).
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
PASS_SPLIT_STEPS = 5  # untimed steps after the timed region that time the encode / decode passes apart
# second decode pattern per config, data and parity mixed
MIXED_PATTERNS = {"c3": [0, 5, 10, 13], "c2": [0, 4], "c5": [0, 2, 4, 6, 20, 22, 24, 26]}
GIB = float(1 << 30)
ROUND = "r05"  # profiles/<round>_* written by tools/gpu_prof.sh for this bench

CONFIGS = {
    # name: (k, m, fragment bytes, stripes per GPU, decode erasures, description)
    "c3": (10, 4, 1 << 20, 256, [0, 1, 2, 3],
           "C3 liberasurecode_rs_vand k=10 m=4, 1 MiB fragments, encode + decode(4 data missing)"),
    "c2": (4, 2, 64 << 10, 4096, [0, 1],
           "C2 liberasurecode_rs_vand k=4 m=2, 64 KiB fragments, encode + decode(2 data missing)"),
    "c5": (20, 8, 4 << 20, 32, list(range(8)),
           "C5 liberasurecode_rs_vand k=20 m=8, 4 MiB fragments, encode + decode(8 data missing)"),
}
# c5 fields gathered from every rank (the rest of the c5 object is rank 0's)
C5_PER_RANK = ("encode_frac", "rebuild8_data_frac", "rebuild8_mixed_frac", "reconstruct_x8_gibs")
STRONG_TOTAL = 2048  # C4 strong scaling, 2048 C3 stripes over all GPUs


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle", type=int, default=60,
                    help="untimed steps before the warm-up steps (clock ramp-up; reported)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=0,
                    help="stripes per GPU (weak) or in total (strong); 0 = the config's")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 rebuild-8 fields")
    ap.add_argument("--no-scatter", action="store_true",
                    help="skip the peer-scatter fields of multi-GPU runs")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every usable host core")
    ap.add_argument("--cpu-seconds", type=float, default=2.0,
                    help="target wall seconds of the multi-thread CPU-baseline leg")
    ap.add_argument("--dry-run", action="store_true",
                    help="GPU-less rehearsal of the rank / shard plumbing (gloo, no kernels)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ rank launcher ----

def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Start n rank processes of this script (fresh interpreters; this process never touches
    the GPU) and return the highest exit code.  A failing rank takes the others down with it."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        out = None if r == 0 else subprocess.DEVNULL  # rank 0 prints the line
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=out))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = max(rc, abs(code))
                for q in live:  # the others would wait forever at the next barrier
                    q.kill()
        time.sleep(0.05)
    return rc


def world_from_env(gpus):
    """(world, launched_by_us) -- fails loudly when --gpus disagrees with the launcher's world."""
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; they must agree")
        return world
    return 1 if gpus <= 1 else None


# ------------------------------------------------------------------ CPU baseline ----

def usable_cores():
    """(usable, visible, quota): CPUs this process may run on -- the affinity set, capped by a
    cgroup v2 CPU quota when one is set (cpu.max) -- and what os.cpu_count() shows."""
    visible = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = visible
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, math.floor(quota)))
    return usable, visible, aff, quota


def cpu_baseline(k, m, F, missing, threads, target_s):
    """Host-CPU baseline of the same hot path on this machine.

    Uses the REFERENCE codec itself (oracle/_ref/liberasurecode_rs_vand.so.1, compiled from the
    reference sources by oracle/Makefile, kind "reference") when it is present, else the oracle
    restatement (oracle/ec_oracle.c, same log/antilog algorithm, kind "port").  One stripe per task
    on `threads` threads (ctypes releases the GIL), sized from a 1-thread calibration so the
    multi-thread leg runs about target_s seconds; also reported per core."""
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

    one, one_total, one_s = run(1, 4)
    per_stripe_s = one_s / one_total
    per = max(2, int(round(target_s / per_stripe_s)))
    value, total, cpu_s = run(threads, per)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable, visible, aff, quota = usable_cores()
    return {"value": round(value, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1core": round(one, 4),
            "sample": f"{total} stripes x (encode + decode {list(missing)}) of k={k} m={m} F={F} "
                      f"on {threads} threads, plus {one_total} on 1 thread; {what}",
            "cpu_seconds": round(cpu_s + one_s, 2), "cpu_model": model,
            "cores_usable": usable, "host_cpus_visible": visible, "affinity_cpus": aff,
            "cgroup_cpu_quota": quota,
            "note": "cores = the CPUs this job may use (affinity capped by the cgroup CPU quota); "
                    "host_cpus_visible is the whole machine"}


# ------------------------------------------------------------------ GPU helpers ----

def measured_copy_peak(D, stream, nbytes=1 << 30):
    """Second roofline denominator: the fastest of two non-temporal 16 B/lane copies of 1 GiB on this
    GPU (GB/s) from the measurement library (liberasurecode_amd/lib/libecamd_probe.so, not the
    product) -- the round-1 probe (2 resident 256-lane workgroups per CU, 4 chunks per lane, grid-
    stride) and one one-wave workgroup per 1 KiB tile in dispatcher order, which copies ~15% faster
    (DESIGN.md §4).  Returns (GB/s, per-probe GB/s)."""
    from liberasurecode_amd import _lib
    p = _lib.probe()
    buf = D.DeviceBuffer(2 * nbytes)
    a, b = D.Event(), D.Event()
    probes = {"grid_stride_4x256": lambda: p.ecamd_probe_bw(0, 4, 2, buf.ptr + nbytes, buf.ptr, nbytes,
                                                            stream.handle),
              "wave_per_1KiB_tile": lambda: p.ecamd_probe_copy_tiles(64, buf.ptr + nbytes, buf.ptr, nbytes,
                                                                     stream.handle)}
    rates = {}
    for _ in range(3):
        for name, fn in probes.items():
            _lib.check(fn(), "copy probe " + name)
            a.record(stream)
            for _ in range(4):
                fn()
            b.record(stream)
            rate = 2 * nbytes * 4 / (a.elapsed_ms(b) * 1e-3) / 1e9
            rates[name] = max(rates.get(name, 0.0), rate)
    buf.free()
    return max(rates.values()), {k: round(v, 1) for k, v in rates.items()}


def dispatches_per_pass(k, width, F, S, cus):
    """Launches of the stream kernel one strided rs_encode / rs_decode pass makes
    (ecamd_device.hip launch_stream_pass): at most 32 (4-output passes) or 64 tiles per resident
    workgroup per launch -- a tile is 256 lanes x 16 B of every fragment, 4 workgroups per CU --
    split as evenly as the stripes allow.  C3 (256 stripes of 1 MiB, 256 CUs): 2."""
    if width == 8:
        return 1  # 8-output passes: the bitsliced kernel
    tiles = S * -(-F // 4096)
    limit = (32 if width == 4 else 64) * cus * 4
    return max(1, -(-tiles // limit))


def profile_summary(cfg):
    """The committed rocprofv3 evidence for this command (tools/gpu_prof.sh ->
    tools/summarize_prof.py): profiles/<round>_<cfg>_summary.json, newest round first."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{cfg}_summary.json")),
                       reverse=True):
        try:
            return json.load(open(path)), os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


def _profile_world(command):
    """--gpus N of the profiled command line (1 when absent); None when the summary names no bench.py
    command -- such a summary is never quoted as this run's trace."""
    if "bench.py" not in command:
        return None
    parts = command.split()
    for i, p in enumerate(parts[:-1]):
        if p == "--gpus":
            try:
                return int(parts[i + 1])
            except ValueError:
                return None
    return 1


def kernel_entry(summ, kernel):
    for name, d in (summ or {}).get("kernels", {}).items():
        if kernel in name:
            return d
    return None


def c5_rebuild(D, stream, reps=30, warm=120):
    """BASELINE configs[4]: k=20 m=8, 4 MiB fragments, 8 fragments lost, 32 stripes in HBM.
    'reconstruct with 8 missing' two ways: one pass that rebuilds all 8 (ecamd_rs_decode with
    rebuild_parity: the k inputs are read once, inverse / composite rows from one host-side
    inversion) and 8 single-destination ecamd_rs_reconstruct launches (what 8
    liberasurecode_reconstruct_fragment calls do, src/erasurecode.c:748)."""
    from liberasurecode_amd import _lib
    k, m, F, S, lost, _ = CONFIGS["c5"]
    dev = _lib.dev()
    # 8-output passes run the run-time compiled bitsliced kernel (ecamd_jit.hip): compile it on the
    # warm-up launch of each matrix (knob 2 waits for the compile), time the steady state
    dev.ecamd_tune(b"bitslice", 2)
    lay = D.Layout.alloc(k + m, F, S)
    lay.fill_splitmix(nfrags=k, stream=stream)
    D.rs_encode(k, m, lay, stream=stream)
    out = {"workload": "C5 k=20 m=8, 4 MiB fragments, 32 stripes, 8 lost", "stripes": S,
           "kernel": ("ecamd_bs_kernel (bitsliced, run-time compiled per matrix)"
                      if dev.ecamd_bitslice_available() else "gf16_hybrid_kernel<5> (LDS tables)")}
    a, b = D.Event(), D.Event()

    def timed(fn):
        # steady state: the clock settles over the first launches of a new kernel mix, and it has
        # dropped while the compiles above kept the GPU idle -- 120 launches are ~80 ms of load,
        # the settle the main steps use
        for _ in range(warm):
            fn()
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        stream.synchronize()
        return a.elapsed_ms(b) / reps

    # compile every matrix first (one launch each), so no timed() warm-up straddles a compile stall
    D.rs_encode(k, m, lay, stream=stream)
    for pat in (lost, MIXED_PATTERNS["c5"]):
        D.rs_decode(k, m, pat, lay, stream=stream)
    for d in lost:  # single-destination maps (bitsliced when bs_narrow_min_k takes them)
        D.rs_reconstruct(k, m, lost, d, lay, stream=stream)
    stream.synchronize()
    # per launch: k inputs read + 8 outputs written per stripe (algorithmic bytes)
    algo = S * (k + 8) * F
    for name, pat in (("data", lost), ("mixed", MIXED_PATTERNS["c5"])):
        ms = timed(lambda: D.rs_decode(k, m, pat, lay, stream=stream))
        out[f"rebuild8_{name}_pattern"] = pat
        out[f"rebuild8_{name}_ms"] = round(ms, 4)
        out[f"rebuild8_{name}_gibs"] = round(S * k * F / GIB / (ms * 1e-3), 2)
        out[f"rebuild8_{name}_frac"] = round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    ms = timed(lambda: [D.rs_reconstruct(k, m, lost, d, lay, stream=stream) for d in lost])
    out["reconstruct_x8_ms"] = round(ms, 4)
    out["reconstruct_x8_gibs"] = round(S * k * F / GIB / (ms * 1e-3), 2)
    ms = timed(lambda: D.rs_encode(k, m, lay, stream=stream))
    out["encode_ms"] = round(ms, 4)
    out["encode_frac"] = round(S * (k + m) * F / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    out["bitslice_compile_failures"] = dev.ecamd_bitslice_wait()
    # the same launches on the LDS-table kernel, for comparison
    dev.ecamd_tune(b"bitslice", 0)
    ms = timed(lambda: D.rs_decode(k, m, lost, lay, stream=stream))
    out["lds_rebuild8_data_frac"] = round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    ms = timed(lambda: D.rs_encode(k, m, lay, stream=stream))
    out["lds_encode_frac"] = round(S * (k + m) * F / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    dev.ecamd_tune(b"bitslice", 1)
    lay.buf.free()
    return out


def peer_scatter(D, stream, home, ndev, S=8, reps=5):
    """SURVEY §8f f4 on a multi-GPU node (rank 0, after the timed steps): S encoded C3 stripes on
    this rank's GPU, fragment f of every stripe placed on device f % ndev with
    ecamd_scatter_fragments (per-destination copy lanes over xGMI), every destination byte checked
    against the source, then `reps` timed scatters.  Reference anchor: the placement the rs_vand
    shim's callers do per fragment (src/backends/rs_vand/liberasurecode_rs_vand.c:119-145)."""
    import ctypes as C

    import torch

    from liberasurecode_amd import _lib
    k, m, F = 10, 4, 1 << 20
    h = _lib.dev()
    f_scatter = h.ecamd_scatter_fragments
    f_scatter.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int,
                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lay = D.Layout.alloc(k + m, F, S)
    lay.fill_splitmix(nfrags=k, stream=stream)
    D.rs_encode(k, m, lay, stream=stream)
    stream.synchronize()
    src = lay.download_stripes()
    devs = [(home + f) % ndev for f in range(k + m)]
    bufs = []
    try:
        for f in range(k + m):
            torch.cuda.set_device(devs[f])
            bufs.append(D.DeviceBuffer(S * F))
        torch.cuda.set_device(home)
        args = (lay.buf.ptr, lay.stripe_stride, lay.frag_stride, F, k + m, S, _lib.ints(devs),
                (C.c_void_p * (k + m))(*[b.ptr for b in bufs]), _lib.i64s([F] * (k + m)),
                stream.handle)

        def run():
            _lib.check(f_scatter(*args), "ecamd_scatter_fragments")

        run()
        stream.synchronize()
        exact = True
        for f in range(k + m):
            torch.cuda.set_device(devs[f])
            got = bufs[f].download(S * F).reshape(S, F)
            exact = exact and bool((got == src[:, f]).all())
        torch.cuda.set_device(home)
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        stream.synchronize()
        dt = time.perf_counter() - t0
        remote = sum(1 for d in devs if d != home)
        return {"devices": ndev, "stripes": S, "fragment_bytes": F, "dst_devices": devs,
                "bytes_exact": exact, "ms": round(dt * 1e3 / reps, 4),
                "gbs_total": round(reps * S * (k + m) * F / dt / 1e9, 2),
                "gbs_over_xgmi": round(reps * S * remote * F / dt / 1e9, 2)}
    finally:
        for f, b in enumerate(bufs):
            torch.cuda.set_device(devs[f])
            b.free()
        torch.cuda.set_device(home)
        lay.buf.free()


def rank0_cpu_baseline(co, args, k, m, F, missing):
    """The host-CPU baseline at every N (north_star: "from the same run"): rank 0 times it after
    every GPU measurement of the run, while the other ranks wait on a gloo barrier (blocked in a
    socket read, not spinning on a core).  Returns rank 0's figure (None elsewhere / when off)."""
    if args.no_cpu_baseline:
        return None
    co.cpu_barrier()  # every rank is done with the GPU
    out = None
    if co.rank == 0:
        usable = usable_cores()[0]
        out = cpu_baseline(k, m, F, missing, args.cpu_threads or usable, args.cpu_seconds)
        out["ranks_idle"] = co.world - 1
    co.cpu_barrier()
    return out


# ------------------------------------------------------------------ main ----

def main():
    args = parse_args()
    world = world_from_env(args.gpus)
    if world is None:  # --gpus N > 1 without a launcher: start the ranks (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    if args.dry_run:
        os.environ.setdefault("ECAMD_DIST_BACKEND", "gloo")
    from liberasurecode_amd.shard import Coordinator, split_range, stripe_range

    # one process per GPU; RCCL only for the barrier and time reductions.  Device identities are
    # all-gathered over gloo first; ranks that landed on one GPU fail here, named (shard.py)
    try:
        co = Coordinator()
    except Exception as e:
        sys.stderr.write(f"bench.py: coordinator setup failed: {e}\n")
        sys.exit(2)
    world, rank = co.world, co.rank
    ranks_seen = int(co.reduce([1.0], op="sum")[0])
    if ranks_seen != world:
        raise SystemExit(f"bench.py: process group has {ranks_seen} ranks, expected {world}")

    k, m, F, S_cfg, missing, desc = CONFIGS[args.config]
    if args.scaling == "weak":
        first, S = stripe_range(rank, world, args.stripes or S_cfg)
    else:
        first, S = split_range(rank, world, args.stripes or STRONG_TOTAL)
    total_stripes = int(co.reduce([float(S)], op="sum")[0])
    # every stripe exactly once over the ranks (independent shards, no data-path collective)
    cover = [0.0] * total_stripes
    for s in range(first, first + S):
        cover[s] = 1.0
    cover = co.reduce(cover, op="sum")
    if any(c != 1.0 for c in cover):
        raise SystemExit("bench.py: stripe shards do not cover the batch exactly once")

    if args.dry_run:
        co.barrier()
        per_rank_stripes = [int(x) for x in co.per_rank(S)]
        cpu = rank0_cpu_baseline(co, args, k, m, F, missing)
        if rank == 0:
            line = {"dry_run": True, "n_gpus": world, "ranks_seen": ranks_seen,
                    "scaling": args.scaling, "total_stripes": total_stripes,
                    "stripes_per_rank": per_rank_stripes,
                    "covered_once": True, "coord_backend": co.coord_backend,
                    "devices": co.devices, "shared_devices": co.shared_devices}
            if cpu is not None:
                line["cpu_baseline"] = cpu
            print(json.dumps(line), flush=True)
        co.close()
        return

    import torch

    from liberasurecode_amd import device as D

    assert D.available(), "no HIP device"
    from liberasurecode_amd import _lib
    # passes of 5-8 outputs (--config c5) take the run-time compiled bitsliced kernel: compile it in
    # the first (untimed) launches so the timed steps never switch kernels midway
    _lib.dev().ecamd_tune(b"bitslice", 2)
    lay = D.Layout.alloc(k + m, F, S)
    stream = D.Stream()
    lay.fill_splitmix(nfrags=k, stripe0=first, stream=stream)
    D.rs_encode(k, m, lay, stream=stream)
    D.rs_decode(k, m, missing, lay, stream=stream)
    stream.synchronize()
    # which kernel a pass runs, and in how many launches: the run-time compiled bitsliced kernel
    # (3-4 outputs in one-wave 4 KiB tiles, 5-8 in 16 KiB tiles) counts its launches
    import ctypes
    bs_count = _lib.dev().ecamd_bitslice_launches
    bs_count.restype = ctypes.c_longlong
    n0 = bs_count()
    D.rs_encode(k, m, lay, stream=stream)
    stream.synchronize()
    bs_enc = bs_count() - n0
    n0 = bs_count()
    D.rs_decode(k, m, missing, lay, stream=stream)
    stream.synchronize()
    bs_dec = bs_count() - n0
    # one per-launch figure for both passes only when both run the same form in as many launches
    if (bs_enc > 0) != (bs_dec > 0) or (bs_enc and bs_enc != bs_dec):
        raise SystemExit(f"bench.py: encode / decode passes run different kernels or launch counts "
                         f"(bitsliced launches {bs_enc} / {bs_dec}); the per-launch roofline would be misstated")
    bs_per_pass = bs_enc

    # The timed steps carry ONE event pair (around all of them): events recorded between the passes
    # are markers the command processor serialises on, and cost ~1% of the value at C3
    # (profiles/r06_gap_ab.json).  The encode / decode split is timed afterwards, outside the region.
    ev_all = (D.Event(), D.Event())

    def step():
        D.rs_encode(k, m, lay, stream=stream)
        D.rs_decode(k, m, missing, lay, stream=stream)

    # Settle: the GPU leaves its idle clocks only after tens of ms of sustained load (C3 at warm-up
    # 2 / 5 / 20 / 80 steps: 0.70 / 0.72 / 0.739 / 0.741 of 8 TB/s, profiles/r02_warmup_sweep.log),
    # so a fixed number of untimed steps runs before the W warm-up steps; reported in the line.
    settle_t0 = time.perf_counter()
    for _ in range(args.settle):
        step()
    stream.synchronize()
    settle_ms = (time.perf_counter() - settle_t0) * 1e3
    for _ in range(args.warmup):
        step()
    stream.synchronize()

    def sync_all():
        D.synchronize()
        torch.cuda.synchronize()

    sync_all()
    co.barrier()
    t0 = time.perf_counter()
    ev_all[0].record(stream)
    for _ in range(args.steps):
        step()
    ev_all[1].record(stream)
    sync_all()
    elapsed = time.perf_counter() - t0
    elapsed = co.reduce([elapsed], op="max")[0]
    co.barrier()

    region_ms = ev_all[0].elapsed_ms(ev_all[1])
    # encode / decode split: PASS_SPLIT_STEPS more steps with an event between the passes (untimed)
    ev = [(D.Event(), D.Event(), D.Event()) for _ in range(PASS_SPLIT_STEPS)]
    for a, b, c in ev:
        a.record(stream)
        D.rs_encode(k, m, lay, stream=stream)
        b.record(stream)
        D.rs_decode(k, m, missing, lay, stream=stream)
        c.record(stream)
    stream.synchronize()
    enc_ms = [a.elapsed_ms(b) for a, b, _ in ev]
    dec_ms = [b.elapsed_ms(c) for _, b, c in ev]
    obj_bytes = S * k * F  # object bytes per batch on this rank
    value = 2 * total_stripes * k * F * args.steps / GIB / elapsed
    enc_gibs = obj_bytes / GIB / (sum(enc_ms) / len(enc_ms) / 1e3)
    dec_gibs = obj_bytes / GIB / (sum(dec_ms) / len(dec_ms) / 1e3)
    per_rank = co.reduce([enc_gibs if r == rank else 0.0 for r in range(world)] +
                         [dec_gibs if r == rank else 0.0 for r in range(world)], op="sum")
    # dominant kernel: the stream kernel (C3 encode and decode: 10 in, 4 out per launch); a pass
    # (one rs_encode / rs_decode call) may run as several launches of it, see dispatches_per_pass
    width = 2 if max(m, len(missing)) <= 2 else (4 if max(m, len(missing)) <= 4 else 8)
    bitsliced = bs_per_pass > 0
    per_pass = bs_per_pass if bitsliced else dispatches_per_pass(k, width, F, S, torch.cuda.get_device_properties(
        torch.cuda.current_device()).multi_processor_count)
    pass_ms = region_ms / (2 * args.steps)
    launch_ms = pass_ms / per_pass  # HIP events bracket the timed steps: gaps between launches count
    # algorithmic HBM bytes per launch: k inputs read + outputs written, per stripe
    algo_bytes = S * (2 * k + m + len(missing)) * F // 2 // per_pass
    achieved = algo_bytes / (launch_ms * 1e-3) / 1e9
    per_rank_launch_ms = co.per_rank(launch_ms)
    kernel = ("ecamd_bs_kernel" if bitsliced else f"gf16_hybrid_kernel<{(k + 3) // 4}>" if width == 8 else
              f"gf16_stream_kernel<{width}, {(k + 3) // 4}, 1, false, false>")
    kernel_form = (("bitsliced, one-wave 4 KiB tiles" if width <= 4 else "bitsliced, 16 KiB tiles")
                   if bitsliced else "LDS split tables")

    # The survey's second decode pattern per config, outside the timed steps:
    # erasures mixing data and parity.  Every rank decodes its own shard at once (as in the timed
    # steps), so at N > 1 the figure is per GPU under the same concurrent load.
    mixed = MIXED_PATTERNS.get(args.config)
    mixed_gibs = None
    per_rank_mixed = None
    if mixed is not None:
        D.rs_decode(k, m, mixed, lay, stream=stream)
        stream.synchronize()
        co.barrier()
        a, b = D.Event(), D.Event()
        a.record(stream)
        for _ in range(5):
            D.rs_decode(k, m, mixed, lay, stream=stream)
        b.record(stream)
        stream.synchronize()
        mixed_gibs = obj_bytes / GIB / (a.elapsed_ms(b) / 5 / 1e3)
        per_rank_mixed = co.reduce([mixed_gibs if r == rank else 0.0 for r in range(world)], "sum")
    co.barrier()

    out = None
    if rank == 0:
        copy_gbs, copy_probes = measured_copy_peak(D, stream)
        summ, summ_src = profile_summary(args.config)
        # the committed trace describes ONE command (bench.py --gpus 1, its config and stripes):
        # quote it only for a run of that shape
        prof_world = _profile_world((summ or {}).get("command", ""))
        prof_stripes = (summ or {}).get("stripes_per_gpu", S_cfg)
        trace_match = (summ is not None and summ.get("config") == args.config and
                       prof_world == world and prof_stripes == S and args.scaling == "weak")
        kd = kernel_entry(summ, kernel) or {}
        # PMC traffic is a measurement of the profiled command only: quoted for a run of that shape
        traffic = kd.get("hbm_bytes_per_launch") if trace_match else None
        trace = None if trace_match else {
            "omitted": f"{summ_src} profiles config={(summ or {}).get('config')} "
                       f"gpus={prof_world} stripes={prof_stripes}, not this run"}
        timed_ns = kd.get("timed_avg_ns")
        if timed_ns and trace_match:
            t_pass = kd.get("dispatches_per_pass", 1)
            t_algo = algo_bytes * per_pass // t_pass * prof_stripes // S
            trace = {"source": summ_src, "timed_launches": kd.get("timed_calls"),
                     "dispatches_per_pass": t_pass,
                     "launch_ms": round(timed_ns / 1e6, 4),
                     "achieved": round(t_algo / timed_ns, 1),
                     "frac": round(t_algo / timed_ns / HBM_PEAK_GBS, 4),
                     "kernel_ms_per_step": round(2 * t_pass * timed_ns / 1e6, 4),
                     "profiled_ms_per_step": (summ or {}).get("ms_per_step")}
        out = {
            "metric": "device-resident encode+decode GiB/s (RS k=10 m=4, 1 MiB frags), 1/2/4/8 GPU"
            if args.config == "c3" else f"device-resident encode+decode GiB/s ({desc})",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"steps": args.settle, "ms": round(settle_ms, 1),
                       "note": "untimed steps before the warm-up: the GPU's clocks ramp under sustained load"},
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u16 (GF(2^16) words)",
            "data": "synthetic (splitmix64 fragments generated in HBM)",
            "config": {"workload": desc, "k": k, "m": m, "fragment_bytes": F,
                       "stripes_per_gpu": S, "stripes_total": total_stripes,
                       "decode_missing": missing,
                       "parallelism": f"stripe-sharded x{world} (no data-path collective)"},
            "ranks_seen": ranks_seen,
            "per_rank_encode_gibs": [round(x, 2) for x in per_rank[:world]],
            "per_rank_decode_gibs": [round(x, 2) for x in per_rank[world:]],
            "encode_gibs_per_gpu": round(enc_gibs, 3),
            "decode_gibs_per_gpu": round(dec_gibs, 3),
            "decode_mixed_pattern": mixed,
            "decode_mixed_gibs_per_gpu": (round(sum(per_rank_mixed) / world, 3)
                                          if per_rank_mixed else None),
            "per_rank_decode_mixed_gibs": ([round(x, 2) for x in per_rank_mixed]
                                           if per_rank_mixed else None),
            "coord_backend": co.coord_backend,
            "devices": co.devices,
            "shared_devices": co.shared_devices,
            "roofline": {"bound": "hbm", "kernel": kernel, "kernel_form": kernel_form,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": (summ_src if trace_match else
                                            "none: the committed PMC profile is of another run shape "
                                            "(see trace.omitted)"),
                         "launch_ms": round(launch_ms, 4),
                         "per_rank_launch_ms": [round(x, 4) for x in per_rank_launch_ms],
                         "per_rank_frac": [round(algo_bytes / (x * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                           for x in per_rank_launch_ms],
                         "dispatches_per_pass": per_pass,
                         "timed_region_event_ms": round(region_ms, 4),
                         "encode_pass_ms": round(sum(enc_ms) / len(enc_ms), 4),
                         "decode_pass_ms": round(sum(dec_ms) / len(dec_ms), 4),
                         "pass_split": f"{PASS_SPLIT_STEPS} untimed steps after the region, "
                                       "an event between the passes",
                         "copy_peak_measured": round(copy_gbs, 1),
                         "copy_peak_rank": 0,
                         "copy_probes": copy_probes,
                         "frac_of_measured_copy": round(achieved / copy_gbs, 4),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "trace": trace},
        }
    lay.buf.free()
    # C5 (BASELINE configs[4]) on every rank at once, after one barrier: each GPU rebuilds its own
    # 32 stripes under the same concurrent load as the timed steps
    if not args.no_c5 and args.config == "c3":
        co.barrier()
        c5 = c5_rebuild(D, stream)
        per_rank_c5 = {key: co.per_rank(c5[key]) for key in C5_PER_RANK}
        if rank == 0:
            c5["ranks"] = f"all {world} ranks at once" if world > 1 else "one rank"
            c5["per_rank"] = {key: [round(x, 4) for x in v] for key, v in per_rank_c5.items()}
            out["c5"] = c5
    co.barrier()
    if rank == 0:
        ndev = torch.cuda.device_count()
        if world > 1 and not args.no_scatter:  # (one visible GPU: the all-local rehearsal)
            try:
                out["peer_scatter"] = peer_scatter(D, stream, co.device or 0, ndev)
            except Exception as e:  # evidence only: never costs the bench line
                out["peer_scatter"] = {"error": str(e)[:300]}
    torch.cuda.synchronize()
    cpu = rank0_cpu_baseline(co, args, k, m, F, missing)
    if rank == 0:
        if cpu is not None:
            out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    co.barrier()
    co.close()


if __name__ == "__main__":
    main()
