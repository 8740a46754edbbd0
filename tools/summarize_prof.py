#!/usr/bin/env python3
"""Summarise rocprofv3 CSVs from gpurun_out/prof_*_<cfg>/ into profiles/<round>_<cfg>_*.

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB, collected in separate passes; on gfx950 FETCH_SIZE reports exactly half the
bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16 B/lane
streaming stores.
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main(cfg, rnd="r01"):
    g = os.path.join(ROOT, "gpurun_out")
    out = {"config": cfg, "round": rnd, "kernels": {}}
    # cfg "frame": tools/gpu_prof_frame.sh (framing / CRC kernels), dirs gpurun_out/fprof_<tag>
    d_of = (lambda tag: f"fprof_{tag}") if cfg == "frame" else (lambda tag: f"prof_{tag}_{cfg}")
    stats = os.path.join(g, d_of("trace"), "run_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        out["kernels"][r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                     "pct": float(r["Percentage"])}
    for tag in ("fetch", "write", "lds"):
        p = os.path.join(g, d_of(tag), "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for (kern, cname), vals in counters(p).items():
            d = out["kernels"].setdefault(kern, {})
            d[cname] = statistics.mean(vals)
    for kern, d in out["kernels"].items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            rd = d["FETCH_SIZE"] * 1024 * 2   # gfx950: FETCH_SIZE = half the streamed bytes
            wr = d["WRITE_SIZE"] * 1024
            d["hbm_read_bytes"] = rd
            d["hbm_write_bytes"] = wr
            d["hbm_bytes_per_launch"] = rd + wr
            if d.get("avg_ns"):
                d["hbm_GBps"] = round((rd + wr) / d["avg_ns"], 1)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    dst = os.path.join(ROOT, "profiles", f"{rnd}_{cfg}_summary.json")
    json.dump(out, open(dst, "w"), indent=1)
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{rnd}_{cfg}_kernel_stats.csv"))
    blog = os.path.join(g, f"bench_full_{cfg}.log")
    if os.path.exists(blog):
        shutil.copy(blog, os.path.join(ROOT, "profiles", f"{rnd}_{cfg}_bench.log"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c3", sys.argv[2] if len(sys.argv) > 2 else "r01")
