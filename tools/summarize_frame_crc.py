#!/usr/bin/env python3
"""Summarise tools/gpu_prof_frame_crc.sh (rocprofv3 of tools/frame_crc_prof.py) into
profiles/<round>_framecrc_summary.json: per path (the bitsliced crc variant `ecamd_bs_kernel`,
then the LDS-table `gf16_frame_crc_kernel`), the steady launches (the last `reps` of each: 5
warm-up encodes come first), their average duration, the finalize kernel beside them, HBM bytes
per launch from the FETCH_SIZE / WRITE_SIZE passes (x2 FETCH correction on gfx950) and the
fraction of 8 TB/s of the algorithmic bytes (10 MiB read + 14 MiB written per C3 stripe).

usage: summarize_frame_crc.py <round> [--reps 20]"""
import argparse
import csv
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(tag, counter=None):
    pat = "*counter_collection.csv" if counter else "*kernel_trace.csv"
    p = glob.glob(os.path.join(ROOT, "gpurun_out", f"prof_{tag}_framecrc", "**", pat), recursive=True)[0]
    out = []
    for r in csv.DictReader(open(p)):
        if counter and r["Counter_Name"] != counter:
            continue
        v = float(r["Counter_Value"]) if counter else int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], v))
    out.sort()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    algo = 256 * (10 + 14) * (1 << 20)
    trace, fetch, write = load("trace"), load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
    out = {"round": args.round, "command": "python3 tools/frame_crc_prof.py (tools/gpu_prof_frame_crc.sh)",
           "algorithmic_bytes_per_encode": algo, "paths": {}}
    for path, kern in (("bitsliced_crc", "ecamd_bs_kernel"), ("lds_fused", "gf16_frame_crc_kernel")):
        def pick(rows):
            sel = [x for x in rows if kern in x[1]]
            return sel[-args.reps:]
        main_t = pick(trace)
        ids = [x[0] for x in main_t]
        fin = [x for x in trace if "crc_finalize_kernel" in x[1] and ids[0] < x[0] <= ids[-1] + 1]
        avg = statistics.mean(x[2] for x in main_t)
        favg = statistics.mean(x[2] for x in fin) if fin else 0.0
        f, w = pick(fetch), pick(write)
        hbm = statistics.mean(a[2] * 2048 + b[2] * 1024 for a, b in zip(f, w))
        out["paths"][path] = {
            "kernel": kern, "launches": len(main_t), "avg_ns": round(avg, 1),
            "min_ns": min(x[2] for x in main_t), "finalize_avg_ns": round(favg, 1),
            "frac_kernel": round(algo / avg / 8000, 4),
            "frac_with_finalize": round(algo / (avg + favg) / 8000, 4),
            "hbm_bytes_per_launch": round(hbm), "traffic_over_algorithmic": round(hbm / algo, 4)}
    dst = os.path.join(ROOT, "profiles", f"{args.round}_framecrc_summary.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
