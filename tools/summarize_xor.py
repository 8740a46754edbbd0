#!/usr/bin/env python3
"""Summarise the rocprofv3 runs of tools/gpu_prof_xor.sh (tools/xor_prof.py under --kernel-trace,
then --pmc FETCH_SIZE, then --pmc WRITE_SIZE) into profiles/<round>_xor_summary.json.

xor_prof.py runs, per shape, 2 + reps encode passes then 2 + reps decode passes; a pass may be
several launches of xor_stream_kernel<KG> (the launch split, ecamd_device.hip launch_xor), so the
launches are grouped into passes by count.  Per shape and op: pass time (avg over the `reps`
steady passes), algorithmic bytes (encode: (k + m) fragments per stripe), fraction of 8 TB/s, and
HBM bytes per pass from the PMC passes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction).

usage: summarize_xor.py <round> [--reps 10]"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def rows(tag, counter=None):
    p = glob.glob(os.path.join(ROOT, "gpurun_out", f"prof_{tag}_xor", "**",
                               "*counter_collection.csv" if counter else "*kernel_trace.csv"), recursive=True)
    out = []
    for r in csv.DictReader(open(p[0])):
        if counter and r["Counter_Name"] != counter:
            continue
        v = float(r["Counter_Value"]) if counter else int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], v))
    out.sort()
    return [x for x in out if "xor_stream_kernel" in x[1]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import xor_prof
    trace = rows("trace")
    fetch = rows("fetch", "FETCH_SIZE")
    write = rows("write", "WRITE_SIZE")
    out = {"round": args.round, "command": "python3 tools/xor_prof.py (tools/gpu_prof_xor.sh)", "shapes": []}
    pos = 0
    passes_per_op = 2 + args.reps
    for k, m, hd, F, S, lost in xor_prof.SHAPES:
        kern = trace[pos][1]
        n = 0
        while pos + n < len(trace) and trace[pos + n][1] == kern:
            n += 1
        per = n // (2 * passes_per_op)  # launches per pass
        rec = {"code": [k, m, hd], "fragment_bytes": F, "stripes": S, "kernel": kern,
               "launches_per_pass": per}
        for i, op in enumerate(("encode", "decode")):
            base = pos + i * passes_per_op * per
            steady = range(base + 2 * per, base + passes_per_op * per, per)
            pt = [sum(trace[j][2] for j in range(b, b + per)) for b in steady]
            hb = [sum(fetch[j][2] * 2048 + write[j][2] * 1024 for j in range(b, b + per)) for b in steady]
            d = {"pass_avg_ns": round(statistics.mean(pt), 1), "pass_min_ns": min(pt),
                 "hbm_bytes_per_pass": round(statistics.mean(hb)), "passes": len(pt)}
            if op == "encode":
                algo = S * (k + m) * F
                d.update({"algorithmic_bytes": algo, "achieved_GBps": round(algo / d["pass_avg_ns"], 1),
                          "frac": round(algo / d["pass_avg_ns"] / 8000, 4),
                          "traffic_over_algorithmic": round(d["hbm_bytes_per_pass"] / algo, 4)})
            else:
                d["missing"] = lost
            rec[op] = d
        out["shapes"].append(rec)
        pos += 2 * passes_per_op * per
    dst = os.path.join(ROOT, "profiles", f"{args.round}_xor_summary.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
