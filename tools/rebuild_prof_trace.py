#!/usr/bin/env python3
"""Kernel-trace table of tools/rebuild_prof.py (rocprofv3 --kernel-trace of it): the `ecamd_bs_kernel`
dispatches in dispatch order are 1 + SETTLE encodes, (1 + reps) single-destination reconstructs per
destination 0..13, (1 + reps) x 4 decode_multi launches (grouped), the same interleaved -- for multi_streams 1, 2, 4 -- (1 + reps)
strided decodes.  Per case: the first call's duration and the steady calls' mean (decode_multi: the
span from its first launch's start to its fourth launch's end), as a fraction of 8 TB/s of the
algorithmic bytes.  Refuses a trace whose bitsliced dispatch count differs from that plan (a map
served by the LDS tables would shift every window).

usage: rebuild_prof_trace.py TRACE_DIR OUT.json --command TEXT [--reps 20]"""
import argparse
import csv
import glob
import json
import os
import statistics

K, M, F, S = 10, 4, 1 << 20, 256
SETTLE = 60


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("out")
    ap.add_argument("--command", required=True)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    path = sorted(glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    bs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "ecamd_bs_kernel" in r["Kernel_Name"]]
    n = 1 + a.reps
    plan = [("encode", 1 + SETTLE, 1, S * (K + M) * F)]
    plan += [(f"reconstruct_{d}", n, 1, S * (K + 1) * F) for d in range(K + M)]
    for sfx in ("", "_streams2", "_streams4"):
        plan += [("decode_multi_4patterns" + sfx, n, 4, S * (K + 4) * F),
                 ("decode_multi_4patterns_interleaved" + sfx, n, 4, S * (K + 4) * F)]
    plan += [("decode_strided_0123", n, 1, S * (K + 4) * F)]
    want = sum(c * per for _, c, per, _ in plan)
    if len(bs) != want:
        raise SystemExit(f"{len(bs)} bitsliced dispatches, the plan has {want}: some call ran on the tables")
    out = {"source": path, "command": a.command, "reps": a.reps, "cases": {}}
    i = 0
    for name, calls, per, algo in plan:
        spans = []
        for _ in range(calls):
            grp = bs[i:i + per]
            i += per
            spans.append(max(e for _, e in grp) - min(b for b, _ in grp))  # launches may overlap
        steady = spans[1:] if name != "encode" else spans[-20:]
        mean = statistics.mean(steady)
        out["cases"][name] = {"first_call_ns": spans[0], "steady_mean_ns": round(mean, 1), "calls": len(steady),
                              "launches_per_call": per, "algo_bytes": algo,
                              "first_call_frac": round(algo / spans[0] / 8000, 4),
                              "steady_frac": round(algo / mean / 8000, 4)}
    rec = [v["steady_frac"] for k, v in out["cases"].items() if k.startswith("reconstruct_")]
    out["reconstruct_steady_frac_min"] = min(rec)
    out["reconstruct_steady_frac_mean"] = round(statistics.mean(rec), 4)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    for k, v in out["cases"].items():
        print(k, v["first_call_frac"], v["steady_frac"])


if __name__ == "__main__":
    main()
