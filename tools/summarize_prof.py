#!/usr/bin/env python3
"""Summarise rocprofv3 output of tools/gpu_prof.sh into profiles/<round>_<cfg>_summary.json.

Per kernel: launch count and duration statistics from the kernel trace (per-dispatch start / end
timestamps), plus -- for the bench's dominant kernel -- the same statistics over the TIMED steps
only: the bench launches it `--pre` times before the settle steps (2: an encode and a decode, which
also compile any bitsliced kernel the config needs), twice per settle step (`--settle`, bench.py's
untimed clock ramp-up), twice per warm-up step, twice per timed step,
then twice per untimed pass-split step (bench.PASS_SPLIT_STEPS) and for the untimed mixed-pattern
decodes; the timed launches are dispatches
[pre + 2*(settle + warmup), pre + 2*(settle + warmup) + 2*steps) of that kernel in dispatch order
(times --per-pass when a pass is several launches).  bench.py reads
"timed_avg_ns" to put the trace-derived roofline fraction beside its HIP-event one.

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB, collected in separate passes; on gfx950 FETCH_SIZE reports half the bytes
of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16 B/lane streaming
stores.  Counter values are averaged over the same timed dispatches when the kernel is the
dominant one, else over all its dispatches.

usage: summarize_prof.py <cfg> <round> [--kernel NAME --warmup W --steps K --stripes S --bench LOG]
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find_csv(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    return hits[0] if hits else None


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def trace_rows(path):
    """(kernel, dispatch id, duration ns) per dispatch, in dispatch order."""
    out = []
    for r in csv.DictReader(open(path)):
        name = col(r, "Kernel_Name", "KernelName")
        start = int(col(r, "Start_Timestamp", "BeginNs"))
        end = int(col(r, "End_Timestamp", "EndNs"))
        did = int(col(r, "Dispatch_Id", "Index", "Correlation_Id"))
        out.append((name, did, end - start))
    out.sort(key=lambda x: x[1])
    return out


def stats(durs):
    return {"calls": len(durs), "avg_ns": round(statistics.mean(durs), 1),
            "min_ns": min(durs), "max_ns": max(durs),
            "median_ns": round(statistics.median(durs), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("round")
    ap.add_argument("--kernel", default="", help="dominant kernel (name prefix)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle", type=int, default=60, help="bench.py's untimed settle steps")
    ap.add_argument("--pre", type=int, default=2, help="launches of the kernel before the warm-up")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--per-pass", type=int, default=1,
                    help="dispatches of the dominant kernel per encode / decode pass (a long pass "
                         "runs as several launches, ecamd_device.hip launch_stream_pass)")
    ap.add_argument("--stripes", type=int, default=256)
    ap.add_argument("--bench", default="", help="bench JSON log of the profiled command")
    ap.add_argument("--command", default="")
    ap.add_argument("--algo-bytes", type=float, default=0,
                    help="algorithmic bytes per launch of the windows' kernels (frac vs 8 TB/s)")
    ap.add_argument("--window", action="append", default=[],
                    help="label:kernel-substring:first:count -- stats over dispatches [first, "
                         "first+count) of that kernel in dispatch order (repeatable)")
    args = ap.parse_args()
    if not args.command.strip():  # bench.py quotes a summary only for the command it names
        ap.error("--command: the exact profiled command line is required")
    g = os.path.join(ROOT, "gpurun_out")
    pre = f"prof_{{}}_{args.cfg}"
    out = {"config": args.cfg, "round": args.round, "command": args.command,
           "stripes_per_gpu": args.stripes, "warmup": args.warmup, "steps": args.steps,
           "kernels": {}}

    tpath = find_csv(os.path.join(g, pre.format("trace")), "kernel_trace.csv")
    win_pmc = None
    rows = trace_rows(tpath)
    by = defaultdict(list)
    for name, did, dur in rows:
        by[name].append((did, dur))
    timed_ids = set()
    for name, lst in by.items():
        d = stats([x[1] for x in lst])
        if args.kernel and args.kernel in name:
            P = args.per_pass
            lo = (args.pre + 2 * (args.settle + args.warmup)) * P
            timed = lst[lo:lo + 2 * args.steps * P]
            timed_ids = {x[0] for x in timed}
            t = stats([x[1] for x in timed])
            passes = [sum(x[1] for x in timed[i:i + P]) for i in range(0, len(timed), P)]
            d.update({"timed_calls": t["calls"], "timed_avg_ns": t["avg_ns"],
                      "timed_min_ns": t["min_ns"], "timed_max_ns": t["max_ns"],
                      "timed_median_ns": t["median_ns"],
                      "dispatches_per_pass": P,
                      "timed_pass_avg_ns": round(statistics.mean(passes), 1) if passes else None,
                      "first_dispatch_ns": lst[0][1],
                      "note": f"timed = dispatches {lo}..{lo + 2 * args.steps * P - 1} of this kernel "
                              f"({P} per pass)"})
        out["kernels"][name] = d

    # labelled windows (e.g. the steady-state launches of each C5 operation)
    windows = []
    for spec in args.window:
        label, sub, first, count = spec.split(":")
        windows.append((label, sub, int(first), int(count)))
    out["windows"] = {}
    for label, sub, first, count in windows:
        for name, lst in by.items():
            if sub in name:
                sel = lst[first:first + count]
                w = stats([x[1] for x in sel])
                w["kernel"] = name
                w["dispatch_ids"] = [sel[0][0], sel[-1][0]] if sel else []
                if args.algo_bytes and sel:
                    w["algo_bytes"] = args.algo_bytes
                    w["achieved_GBps"] = round(args.algo_bytes / w["avg_ns"], 1)
                    w["frac"] = round(args.algo_bytes / w["avg_ns"] / 8000, 4)
                out["windows"][label] = w
    win_pmc = {label: [] for label, *_ in windows}

    for tag in ("fetch", "write", "lds", "stall"):
        p = find_csv(os.path.join(g, pre.format(tag)), "counter_collection.csv")
        if not p:
            continue
        per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [(dispatch, value)]
        for r in csv.DictReader(open(p)):
            per[col(r, "Kernel_Name")][col(r, "Counter_Name")].append(
                (int(col(r, "Dispatch_Id")), float(col(r, "Counter_Value"))))
        for label, sub, first, count in windows:
            for kern, cs in per.items():
                if sub not in kern:
                    continue
                w = out["windows"].setdefault(label, {})
                for cname, vals in cs.items():
                    vv = sorted(vals)[first:first + count]
                    if vv:
                        w[cname] = statistics.mean(v for _, v in vv)
        for kern, cs in per.items():
            d = out["kernels"].setdefault(kern, {})
            for cname, vals in cs.items():
                # PMC runs are separate processes: use the same position-based timed window
                vals.sort()
                if args.kernel and args.kernel in kern:
                    lo = (args.pre + 2 * (args.settle + args.warmup)) * args.per_pass
                    sel = [v for _, v in vals[lo:lo + 2 * args.steps * args.per_pass]] or [v for _, v in vals]
                else:
                    sel = [v for _, v in vals]
                d[cname] = statistics.mean(sel)
    for kern, d in list(out["kernels"].items()) + list(out["windows"].items()):
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            rd = d["FETCH_SIZE"] * 1024 * 2   # gfx950: FETCH_SIZE = half the streamed bytes
            wr = d["WRITE_SIZE"] * 1024
            d["hbm_read_bytes"] = rd
            d["hbm_write_bytes"] = wr
            d["hbm_bytes_per_launch"] = rd + wr
            ns = d.get("timed_avg_ns") or d.get("avg_ns")
            if ns:
                d["hbm_GBps"] = round((rd + wr) / ns, 1)
        if d.get("SQ_WAVE_CYCLES"):  # shares of wave time: parked on s_waitcnt / issue-stalled / issuing
            for c, k in (("SQ_WAIT_ANY", "wait_any_share"), ("SQ_WAIT_INST_ANY", "wait_inst_share"),
                         ("SQ_ACTIVE_INST_ANY", "active_inst_share"), ("SQ_ACTIVE_INST_VALU", "active_valu_share")):
                if c in d:
                    d[k] = round(d[c] / d["SQ_WAVE_CYCLES"], 4)
        if "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_ratio"] = round(d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"], 4)
    if args.bench and os.path.exists(args.bench):
        for line in open(args.bench):
            line = line.strip()
            if line.startswith("{"):
                try:
                    b = json.loads(line)
                    out["ms_per_step"] = b.get("ms_per_step")
                    out["bench_value"] = b.get("value")
                except json.JSONDecodeError:
                    pass
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    dst = os.path.join(ROOT, "profiles", f"{args.round}_{args.cfg}_summary.json")
    json.dump(out, open(dst, "w"), indent=1)
    spath = find_csv(os.path.join(g, pre.format("trace")), "kernel_stats.csv")
    if spath:
        shutil.copy(spath, os.path.join(ROOT, "profiles", f"{args.round}_{args.cfg}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
