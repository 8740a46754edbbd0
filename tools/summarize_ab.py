#!/usr/bin/env python3
"""Summarise an interleaved A/B log (JSON lines, one per (round, case, variant)) into one small JSON
for profiles/: per case and variant the median, min and max of a metric over the rounds, variants
sorted best first.  The raw log stays in gpurun_out/ (VERDICT r05 #7).

usage: summarize_ab.py OUT.json LOG --case KEY[,KEY2] --variant KEY[,KEY2] --metric KEY --command TEXT
                       [--lower-is-better] [--note TEXT]"""
import argparse
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("log")
    ap.add_argument("--case", required=True)
    ap.add_argument("--variant", required=True, help="key, or comma-separated keys (first present wins)")
    ap.add_argument("--metric", required=True)
    ap.add_argument("--command", required=True)
    ap.add_argument("--lower-is-better", action="store_true")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    if not a.command.strip():
        raise SystemExit("--command must name the command that produced the log")
    vkeys = a.variant.split(",")
    table = {}
    for line in open(a.log):
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        if a.metric not in r or any(c not in r for c in a.case.split(",")):
            continue
        v = next((f"{k}={r[k]}" for k in vkeys if k in r), None)
        if v is None:
            continue
        table.setdefault("/".join(str(r[c]) for c in a.case.split(",")), {}).setdefault(v, []).append(r[a.metric])
    out = {"source": a.log, "command": a.command, "metric": a.metric, "note": a.note, "cases": {}}
    for case, vs in table.items():
        rows = [{"variant": v, "median": round(statistics.median(x), 4), "min": min(x), "max": max(x), "n": len(x)}
                for v, x in vs.items()]
        rows.sort(key=lambda r: r["median"], reverse=not a.lower_is_better)
        out["cases"][case] = rows
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    for case, rows in out["cases"].items():
        print(case, [(r["variant"], r["median"]) for r in rows[:4]])


if __name__ == "__main__":
    main()
