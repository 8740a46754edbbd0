#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (run_counter_collection.csv of one or more output directories)
per kernel: the mean of every counter over the kernel's dispatches (optionally only dispatches whose
grid size matches), plus derived shares (development tool, round 4).

  lds_active_share    SQ_LDS_IDX_ACTIVE / 256 CUs  /  (GRBM_GUI_ACTIVE / 8 XCDs)
  lds_conflict_share  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  valu_issue_share    SQ_INSTS_VALU x 4 cycles / 1024 SIMDs  /  (GRBM_GUI_ACTIVE / 8)
  wait_any_share      SQ_WAIT_ANY / SQ_WAVE_CYCLES          (waves parked on s_waitcnt / barrier)
  wait_inst_share     SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (issue stalls)
  active_inst_share   SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  valu_active_share   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
(GRBM_GUI_ACTIVE is summed over the 8 XCDs and the SQ counters over the 256 CUs, as the r03 PMC
summaries note; SQ_*_CYCLES are quad-cycles, consistently, so the shares are ratios of like units.)

usage: summarize_pmc.py OUT.json DIR [DIR ...] [--kernel SUBSTR] [--command TEXT]"""
import csv
import json
import sys


def main():
    args = sys.argv[1:]
    kernel, command = None, None
    if "--kernel" in args:
        i = args.index("--kernel")
        kernel = args[i + 1]
        del args[i:i + 2]
    if "--command" in args:
        i = args.index("--command")
        command = args[i + 1]
        del args[i:i + 2]
    out, dirs = args[0], args[1:]
    acc = {}  # kernel -> counter -> [values]
    meta = {}
    for d in dirs:
        with open(f"{d}/run_counter_collection.csv") as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if kernel and kernel not in name:
                    continue
                acc.setdefault(name, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
                meta.setdefault(name, {"vgpr": int(row["VGPR_Count"]), "sgpr": int(row["SGPR_Count"]),
                                       "lds_bytes": int(row["LDS_Block_Size"]),
                                       "scratch": int(row["Scratch_Size"]),
                                       "workgroup": int(row["Workgroup_Size"])})
    res = {"source": "rocprofv3 --pmc passes: " + " ".join(dirs), "command": command, "kernels": {}}
    for name, ctr in acc.items():
        m = {c: sum(v) / len(v) for c, v in ctr.items()}
        m["dispatches"] = max(len(v) for v in ctr.values())
        g = m.get("GRBM_GUI_ACTIVE")
        if g:
            per_xcd = g / 8
            if "SQ_LDS_IDX_ACTIVE" in m:
                m["lds_active_share"] = round(m["SQ_LDS_IDX_ACTIVE"] / 256 / per_xcd, 4)
            if "SQ_INSTS_VALU" in m:
                m["valu_issue_share"] = round(m["SQ_INSTS_VALU"] * 4 / 1024 / per_xcd, 4)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_conflict_share"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c, key in (("SQ_WAIT_ANY", "wait_any_share"), ("SQ_WAIT_INST_ANY", "wait_inst_share"),
                           ("SQ_ACTIVE_INST_ANY", "active_inst_share"),
                           ("SQ_ACTIVE_INST_VALU", "valu_active_share"),
                           ("SQ_WAIT_INST_LDS", "wait_inst_lds_share")):
                if c in m:
                    m[key] = round(m[c] / wc, 4)
        m.update(meta[name])
        res["kernels"][name] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in sorted(m.items())}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: {x: v[x] for x in v if x.endswith("share") or x in ("dispatches", "vgpr")}
                      for k, v in res["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
