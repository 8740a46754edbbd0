#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (run_counter_collection.csv of one or more output directories)
per CODE OBJECT and dispatch window, not per kernel name (development tool; round 5).

The run-time compiled bitsliced kernels all carry the name `ecamd_bs_kernel`, so one name covers
code objects of different shapes (C3's one-wave 4 KiB-tile form, C5's 16 KiB-tile 8-output form, the
crc variant ...).  Dispatches are therefore grouped by (name, workgroup size, VGPRs, SGPRs, LDS,
scratch) -- one group per code object -- and, within a group, optionally restricted to a window of
its dispatches in Dispatch_Id order (`--window A:B`, Python slice semantics over that group's
dispatches in each directory) and to a grid size (`--grid N`).  For every group the mean of every
counter is reported, plus derived shares:

  lds_active_share    SQ_LDS_IDX_ACTIVE / 256 CUs  /  (GRBM_GUI_ACTIVE / 8 XCDs)
  lds_conflict_share  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  valu_issue_share    SQ_INSTS_VALU x 4 cycles / 1024 SIMDs  /  (GRBM_GUI_ACTIVE / 8)
  wait_any_share      SQ_WAIT_ANY / SQ_WAVE_CYCLES          (waves parked on s_waitcnt / barrier)
  wait_inst_share     SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (issue stalls)
  active_inst_share   SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  valu_active_share   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  vmem_per_wave       SQ_INSTS_VMEM / SQ_WAVES
  waves_resident      SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) / 256 CUs   (mean waves per CU)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs and the SQ counters over the 256 CUs; SQ_*_CYCLES are
quad-cycles, consistently, so the shares are ratios of like units.)

usage: summarize_pmc.py OUT.json DIR [DIR ...] [--kernel SUBSTR] [--window A:B] [--grid N]
                        [--workgroup N] [--command TEXT]"""
import csv
import json
import sys


def _opt(args, name, conv=str):
    if name not in args:
        return None
    i = args.index(name)
    v = conv(args[i + 1])
    del args[i:i + 2]
    return v


def _window(text):
    a, b = text.split(":")
    return (int(a) if a else None, int(b) if b else None)


def main():
    args = sys.argv[1:]
    kernel = _opt(args, "--kernel")
    command = _opt(args, "--command")
    window = _opt(args, "--window", _window)
    grid = _opt(args, "--grid", int)
    wg = _opt(args, "--workgroup", int)
    out, dirs = args[0], args[1:]
    groups = {}  # code object -> counter -> [values]
    for d in dirs:
        per = {}  # code object -> dispatch id -> {counter: value}
        with open(f"{d}/run_counter_collection.csv") as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if kernel and kernel not in name:
                    continue
                if grid is not None and int(row["Grid_Size"]) != grid:
                    continue
                if wg is not None and int(row["Workgroup_Size"]) != wg:
                    continue
                key = (name, int(row["Workgroup_Size"]), int(row["VGPR_Count"]), int(row["SGPR_Count"]),
                       int(row["LDS_Block_Size"]), int(row["Scratch_Size"]))
                per.setdefault(key, {}).setdefault(int(row["Dispatch_Id"]), {})[row["Counter_Name"]] = \
                    float(row["Counter_Value"])
                per[key][int(row["Dispatch_Id"])]["_grid"] = float(row["Grid_Size"])
        for key, disp in per.items():
            ids = sorted(disp)
            if window:
                ids = ids[window[0]:window[1]]
            g = groups.setdefault(key, {"_ids": []})
            g["_ids"].extend(ids)
            for i in ids:
                for c, v in disp[i].items():
                    g.setdefault(c, []).append(v)
    res = {"source": "rocprofv3 --pmc passes: " + " ".join(dirs), "command": command,
           "filter": {"kernel": kernel, "window": window, "grid": grid, "workgroup": wg},
           "code_objects": []}
    for key, ctr in groups.items():
        name, wsize, vgpr, sgpr, lds, scratch = key
        ids = ctr.pop("_ids")
        m = {c: sum(v) / len(v) for c, v in ctr.items() if v}
        m["dispatches"] = len(ids)
        m["dispatch_ids"] = [min(ids), max(ids)] if ids else []
        m["grid"] = m.pop("_grid", None)
        gg = m.get("GRBM_GUI_ACTIVE")
        if gg:
            per_xcd = gg / 8
            if "SQ_LDS_IDX_ACTIVE" in m:
                m["lds_active_share"] = round(m["SQ_LDS_IDX_ACTIVE"] / 256 / per_xcd, 4)
            if "SQ_INSTS_VALU" in m:
                m["valu_issue_share"] = round(m["SQ_INSTS_VALU"] * 4 / 1024 / per_xcd, 4)
            if "SQ_WAVE_CYCLES" in m:
                m["waves_resident"] = round(m["SQ_WAVE_CYCLES"] / per_xcd / 256, 3)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_conflict_share"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
        if m.get("SQ_WAVES") and "SQ_INSTS_VMEM" in m:
            m["vmem_per_wave"] = round(m["SQ_INSTS_VMEM"] / m["SQ_WAVES"], 2)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c, k in (("SQ_WAIT_ANY", "wait_any_share"), ("SQ_WAIT_INST_ANY", "wait_inst_share"),
                         ("SQ_ACTIVE_INST_ANY", "active_inst_share"),
                         ("SQ_ACTIVE_INST_VALU", "valu_active_share"),
                         ("SQ_WAIT_INST_LDS", "wait_inst_lds_share")):
                if c in m:
                    m[k] = round(m[c] / wc, 4)
        m.update({"kernel": name, "workgroup": wsize, "vgpr": vgpr, "sgpr": sgpr, "lds_bytes": lds,
                  "scratch": scratch})
        res["code_objects"].append({k: (round(v, 4) if isinstance(v, float) else v) for k, v in sorted(m.items())})
    res["code_objects"].sort(key=lambda e: (e["kernel"], e["dispatch_ids"]))
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps([{x: e[x] for x in e if x.endswith("share") or x in
                       ("kernel", "dispatches", "vgpr", "workgroup", "grid", "waves_resident")}
                      for e in res["code_objects"]], indent=1))


if __name__ == "__main__":
    main()
