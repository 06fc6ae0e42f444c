"""Counter + kernel-time report for one ``scripts/gpu_r3k.sh`` target directory.

    python scripts/pmc_report.py gpurun_out/pmc_gbdt hist_kernel level_finalize hist_sibling

For each kernel-name pattern: dispatches, mean duration (from the separate
``--kernel-trace --stats`` run), the mean of every counter per dispatch, and derived figures —
HBM-side bytes per dispatch and achieved TB/s (total bytes / total kernel time), L2 hit rate,
wait / active fractions, LDS bank-conflict share.  FETCH_SIZE / WRITE_SIZE are KB; gfx950
tallies a 128-B request at 64 B in FETCH_SIZE (MI355X_MICROARCH.md), so the fetch figure is
also given doubled (an upper bound; the true value lies between the two).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def counters(root, pat):
    vals = defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {"kernel": r["Kernel_Name"].split("(")[0][:90], "vgpr": r.get("VGPR_Count"),
                    "lds_bytes": r.get("LDS_Block_Size"), "grid": r.get("Grid_Size"),
                    "workgroup": r.get("Workgroup_Size")}
    return meta, vals


def durations(root, pat):
    calls, tot = 0, 0.0
    for f in glob.glob(os.path.join(root, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Name"]:
                calls += int(r["Calls"])
                tot += float(r["TotalDurationNs"])
    return calls, tot


def report(root, pat):
    meta, vals = counters(root, pat)
    calls, tot_ns = durations(root, pat)
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"pattern": pat, "kernel": meta, "dispatches_traced": calls,
           "mean_us": round(tot_ns / calls / 1e3, 2) if calls else None,
           "counters_mean_per_dispatch": {k: round(v, 1) for k, v in sorted(mean.items())}}
    d = {}
    if calls and "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        ns = tot_ns / calls
        f_kb, w_kb = mean["FETCH_SIZE"], mean["WRITE_SIZE"]
        d["fetch_MB_per_dispatch"] = round(f_kb / 1024, 3)
        d["write_MB_per_dispatch"] = round(w_kb / 1024, 3)
        d["achieved_TBps"] = round((f_kb + w_kb) * 1024 / ns / 1e3, 3)
        d["achieved_TBps_fetch_x2"] = round((2 * f_kb + w_kb) * 1024 / ns / 1e3, 3)
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        d["l2_hit_rate"] = round(mean["TCC_HIT_sum"] / max(1.0, mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"]), 3)
    if "SQ_WAVE_CYCLES" in mean:
        wc = max(1.0, mean["SQ_WAVE_CYCLES"])
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in mean:
                d[k.lower().replace("sq_", "") + "_frac"] = round(mean[k] / wc, 3)
    if "SQ_LDS_BANK_CONFLICT" in mean and "SQ_INSTS_LDS" in mean:
        d["lds_bank_conflict_cycles_per_lds_inst"] = round(mean["SQ_LDS_BANK_CONFLICT"] / max(1.0, mean["SQ_INSTS_LDS"]), 3)
    if "SQ_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
        d["sq_busy_frac"] = round(mean["SQ_BUSY_CYCLES"] / max(1.0, mean["GRBM_GUI_ACTIVE"]), 3)
    out["derived"] = d
    return out


if __name__ == "__main__":
    root = sys.argv[1]
    print(json.dumps([report(root, p) for p in sys.argv[2:]], indent=1))
