"""Summarise rocprofv3 --pmc counter CSVs for the kernels whose name matches a pattern:
per counter, the mean over dispatches (plus the derived per-row / hit-rate figures for FFM).

    python scripts/pmc_summary.py <dir-with-counter_collection.csv files> [pattern] [rows_per_dispatch]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "ffm"
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 262144
    vals = defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(root, "**", "*.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "Counter_Name" not in r:
                break
            if pat not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {"kernel": r["Kernel_Name"][:100], "vgpr": r["VGPR_Count"], "lds": r["LDS_Block_Size"]}
    out = {"kernel": meta, "dispatches": {k: len(v) for k, v in vals.items()}}
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    out["mean_per_dispatch"] = {k: round(v, 1) for k, v in sorted(mean.items())}
    d = {}
    if "FETCH_SIZE" in mean:      # KB; gfx950 tallies 128-B requests at 64 B (MI355X_MICROARCH.md)
        d["fetch_KB_per_row_x2"] = round(2 * mean["FETCH_SIZE"] / rows, 2)
    if "WRITE_SIZE" in mean:
        d["write_KB_per_row"] = round(mean["WRITE_SIZE"] / rows, 2)
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        d["l2_hit_rate"] = round(mean["TCC_HIT_sum"] / max(1.0, mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"]), 3)
    if "SQ_WAIT_ANY" in mean and "SQ_WAVE_CYCLES" in mean:
        d["wait_any_frac"] = round(mean["SQ_WAIT_ANY"] / max(1.0, mean["SQ_WAVE_CYCLES"]), 3)
    if "SQ_ACTIVE_INST_ANY" in mean and "SQ_WAVE_CYCLES" in mean:
        d["active_inst_frac"] = round(mean["SQ_ACTIVE_INST_ANY"] / max(1.0, mean["SQ_WAVE_CYCLES"]), 3)
    if "SQ_INSTS_VMEM_RD" in mean:
        d["vmem_rd_wave_insts_per_row"] = round(mean["SQ_INSTS_VMEM_RD"] / rows, 2)
        d["vmem_wr_wave_insts_per_row"] = round(mean.get("SQ_INSTS_VMEM_WR", 0) / rows, 2)
        d["valu_wave_insts_per_row"] = round(mean.get("SQ_INSTS_VALU", 0) / rows, 1)
        d["lds_wave_insts_per_row"] = round(mean.get("SQ_INSTS_LDS", 0) / rows, 1)
    out["derived"] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
