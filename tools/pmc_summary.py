#!/usr/bin/env python3
"""Summarises rocprofv3 PMC csv files per kernel: dispatches, mean counter
value per dispatch, and HBM bytes per dispatch.  FETCH_SIZE / WRITE_SIZE are
in KiB (rocprofv3 derived counters).  gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE reads 1/2 of the bytes of wide (16 B/lane) coalesced
streaming reads; other widths are uncalibrated -- both raw and x2 are shown.

    python tools/pmc_summary.py gpurun_out/prof_r01
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    root = sys.argv[1]
    acc = load(root)
    out = {}
    for k, ctrs in sorted(acc.items()):
        d = {}
        for c, vals in ctrs.items():
            d[c] = {"dispatches": len(vals), "mean_per_dispatch": sum(vals) / len(vals),
                    "total": sum(vals)}
        if "FETCH_SIZE" in d:
            f = d["FETCH_SIZE"]["mean_per_dispatch"] * 1024
            d["hbm_read_bytes_per_dispatch_raw"] = f
            d["hbm_read_bytes_per_dispatch_x2"] = 2 * f
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes_per_dispatch"] = d["WRITE_SIZE"]["mean_per_dispatch"] * 1024
        out[k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
