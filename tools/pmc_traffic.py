#!/usr/bin/env python3
"""Adds (or replaces) one entry of profiles/pmc_traffic.json (bench.py's
roofline.traffic) from the separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes
summarised by tools/pmc_summary.py.

    python tools/pmc_traffic.py <pmc_summary.json> <kernel> <workload> <round-tag> [<source note>]

HBM bytes per launch = 2 x FETCH_SIZE (gfx950: FETCH_SIZE counts half of the
bytes of wide coalesced reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both
averaged over every dispatch of the kernel's production instances (no hop
record: first template argument false) in the run, like bench.py's
algorithmic bytes per launch.  The summary is copied to profiles/<round-tag>/.
"""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "profiles", "pmc_traffic.json")


def main():
    summ_path, kernel, workload, rtag = sys.argv[1:5]
    note = sys.argv[5] if len(sys.argv) > 5 else f"bench.py --workload {workload.split('-')[0]}"
    summ = json.load(open(summ_path))
    # (full names: the production instances; names truncated by rocprofv3 -T:
    # the kernel itself -- a bench run launches no recording instance)
    names = [k for k in summ if (f"{kernel}<false" in k or k == kernel) and "hbm_write_bytes_per_dispatch" in summ[k]
             and "hbm_read_bytes_per_dispatch_x2" in summ[k]]
    if not names:
        sys.exit(f"no {kernel}<false ...> dispatches with both counters in {summ_path}")
    disp = sum(summ[k]["WRITE_SIZE"]["dispatches"] for k in names)
    rd = sum(summ[k]["hbm_read_bytes_per_dispatch_x2"] * summ[k]["WRITE_SIZE"]["dispatches"] for k in names) / disp
    wr = sum(summ[k]["hbm_write_bytes_per_dispatch"] * summ[k]["WRITE_SIZE"]["dispatches"] for k in names) / disp
    os.makedirs(os.path.join(REPO, "profiles", rtag), exist_ok=True)
    # (one file per kernel and workload: two kernels of one workload may come from different runs)
    dst = os.path.join("profiles", rtag, f"pmc_summary_{workload}_{kernel}.json")
    shutil.copy(summ_path, os.path.join(REPO, dst))
    entry = {"kernel": kernel, "workload": workload, "instances": names, "dispatches": disp,
             "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
             "traffic_bytes_per_launch": rd + wr,
             "source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of {note}; "
                       f"read = 2 x FETCH_SIZE (gfx950); {dst}"}
    try:
        d = json.load(open(OUT))
    except (OSError, ValueError):
        d = {}
    entries = [x for x in d.get("entries", []) if (x.get("kernel"), x.get("workload")) != (kernel, workload)]
    entries.append(entry)
    with open(OUT, "w") as fh:
        json.dump({"entries": entries}, fh, indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
