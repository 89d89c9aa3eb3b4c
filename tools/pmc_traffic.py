#!/usr/bin/env python3
"""Writes profiles/pmc_traffic.json (bench.py's roofline.traffic) from the
separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes of a gpu_check.sh run.

    python tools/pmc_traffic.py gpurun_out/<tag> <kernel> <workload> <round-tag>

HBM bytes per launch = 2 x FETCH_SIZE (gfx950: FETCH_SIZE counts half of the
bytes of wide coalesced reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both
averaged over every dispatch of the kernel's production instance in the run,
like bench.py's algorithmic bytes per launch.  The summary of the passes is
copied to profiles/<round-tag>/ next to it.
"""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    run_dir, kernel, workload, rtag = sys.argv[1:5]
    summ = json.load(open(os.path.join(run_dir, "pmc_summary.json")))
    # production instances: no hop record (first template argument false);
    # the cache-policy variants (plain / nt stores) are one kernel to the
    # roofline, so their traffic is averaged over all of their dispatches
    # (k_pull: its top-levels launch k_pull_top is one of the launches too)
    names = [k for k in summ if (f"{kernel}<false" in k or f"{kernel}_top<false" in k)
             and "hbm_write_bytes_per_dispatch" in summ[k]]
    if not names:
        sys.exit(f"no {kernel}<false ...> dispatches with both counters in {run_dir}")
    disp = sum(summ[k]["WRITE_SIZE"]["dispatches"] for k in names)
    rd = sum(summ[k]["hbm_read_bytes_per_dispatch_x2"] * summ[k]["WRITE_SIZE"]["dispatches"] for k in names) / disp
    wr = sum(summ[k]["hbm_write_bytes_per_dispatch"] * summ[k]["WRITE_SIZE"]["dispatches"] for k in names) / disp
    os.makedirs(os.path.join(REPO, "profiles", rtag), exist_ok=True)
    dst = os.path.join("profiles", rtag, "pmc_summary.json")
    shutil.copy(os.path.join(run_dir, "pmc_summary.json"), os.path.join(REPO, dst))
    out = {"kernel": kernel, "workload": workload, "instances": names,
           "dispatches": disp,
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
           "traffic_bytes_per_launch": rd + wr,
           "source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of "
                     f"bench.py --workload {workload}; read = 2 x FETCH_SIZE (gfx950); {dst}"}
    with open(os.path.join(REPO, "profiles", "pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
