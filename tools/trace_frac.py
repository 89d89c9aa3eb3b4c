#!/usr/bin/env python3
"""k_pull_chain's roofline fraction recomputed from a rocprofv3 kernel trace
of bench.py ("the rocprof-recomputed frac").

    python tools/trace_frac.py <run_kernel_trace.csv> <bytes_per_launch> <instrumented_launches>

bench.py's instrumented steps (blocking, after the timed region) are the
trace's last <instrumented_launches> dispatches: their mean duration is the
per-launch time bench.py's HIP events measure.  The pipelined steps before
them overlap consecutive windows, so a dispatch's
duration includes time it shares the GPU; for them the fraction is the
algorithmic bytes of all their dispatches over the union of the intervals
in which any of them ran."""
import csv
import sys

PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md


def main():
    path, bpl, n_inst = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if "k_pull_chain<false" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    inst = iv[-n_inst:]
    mean_us = sum(e - s for s, e in inst) / len(inst) / 1e3
    print(f"instrumented: {len(inst)} dispatches, mean {mean_us:.1f} us, "
          f"{bpl / (mean_us * 1e3):.0f} GB/s, frac {bpl / (mean_us * 1e3) / PEAK:.3f}")
    pipe = sorted(iv[:-n_inst])
    if pipe:
        busy, (cs, ce) = 0, pipe[0]
        for s, e in pipe[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        gbs = bpl * len(pipe) / busy
        print(f"pipelined: {len(pipe)} dispatches, union busy {busy / 1e3:.1f} us "
              f"({busy / 1e3 / len(pipe):.1f} us per launch), {gbs:.0f} GB/s, frac {gbs / PEAK:.3f}")


if __name__ == "__main__":
    main()
