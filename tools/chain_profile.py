#!/usr/bin/env python3
"""Per-wave profile of the k_pull_chain launches.

    python tools/chain_profile.py [--workload cfg3] [--steps 3] [--out gpurun_out/chain_prof.bin]

Runs blocking steps of the workload with PSAMD_CHAIN_PROFILE set (the engine
records, per chain chunk, s_memrealtime at the wave's start and end, the row
words it wrote, and its CU / XCC), then reports per launch: span, ramp, tail
(last wave start -> launch end), mean / peak concurrency, the wave-duration
distribution, a duration ~ a + b * words fit (a = fixed per-wave cost), and the
write rate per XCC.  `--analyze FILE` re-reads an existing record."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

MAGIC = 0x50524F4643484149
TICK_US = 0.01  # s_memrealtime: 100 MHz


def parse(path: str):
    """Windows of the record: [(launches[(round, len, lo, gsplit, hi)], chunks[n, 8])]."""
    raw = np.fromfile(path, dtype=np.uint64)
    out, i = [], 0
    while i < raw.size:
        assert int(raw[i]) == MAGIC, f"bad record at word {i}"
        nl = int(raw[i + 1])
        i += 2
        launches = [tuple(int(x) for x in raw[i + 5 * k:i + 5 * k + 5]) for k in range(nl)]
        i += 5 * nl
        nc = int(raw[i])
        i += 1
        chunks = raw[i:i + 8 * nc].reshape(nc, 8)
        i += 8 * nc
        out.append((launches, chunks))
    return out


def launch_report(rnd, ln, ch):
    t0, t1, words = ch[:, 0].astype(np.int64), ch[:, 1].astype(np.int64), ch[:, 2].astype(np.float64)
    xcc = (ch[:, 3] >> np.uint64(32)).astype(np.int64) & 0xF
    direct = ((ch[:, 3] >> np.uint64(40)) & np.uint64(1)).astype(bool)
    base = t0.min()
    s, e = (t0 - base) * TICK_US, (t1 - base) * TICK_US
    span = float(e.max())
    dur = e - s
    # concurrency over time (sweep)
    ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    peak = int(conc.max())
    # time-weighted: fraction of the span below half of the peak
    dt = np.diff(ev[:, 0], append=ev[-1, 0])
    low = float(dt[conc < peak / 2].sum())
    ramp = float(ev[np.argmax(conc >= 0.9 * peak), 0])
    last_start = float(s.max())
    A = np.stack([np.ones_like(words), words], 1)
    coef, *_ = np.linalg.lstsq(A, dur, rcond=None)
    per_xcc = {}
    for x in np.unique(xcc):
        m = xcc == x
        per_xcc[int(x)] = {"waves": int(m.sum()), "GB": round(float(words[m].sum()) * 8e-9, 3),
                           "end_us": round(float(e[m].max()), 1)}
    bytes_w = float(words.sum()) * 8
    return {
        "round": rnd, "rounds": ln, "chunks": int(ch.shape[0]), "span_us": round(span, 1),
        "row_GB": round(bytes_w * 1e-9, 3), "write_TBs": round(bytes_w / max(span, 1e-9) * 1e-6, 2),
        "peak_waves": peak, "mean_waves": round(float(dur.sum()) / max(span, 1e-9), 1),
        "ramp_to_90pct_us": round(ramp, 1), "last_start_us": round(last_start, 1),
        "tail_us": round(span - last_start, 1), "below_half_peak_us": round(low, 1),
        "dur_us_p10_p50_p90_max": [round(float(np.percentile(dur, q)), 1) for q in (10, 50, 90, 100)],
        "words_p10_p50_p90_max": [int(np.percentile(words, q)) for q in (10, 50, 90, 100)],
        "fit_dur_us": {"fixed": round(float(coef[0]), 2), "per_kword": round(float(coef[1]) * 1e3, 3)},
        "per_xcc": per_xcc,
        "direct_level0": {"waves": int(direct.sum()), "words": int(words[direct].sum()),
                          "dur_us_p50": round(float(np.median(dur[direct])), 1) if direct.any() else None},
    }


def analyze(path: str):
    wins = parse(path)
    rep = []
    for launches, chunks in wins:
        win = []
        for (rnd, ln, lo, gs, hi) in launches:
            if hi > lo:
                win.append(launch_report(rnd, ln, chunks[lo:hi]))
        rep.append(win)
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "chain_prof.bin"))
    ap.add_argument("--analyze", default=None)
    args = ap.parse_args()
    if args.analyze:
        print(json.dumps(analyze(args.analyze), indent=1))
        return
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    if os.path.exists(args.out):
        os.remove(args.out)
    import psengine as PE
    from psengine import workloads as WL

    wl = WL.CONFIGS[args.workload]()
    os.environ["PSAMD_CHAIN_PROFILE"] = args.out
    prof = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)  # (read at creation)
    del os.environ["PSAMD_CHAIN_PROFILE"]
    WL.build_engine_topics(prof, wl)
    for _ in range(args.warmup):
        prof.publish(wl.msg_topics)
        prof.run()
    if os.path.exists(args.out):
        os.remove(args.out)
    for _ in range(args.steps):
        prof.publish(wl.msg_topics)
        st = prof.run()
        print(f"step: run_ms {st.run_ms:.3f}", file=sys.stderr)
    prof.close()
    rep = analyze(args.out)
    print(json.dumps({"workload": args.workload, "windows": rep}, indent=1))


if __name__ == "__main__":
    main()
