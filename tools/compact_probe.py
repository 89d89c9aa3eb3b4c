#!/usr/bin/env python3
"""The compaction path alone (bench.py's general_path.compaction leg): cfg3
with start rounds uniform over 0..7, every window through k_expand
(PS_F_COMPACT).  Short enough to run under rocprofv3 --pmc passes.

    python tools/compact_probe.py [--steps 4] [--timed 2]

Prints one JSON line: pipelined ms/step, and from `timed` instrumented steps
k_expand's algorithmic bytes, device ms and GB/s per round."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--timed", type=int, default=2)
    ap.add_argument("--max-start", type=int, default=7)
    ap.add_argument("--no-check", action="store_true", help="skip the delivery checks (diagnostic builds)")
    args = ap.parse_args()
    wl = WL.CONFIGS[args.workload]()
    eng = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
    sizes = WL.build_engine_topics(eng, wl)
    expected = wl.expected_deliveries(sizes)
    starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(args.max_start + 1)).astype(np.uint32)
    eng.set_flags(eng.flags | PE.F_COMPACT)
    eng.publish(wl.msg_topics, starts)
    st = eng.run()
    assert args.no_check or st.deliveries == expected and st.expand_mode == PE.MODE_COMPACT, (st.deliveries, expected)
    t0 = time.perf_counter()
    tot = 0
    for i in range(args.steps):
        eng.publish(wl.msg_topics, starts)
        eng.run_async()
        if i:
            tot += eng.wait().deliveries
    tot += eng.wait().deliveries
    wall = time.perf_counter() - t0
    assert args.no_check or tot == expected * args.steps
    eng.set_time_kernels(True)
    b = ms = 0.0
    per_round = []
    for _ in range(args.timed):
        eng.publish(wl.msg_topics, starts)
        st = eng.run()
        d = st.as_dict()
        b += st.expand_bytes
        ms += st.expand_ms
        pr = [(int(x), float(y)) for x, y in zip(d["expand_bytes_per_round"], d["expand_ms_per_round"])]
        per_round = pr if not per_round else [(a + x, c + y) for (a, c), (x, y) in zip(per_round, pr)]
    eng.set_time_kernels(False)
    out = {"ms_per_step": wall * 1e3 / args.steps, "expand_ms_per_step": ms / max(1, args.timed),
           "expand_gbytes_per_step": b / max(1, args.timed) / 1e9, "expand_gbs": b / max(1e-12, ms * 1e-3) / 1e9 if ms else None,
           "launches": int(st.expand_launches), "rounds": int(st.rounds),
           "per_round": [[round(x / max(1, args.timed) / 1e6, 1), round(y / max(1, args.timed) * 1e3, 1),
                          round(x / max(1e-12, y * 1e-3) / 1e9, 0)] for x, y in per_round if x]}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
