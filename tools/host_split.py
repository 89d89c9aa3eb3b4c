#!/usr/bin/env python3
"""Where a pipelined step's wall time goes: host time inside ps_publish,
ps_run_async and ps_wait per step, against the GPU span of each window
(Stats.run_ms: init start to reduce end, stamped on the device).

  python tools/host_split.py [--workload cfg2] [--steps 300]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))

import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--staggered", type=int, default=0, help="start rounds uniform over 0..N (paced publishing)")
    args = ap.parse_args()
    wl = WL.CONFIGS[args.workload]()
    eng = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
    WL.build_engine_topics(eng, wl)
    starts = None
    if args.staggered:
        starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(args.staggered + 1)).astype(np.uint32)
    for _ in range(5):
        eng.publish(wl.msg_topics, starts)
        eng.run()
    for rep in range(args.reps):
        tp = tr = tw = 0
        run_ms = []
        t0 = time.perf_counter_ns()
        for i in range(args.steps):
            a = time.perf_counter_ns()
            eng.publish(wl.msg_topics, starts)
            b = time.perf_counter_ns()
            eng.run_async()
            c = time.perf_counter_ns()
            if i:
                run_ms.append(eng.wait().run_ms)
            d = time.perf_counter_ns()
            tp += b - a
            tr += c - b
            tw += d - c
        run_ms.append(eng.wait().run_ms)
        wall = (time.perf_counter_ns() - t0) / 1e3 / args.steps
        n = args.steps
        print(f"[host_split] {wl.name} rep {rep}: {wall:.1f} us/step; host per step: publish {tp / 1e3 / n:.1f} "
              f"run_async {tr / 1e3 / n:.1f} wait {tw / 1e3 / n:.1f} us; device span per window "
              f"p50 {np.median(run_ms) * 1e3:.1f} us, mean {np.mean(run_ms) * 1e3:.1f} us", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
