#!/usr/bin/env python3
"""Multi-rank path at bench scale on ONE GPU: `world` engines in threads with
the loopback transport (device copies in place of RCCL), weak scaling (world x
the messages).  Checks the job's deliveries against the single engine and
prints per-step times next to `world` x the single-rank step -- an overhead
probe of the exchange path, not a scaling measurement.

    python tools/loopback_bench.py --world 4 --workload cfg4 --scale 0.25 --partition peer
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=4)
ap.add_argument("--workload", default="cfg4")
ap.add_argument("--scale", type=float, default=0.25)
ap.add_argument("--partition", default="peer", choices=["peer", "subtree"])
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--mode", default="zc", choices=["zc", "copy", "inplace"],
                help="zero-copy records (default), records copied (PS_DIST_F_COPY), or rows read in place "
                     "(PS_DIST_F_INPLACE)")
ap.add_argument("--staggered", action="store_true",
                help="start rounds uniform over 0..7 (paced publishing: start groups), both legs")
args = ap.parse_args()
part = PE.PART_PEER if args.partition == "peer" else PE.PART_SUBTREE
wl = WL.CONFIGS[args.workload]() if args.scale == 1.0 else WL.scaled(args.workload, args.scale)
base_msgs = wl.msg_topics.copy()
base_starts = ((WL.stream(wl.seed ^ 0x57A6, np.arange(base_msgs.shape[0])) % np.uint64(8)).astype(np.uint32)
               if args.staggered else None)

# the single-rank step on the same topology and per-rank message count
t0 = time.perf_counter()
one = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, msg_window=1 << 20)
sizes = WL.build_engine_topics(one, wl)
print(f"[loopback] {wl.name} x{args.scale}: {wl.n_peers} peers, setup {time.perf_counter() - t0:.1f}s", flush=True)
exp1 = wl.expected_deliveries(sizes)
one_ms = []
for step in range(args.steps + 1):
    one.publish(base_msgs, base_starts)
    t0 = time.perf_counter()
    st = one.run()
    one_ms.append((time.perf_counter() - t0) * 1e3)
    assert st.deliveries == exp1, (st.deliveries, exp1)
d1 = one.seen_digest()
one.close()
single = float(np.median(one_ms[1:]))

msgs = np.tile(base_msgs, args.world)
starts = None if base_starts is None else np.tile(base_starts, args.world)
lb = PE.Loopback(args.world)
engs = []
t0 = time.perf_counter()
for r in range(args.world):
    e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, msg_window=1 << 20)
    e.dist_init_loopback(lb, r, part, copy=args.mode == "copy", inplace=args.mode == "inplace")
    WL.build_engine_topics(e, wl)
    engs.append(e)
print(f"[loopback] {args.world} ranks ({args.partition} partition, {args.mode}) setup {time.perf_counter() - t0:.1f}s", flush=True)
expected = exp1 * args.world
times = []
for step in range(args.steps + 1):
    stats = [None] * args.world
    errs = []

    def go(r):
        try:
            engs[r].publish(msgs, starts)
            stats[r] = engs[r].run()
        except Exception as ex:  # noqa: BLE001
            errs.append((r, ex))

    t0 = time.perf_counter()
    th = [threading.Thread(target=go, args=(r,)) for r in range(args.world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    dt = (time.perf_counter() - t0) * 1e3
    assert not errs, errs
    times.append(dt)
    tot = sum(s.deliveries for s in stats)
    print(f"step {step}: deliveries {tot} expected {expected} {'OK' if tot == expected else 'MISMATCH'} "
          f"wall {dt:.2f} ms, modes {[s.expand_mode for s in stats]}, rounds {stats[0].rounds}", flush=True)
    assert tot == expected
med = float(np.median(times[1:]))
print(f"[loopback] {args.world} ranks: {med:.2f} ms/step vs {args.world} x single-rank {single:.2f} ms = "
      f"{args.world * single:.2f} ms: ratio {med / (args.world * single):.2f}", flush=True)
for e in engs:
    e.close()
lb.close()
