#!/usr/bin/env python3
"""Multi-rank path at bench scale on ONE GPU: `world` engines in threads with
the loopback transport (device copies in place of RCCL), weak-scaled cfg3
(world x the messages).  Checks the job's deliveries and prints per-step
times -- a correctness and overhead probe, not a scaling measurement.

    python tools/loopback_bench.py [world] [scale] [steps]
"""
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
wl = WL.scaled("cfg3", scale)
wl.msg_topics = np.tile(wl.msg_topics, world)
lb = PE.Loopback(world)
engs = []
for r in range(world):
    e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, msg_window=1 << 20)
    e.dist_init_loopback(lb, r, PE.PART_SUBTREE)
    sizes = WL.build_engine_topics(e, wl)
    engs.append(e)
expected = wl.expected_deliveries(sizes)
for step in range(steps):
    stats = [None] * world
    def go(r):
        engs[r].publish(wl.msg_topics)
        stats[r] = engs[r].run()
    t0 = time.perf_counter()
    th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    tot = sum(s.deliveries for s in stats)
    print(f"step {step}: world {world} deliveries {tot} expected {expected} "
          f"{'OK' if tot == expected else 'MISMATCH'} wall {dt * 1e3:.2f} ms, "
          f"modes {[s.expand_mode for s in stats]}, rounds {stats[0].rounds}", flush=True)
    assert tot == expected
for e in engs:
    e.close()
lb.close()
