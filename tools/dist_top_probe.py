#!/usr/bin/env python3
"""Launch counts per rank of a loopback multi-rank window with and without
the top launch (PSAMD_PULL_TOP_MB=0), and that the job's deliveries agree.

    python tools/dist_top_probe.py [world] [scale]
"""
import os
import sys
import threading

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
wl = WL.scaled("cfg3", scale)
wl.msg_topics = np.tile(wl.msg_topics, world)
for top in ("0", "32"):
    os.environ["PSAMD_PULL_TOP_MB"] = top
    lb = PE.Loopback(world)
    engs = []
    for r in range(world):
        e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, msg_window=1 << 20)
        e.dist_init_loopback(lb, r, PE.PART_SUBTREE)
        WL.build_engine_topics(e, wl)
        engs.append(e)
    stats = [None] * world

    def go(r):
        engs[r].publish(wl.msg_topics)
        stats[r] = engs[r].run()

    for _ in range(2):
        th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    print(f"top_mb={top}: deliveries {sum(s.deliveries for s in stats)}, "
          f"launches per rank {[int(s.expand_launches) for s in stats]}, rounds {[int(s.rounds) for s in stats]}",
          flush=True)
    for e in engs:
        e.close()
