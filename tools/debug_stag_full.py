#!/usr/bin/env python3
"""Debug: the full cfg3 staggered windows of the overlap test, blocking:
aligned (split mismatches reported, not fatal) against align_groups 0, per
round, window by window."""
import os
import sys

import numpy as np

os.environ["PSAMD_SPLIT_WARN"] = "1"
os.environ["PSAMD_CHECK_ROOTS"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402
from test_gpu_async import vary_group_counts  # noqa: E402

wl = WL.cfg3()
starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(8)).astype(np.uint32)
batches = [vary_group_counts(wl.msg_topics, starts, i) for i in range(3)]
rng = np.random.default_rng(12)
live = (rng.random(wl.n_peers) >= 0.02).astype(np.uint8)
live[[ts.root for ts in wl.topics]] = 1
res = {}
for align in (1, 0):
    e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, plan={"align_groups": align, "overlap": 0})
    WL.build_engine_topics(e, wl)
    e.set_live(live)
    out = []
    for i in range(3):
        e.publish(*batches[i])
        st = e.run()
        d = st.as_dict()
        out.append((st.deliveries, d["deliveries_per_round"][:30], e.seen_digest()))
        # sampled delivered sets of the hot topic's first and last message
    res[align] = out
    e.close()
for i in range(3):
    a, b = res[1][i], res[0][i]
    print(i, "deliv", a[0], b[0], "digest eq", a[2] == b[2])
    print("  per round aligned", a[1])
    print("  per round rounds ", b[1])
