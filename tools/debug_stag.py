#!/usr/bin/env python3
"""Debug: staggered windows, blocking vs pipelined, per plan variant: the
final seen digest and every window's counters (tests/test_gpu_async.py's
staggered overlap case)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402
from test_gpu_async import stats_key, vary_group_counts  # noqa: E402

wl = WL.cfg3(200_000, 16, 5000)
rng = np.random.default_rng(12)
live = (rng.random(wl.n_peers) >= 0.03).astype(np.uint8)
live[[ts.root for ts in wl.topics]] = 1
starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(8)).astype(np.uint32)
batches = [vary_group_counts(wl.msg_topics, starts, i) for i in range(8)]
for variant in json.loads(sys.argv[1] if len(sys.argv) > 1 else '[{}]'):
    for pipelined in (False, True):
        e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, plan={"overlap_min_bytes": 0, **variant})
        WL.build_engine_topics(e, wl)
        e.set_live(live)
        res, dig = [], []
        if pipelined:
            for i in range(8):
                e.publish(*batches[i])
                e.run_async()
                if i:
                    res.append(stats_key(e.wait()))
            res.append(stats_key(e.wait()))
        else:
            for i in range(8):
                e.publish(*batches[i])
                res.append(stats_key(e.run()))
                dig.append(e.seen_digest())
        print(json.dumps({"variant": variant, "pipelined": pipelined, "digest": e.seen_digest(),
                          "overlapped": e.overlapped_windows(), "digests": dig,
                          "deliv": [r[0] for r in res], "rounds": [r[2] for r in res],
                          "per_round0": list(res[0][5][:30]), "per_round_last": list(res[-1][5][:30])}), flush=True)
        e.close()
