#!/usr/bin/env python3
"""Dumps cfg5's initial join order and churn plan for tools/tree_bench.cpp.

    python tools/tree_bench.py /tmp/plan.bin [batches]
"""
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
from psengine import workloads as WL  # noqa: E402

out = sys.argv[1]
batches = int(sys.argv[2]) if len(sys.argv) > 2 else 12
wl = WL.cfg5()
ts = wl.topics[0]
plan = WL.churn_plan(wl, batches)
with open(out, "wb") as fh:
    fh.write(struct.pack("<5I", wl.n_peers, ts.root, ts.width, ts.max_width, batches))
    for arr in [ts.join_order] + [a for lj in plan for a in lj]:
        a = np.asarray(arr, dtype=np.uint32)
        fh.write(struct.pack("<I", a.size))
        fh.write(a.tobytes())
