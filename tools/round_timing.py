#!/usr/bin/env python3
"""Per-launch device time of one workload's window (HIP events around every
launch, PS_F_TIME_KERNELS): round, launch kind, row bytes of the rounds it
writes, microseconds.  Averages over the steps after one warm-up.

    [PSAMD_...=...] python tools/round_timing.py [cfg3] [steps]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
wl = WL.CONFIGS[name]()
eng = PE.Engine(wl.n_peers, len(wl.topics), time_kernels=True, seed=wl.seed)
WL.build_engine_topics(eng, wl)
ms, st = None, None
for i in range(steps + 1):
    eng.publish(wl.msg_topics)
    st = eng.run()
    if i == 0:
        continue
    m = np.array([float(x) for x in st.expand_ms_per_round])
    ms = m if ms is None else ms + m
ms /= steps
kinds = list(st.round_kernel)
n = min(int(st.rounds), PE.MAX_ROUNDS - 1)
env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("PSAMD_"))
print(f"[{name}] {env or 'defaults'}: rounds {n}")
tot = 0.0
for q in range(1, n + 1):
    b = int(st.expand_bytes_per_round[q])
    k = PE.ROUND_KERNEL.get(kinds[q], "-")
    if ms[q] > 0:
        tot += ms[q]
    print(f"  round {q:2d} {k:12s} {b / 1e6:9.2f} MB {1e3 * ms[q]:8.1f} us")
print(f"  total {1e3 * tot:.1f} us")
eng.close()
