#!/usr/bin/env python3
"""Host/GPU split of one bench step (publish + ps_run) on a workload.

    PSAMD_HOST_TIMING=1 python tools/step_timing.py [cfg3] [steps]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
wl = WL.CONFIGS[name]()
eng = PE.Engine(wl.n_peers, len(wl.topics), time_kernels=os.environ.get("TIMEK", "1") == "1", seed=wl.seed)
WL.build_engine_topics(eng, wl)
for i in range(steps):
    t0 = time.perf_counter()
    eng.publish(wl.msg_topics)
    t1 = time.perf_counter()
    st = eng.run()
    t2 = time.perf_counter()
    print(f"step {i}: publish {1e3 * (t1 - t0):.3f} ms, run {1e3 * (t2 - t1):.3f} ms "
          f"(host_ms {st.host_ms:.3f}, gpu run_ms {st.run_ms:.3f}, expand {st.expand_ms:.3f})",
          file=sys.stderr, flush=True)
eng.close()

# pipelined loop (bench.py's default): where the host spends a step
if os.environ.get("PIPE", "1") == "1":
    eng = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
    WL.build_engine_topics(eng, wl)
    for i in range(steps + 1):
        t0 = time.perf_counter()
        eng.publish(wl.msg_topics)
        t1 = time.perf_counter()
        eng.run_async()
        t2 = time.perf_counter()
        if i:
            st = eng.wait()
        t3 = time.perf_counter()
        print(f"pipe {i}: publish {1e3 * (t1 - t0):.3f} ms, run_async {1e3 * (t2 - t1):.3f} ms, "
              f"wait {1e3 * (t3 - t2):.3f} ms", file=sys.stderr, flush=True)
    eng.wait()
    eng.close()
