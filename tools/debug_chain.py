#!/usr/bin/env python3
"""Debug aid: test_chain_column_slices' case through one plan, hops against
the oracle, the first mismatches with their BFS levels."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle as O  # noqa: E402
import psengine as PE  # noqa: E402
from test_gpu_pair import oracle_hops, random_tree  # noqa: E402

n_msgs = int(sys.argv[1]) if len(sys.argv) > 1 else 21000
chain = int(sys.argv[2]) if len(sys.argv) > 2 else 4
record = int(sys.argv[3]) if len(sys.argv) > 3 else 1
rng = np.random.default_rng(1950 + n_msgs)
n = 3000
topics = [(0, random_tree(rng, n, 0, 3)), (7, random_tree(rng, n, 7, 5))]
live = (rng.random(n) > 0.05).astype(np.uint8)
live[0] = live[7] = 1
msg_topics = np.concatenate([np.zeros(n_msgs, dtype=np.uint32), np.ones(150, dtype=np.uint32)])
rng.shuffle(msg_topics)
exp = oracle_hops(topics, live)
for ch in (1, chain):
    opts = {"chain_max": ch, "chain_max_groups": ch, "flood": 0}
    with PE.Engine(n, 2, record_hops=bool(record), msg_window=1 << 16, plan=opts) as eng:
        for t, (root, parent) in enumerate(topics):
            eng.set_tree(t, root, parent)
        eng.set_live(live)
        first = eng.publish(msg_topics)
        st = eng.run()
        d = st.as_dict()
        print(f"chain={ch} deliveries {st.deliveries} kinds {d['round_kernel']}")
        print("  per round", d["deliveries_per_round"][:12])
        if record:
            bad = 0
            for m in range(len(msg_topics)):
                h = eng.hops(first + m)
                t = int(msg_topics[m])
                if not np.array_equal(h, exp[t]):
                    diff = np.nonzero(h != exp[t])[0]
                    print(f"  msg {m} topic {t}: {diff.size} peers differ, e.g. {diff[:6]} got {h[diff[:6]]} "
                          f"want {exp[t][diff[:6]]}")
                    bad += 1
                    if bad > 4:
                        break
            print("  mismatching messages:", bad)
