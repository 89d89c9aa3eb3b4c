"""GPU: the per-subscriber delivery surface (ps_read_peer_messages) -- what
client.Messages() (client.go:26-28, filled by processMessages
client.go:124-128) yields for one peer, in arrival order, checked against
the oracle's hops (oracle/psoracle.c or_disseminate) on the same inputs.
"""
import numpy as np
import pytest

import oracle as O
import psengine as PE

pytestmark = pytest.mark.gpu


def random_tree(rng, n, root):
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, O.NONE, dtype=np.uint32)
    for i in range(1, n):
        parent[perm[i]] = perm[rng.integers(0, i)]
    return parent


@pytest.mark.parametrize("paced", [False, True])
def test_peer_messages_match_oracle(paced):
    rng = np.random.default_rng(11 + paced)
    n, root = 2500, 7
    parent = random_tree(rng, n, root)
    live = (rng.random(n) > 0.1).astype(np.uint8)
    n_msgs = 300
    starts = rng.integers(0, 5, size=n_msgs) if paced else np.zeros(n_msgs, dtype=np.int64)
    with PE.Engine(n, 2) as eng:  # no hop record: the seen rows alone answer
        eng.set_tree(0, root, parent)
        eng.set_tree(1, root, parent)
        eng.set_live(live)
        topics = np.arange(n_msgs) % 2  # interleaved topics
        first = eng.publish(topics, starts if paced else None)
        eng.run()
        rp, cl = O.parents_to_csr(parent)
        _, ohops, _ = O.disseminate(rp, cl, root, live, 1)
        hop = ohops[0]  # one tree: every message reaches the same peers at the same hop
        for peer in list(rng.choice(n, 40, replace=False)) + [root]:
            for t in (0, 1):
                got = eng.peer_messages(t, int(peer))
                ids = [m for m in range(n_msgs) if topics[m] == t]
                if peer == root or hop[peer] == 0xFF:
                    exp = []
                else:  # arrival round = start + hop: entry round, then publish order
                    exp = sorted(ids, key=lambda m: (int(starts[m]), m))
                assert got.tolist() == [first + m for m in exp], (peer, t)


def test_peer_messages_errors_and_capacity():
    with PE.Engine(100, 1) as eng:
        with pytest.raises(PE.EngineError):
            eng.peer_messages(0, 1)  # no run yet
        eng.set_tree(0, 0, np.array([O.NONE] + [0] * 99, dtype=np.uint32))
        first = eng.publish(np.zeros(2000))
        eng.run()
        got = eng.peer_messages(0, 5)  # > the binding's first 1024-slot buffer
        assert got.tolist() == list(range(first, first + 2000))
        with pytest.raises(PE.EngineError):
            eng.peer_messages(1, 5)
        with pytest.raises(PE.EngineError):
            eng.peer_messages(0, 100)
