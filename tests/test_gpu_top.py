"""The top-levels launch (k_pull_top) against the oracle.

The leading rounds of a single-start window run in one launch whose nodes
decide reachability by walking their ancestors (root reached, every ancestor
below it live) and copy the root's arrival row.  These tests pin it to the
restatement (subtree.go:319-354, client.go:100-132) with dead nodes at every
depth of the top levels, and show that every split between the top launch
and the per-level launches (PSAMD_PULL_TOP_MB, read at engine creation)
gives the same hops, deliveries and per-round counts.
"""
import numpy as np
import pytest

import oracle as O
import psengine as PE

pytestmark = pytest.mark.gpu


def random_tree(rng, n, root, fan):
    """Random tree, fan-out <= fan, labels shuffled, root given."""
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, O.NONE, dtype=np.uint32)
    kids = np.zeros(n, dtype=np.int64)
    for i in range(1, n):
        while True:
            p = perm[rng.integers(max(0, i - 4 * fan), i)]
            if kids[p] < fan:
                break
        parent[perm[i]] = p
        kids[p] += 1
    return parent


def run_variant(monkeypatch, top_mb, n, topics, live, msg_topics, record=True):
    if top_mb is None:
        monkeypatch.delenv("PSAMD_PULL_TOP_MB", raising=False)
    else:
        monkeypatch.setenv("PSAMD_PULL_TOP_MB", str(top_mb))
    with PE.Engine(n, len(topics), record_hops=record) as eng:
        for t, (root, parent) in enumerate(topics):
            eng.set_tree(t, root, parent)
        eng.set_live(live)
        first = eng.publish(msg_topics)
        st = eng.run()
        hops = [eng.hops(first + m) for m in range(len(msg_topics))] if record else None
    return st, hops


@pytest.mark.parametrize("seed", range(4))
def test_top_split_parity(monkeypatch, seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(500, 4000))
    nt = int(rng.integers(1, 5))
    topics = []
    for t in range(nt):
        root = int(rng.integers(0, n))
        topics.append((root, random_tree(rng, n, root, fan=int(rng.integers(2, 9)))))
    # dead peers at every depth, roots' children included
    live = (rng.random(n) > 0.15).astype(np.uint8)
    for root, parent in topics:
        live[root] = 1
        kids = np.nonzero(parent == root)[0]
        if len(kids):
            live[kids[0]] = 0
    n_msgs = int(rng.integers(1, 400))
    msg_topics = rng.integers(0, nt, size=n_msgs).astype(np.uint32)
    # expected: the restatement, message by message
    exp = {}
    for t, (root, parent) in enumerate(topics):
        rp, cl = O.parents_to_csr(parent)
        cnt = int((msg_topics == t).sum())
        if cnt:
            _, oh, _ = O.disseminate(rp, cl, root, live, 1)
            exp[t] = oh[0]
    total = sum(int((exp[t] != 0xFF).sum()) * int((msg_topics == t).sum()) for t in exp)
    ref = None
    for top_mb in (0, 0.0005, 0.002, None):  # per-level only, two splits, the default
        st, hops = run_variant(monkeypatch, top_mb, n, topics, live, msg_topics)
        assert st.deliveries == total, (top_mb, st.deliveries, total)
        assert st.duplicates == 0
        for m, t in enumerate(msg_topics):
            if not np.array_equal(hops[m], exp[int(t)]):
                bad = np.nonzero(hops[m] != exp[int(t)])[0][:8]
                raise AssertionError(f"top_mb={top_mb} msg {m}: peers {bad} got {hops[m][bad]} "
                                     f"want {exp[int(t)][bad]}")
        d = st.as_dict()
        key = (st.rounds, d["frontier_per_round"], d["deliveries_per_round"])
        if ref is None:
            ref = key
        assert key == ref, (top_mb, key, ref)


def test_top_no_record_counts(monkeypatch):
    """Production instance (no hop record): the same deliveries and rounds
    with and without the top launch on a deeper, wider workload."""
    rng = np.random.default_rng(7)
    n = 60000
    topics = [(0, random_tree(rng, n, 0, fan=2)), (5, random_tree(rng, n, 5, fan=8))]
    live = (rng.random(n) > 0.02).astype(np.uint8)
    live[0] = live[5] = 1
    msg_topics = rng.integers(0, 2, size=3000).astype(np.uint32)
    a, _ = run_variant(monkeypatch, 0, n, topics, live, msg_topics, record=False)
    b, _ = run_variant(monkeypatch, None, n, topics, live, msg_topics, record=False)
    assert a.deliveries == b.deliveries and a.rounds == b.rounds
    da, db = a.as_dict(), b.as_dict()
    assert da["frontier_per_round"] == db["frontier_per_round"]
    assert da["deliveries_per_round"] == db["deliveries_per_round"]
    assert db["expand_launches"] < da["expand_launches"]  # the top launch replaced several


def test_top_cache_follows_live_changes():
    """The per-node path-liveness the top launch keeps between windows is
    dropped when the live mask changes: kill and revive top-level peers
    between runs of one engine, each run equal to the restatement."""
    rng = np.random.default_rng(9)
    n = 3000
    parent = random_tree(rng, n, 0, fan=3)
    rp, cl = O.parents_to_csr(parent)
    live = np.ones(n, dtype=np.uint8)
    kids = np.nonzero(parent == 0)[0]
    grand = np.nonzero(np.isin(parent, kids))[0]
    with PE.Engine(n, 1, record_hops=True) as eng:
        eng.set_tree(0, 0, parent)
        for step, change in enumerate([None, kids[:1], grand[:3], None, "revive"]):
            if isinstance(change, str):
                live[:] = 1
            elif change is not None:
                live[change] = 0
            eng.set_live(live)
            first = eng.publish(np.zeros(70))
            st = eng.run()
            total, oh, _ = O.disseminate(rp, cl, 0, live, 1)
            assert st.deliveries == total * 70, step
            for m in (0, 69):
                assert np.array_equal(eng.hops(first + m), oh[0]), (step, m)


def _odd_digests(monkeypatch, odd_mode, record, n, topics, live, msg_topics):
    """Seen digests and deliveries of two back-to-back runs (the second reads
    the path-liveness cache) with PSAMD_TOP_ODD_WIDE = odd_mode."""
    monkeypatch.delenv("PSAMD_PULL_TOP_MB", raising=False)
    monkeypatch.setenv("PSAMD_TOP_ODD_WIDE", str(odd_mode))
    out = []
    with PE.Engine(n, len(topics), record_hops=record) as eng:
        for t, (root, parent) in enumerate(topics):
            eng.set_tree(t, root, parent)
        eng.set_live(live)
        for _ in range(2):
            eng.publish(msg_topics)
            st = eng.run()
            out.append((st.deliveries, st.as_dict()["deliveries_per_round"], eng.seen_digest()))
    return out


@pytest.mark.parametrize("seed", range(4))
def test_top_odd_row_stores(monkeypatch, seed):
    """Odd W (rows of an odd number of 64-message words): the non-recording
    launch stores aligned 16-B pairs that straddle two nodes' rows, with a
    head and a tail word; its seen state must equal the per-word stream's and
    the recording launch's (whose hops the oracle pins above), dead nodes
    and odd run alignments included."""
    rng = np.random.default_rng(700 + seed)
    n = int(rng.integers(300, 3000))
    nt = int(rng.integers(1, 4))
    topics = []
    for t in range(nt):
        root = int(rng.integers(0, n))
        topics.append((root, random_tree(rng, n, root, fan=int(rng.integers(2, 9)))))
    live = rng.random(n) > 0.05
    for root, _ in topics:
        live[root] = True
    # per topic an odd word count (1, 3, 5, 7, 9 words), last word ragged
    counts = [64 * int(rng.choice([0, 2, 4, 6, 8])) + int(rng.integers(1, 65)) for _ in range(nt)]
    msg_topics = rng.permutation(np.repeat(np.arange(nt), counts)).astype(np.uint32)
    ref = _odd_digests(monkeypatch, 1, True, n, topics, live, msg_topics)
    for mode in (2, 1, 0):
        got = _odd_digests(monkeypatch, mode, False, n, topics, live, msg_topics)
        assert got == ref, (mode, counts)
    # blocks dealt to the XCDs as contiguous ranges (PSAMD_TOP_XCD): same state
    monkeypatch.setenv("PSAMD_TOP_XCD", "1")
    assert _odd_digests(monkeypatch, 2, False, n, topics, live, msg_topics) == ref
    assert _odd_digests(monkeypatch, 1, True, n, topics, live, msg_topics) == ref
