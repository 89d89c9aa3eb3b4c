"""k_pull_pair -- rounds q and q + 1 of a level window in one launch, each
wave writing a run of level-d nodes and then all their children from the
rows it holds in LDS -- against the restatement
(oracle/psoracle.c) and against one k_pull launch per round
(ps_plan_opts.chain_max = 1).

Round q delivers to BFS level q - s of each topic: a node receives its
parent's row of round q - 1 if the parent was reached this window and the
node is live (subtree.forwardMessage, subtree.go:319-354, the dead-child skip
at :326-331; client.processMessages, client.go:100-132).  The pair launch
must give the oracle's (peer, message, hop) exactly and leave the same
per-round counters and final seen state as the per-round launches --
recording and production instances, single starts and start groups, lazy
and eager seen, narrow and fan-out-heavy trees, rows too wide for the LDS
stage (no pairing then).
"""
import numpy as np
import pytest

import oracle as O
import psengine as PE

pytestmark = pytest.mark.gpu


def random_tree(rng, n, root, fan, lo=0):
    """Random tree, fan-out in [lo, fan] for the nodes that get children."""
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


def oracle_hops(topics, live):
    out = {}
    for t, (root, parent) in enumerate(topics):
        rp, cl = O.parents_to_csr(parent)
        _, oh, _ = O.disseminate(rp, cl, root, live, 1)
        out[t] = oh[0]
    return out


def run(monkeypatch, pair, n, topics, live, msg_topics, starts=None, record=True, flood=False, flags=0,
        msg_window=65536):
    # pairs only (chain_max 2; k_pull_chain: test_gpu_chain.py), or one k_pull per round
    opts = {"chain_max": 2 if pair else 1, "chain_max_groups": 2 if pair else 1, "flood": int(flood)}
    with PE.Engine(n, len(topics), record_hops=record, flags=flags, msg_window=msg_window, plan=opts) as eng:
        for t, (root, parent) in enumerate(topics):
            eng.set_tree(t, root, parent)
        eng.set_live(live)
        first = eng.publish(msg_topics, starts)
        st = eng.run()
        kinds = list(st.round_kernel)[: st.rounds + 1]
        hops = [eng.hops(first + m) for m in range(len(msg_topics))] if record else None
        deliv = [eng.delivered(first + m) for m in (0, len(msg_topics) - 1)]
        d = st.as_dict()
        key = (st.deliveries, st.duplicates, st.rounds, d["deliveries_per_round"], d["frontier_per_round"],
               eng.seen_digest())
    return st, kinds, hops, deliv, key


def check_hops(hops, exp, msg_topics, tag):
    for m, t in enumerate(msg_topics):
        if not np.array_equal(hops[m], exp[int(t)]):
            bad = np.nonzero(hops[m] != exp[int(t)])[0][:8]
            raise AssertionError(f"{tag} msg {m}: peers {bad} got {hops[m][bad]} want {exp[int(t)][bad]}")


def make_case(rng, n_lo=500, n_hi=4000, nt_hi=4, fan_lo=2, fan_hi=9, dead=0.15):
    n = int(rng.integers(n_lo, n_hi))
    nt = int(rng.integers(1, nt_hi + 1))
    topics = []
    for _ in range(nt):
        root = int(rng.integers(0, n))
        topics.append((root, random_tree(rng, n, root, fan=int(rng.integers(fan_lo, fan_hi)))))
    live = (rng.random(n) > dead).astype(np.uint8)
    for root, parent in topics:
        live[root] = 1
        kids = np.nonzero(parent == root)[0]
        if len(kids):
            live[kids[0]] = 0  # a dead child of the root: its subtree unreached
    return n, topics, live


@pytest.mark.parametrize("seed", range(6))
def test_pair_parity(monkeypatch, seed):
    """Random trees, several topics, ~15 % dead peers at every depth, ragged
    word counts (odd and even W): the pair launches equal the oracle message
    by message and the per-round launches in every counter and the digest."""
    rng = np.random.default_rng(900 + seed)
    n, topics, live = make_case(rng)
    nt = len(topics)
    n_msgs = int(rng.integers(1, 900))
    msg_topics = rng.integers(0, nt, size=n_msgs).astype(np.uint32)
    exp = oracle_hops(topics, live)
    total = sum(int((exp[t] != 0xFF).sum()) * int((msg_topics == t).sum()) for t in exp)
    ref = None
    for pair, record in ((False, True), (True, True), (True, False)):
        st, kinds, hops, _, key = run(monkeypatch, pair, n, topics, live, msg_topics, record=record)
        assert st.deliveries == total
        if pair:
            assert PE.K_PAIR in kinds and PE.K_PAIR2 in kinds, kinds
            assert st.expand_launches < st.rounds
        else:
            assert PE.K_PAIR not in kinds
        if record:
            check_hops(hops, exp, msg_topics, f"pair={pair}")
        ref = ref or key
        assert key == ref, (pair, record)


@pytest.mark.parametrize("seed", range(3))
def test_pair_after_flood(monkeypatch, seed):
    """k_flood for the leading rounds, pair launches after (the default
    schedule): the same hops, counters and digest as per-round launches."""
    rng = np.random.default_rng(950 + seed)
    n, topics, live = make_case(rng, 20000, 40000, nt_hi=3, fan_lo=2, fan_hi=4, dead=0.03)
    msg_topics = rng.integers(0, len(topics), size=int(rng.integers(300, 3000))).astype(np.uint32)
    exp = oracle_hops(topics, live)
    # k_flood for the rounds writing no more row bytes than round 1 (rows of
    # 16+ words padded to an even length, plan.cpp window_layout)
    def width(k):
        w = -(-k // 64)
        return w + (w & 1) if w >= 16 else w
    top = sum(int((parent == root).sum()) * width(int((msg_topics == t).sum())) * 8
              for t, (root, parent) in enumerate(topics))
    outs = []
    for pair in (False, True):
        # (overlap 0: deep windows plan no k_flood otherwise)
        opts = {"flood_top_bytes": top, "chain_max": 2 if pair else 1, "chain_max_groups": 2 if pair else 1,
                "overlap": 0, "flood_min_rounds": 1}
        with PE.Engine(n, len(topics), record_hops=True, plan=opts) as eng:
            for t, (root, parent) in enumerate(topics):
                eng.set_tree(t, root, parent)
            eng.set_live(live)
            first = eng.publish(msg_topics)
            st = eng.run()
            kinds = list(st.round_kernel)[: st.rounds + 1]
            assert st.flood_rounds >= 1 and kinds[1] == PE.K_FLOOD
            if pair:
                assert PE.K_PAIR in kinds
            for m in range(0, len(msg_topics), max(1, len(msg_topics) // 40)):
                assert np.array_equal(eng.hops(first + m), exp[int(msg_topics[m])]), (pair, m)
            d = st.as_dict()
            outs.append((st.deliveries, d["deliveries_per_round"], d["frontier_per_round"], eng.seen_digest()))
    assert outs[0] == outs[1]


@pytest.mark.parametrize("seed", range(4))
def test_pair_start_groups(monkeypatch, seed):
    """Start rounds 0..7 per message (group-major blocks; groups entering at
    round q run their level 1 inside the pair launch of rounds q - 1, q):
    the oracle's hops relative to each start, and the per-round launches'
    counters and digest."""
    rng = np.random.default_rng(970 + seed)
    n, topics, live = make_case(rng, 800, 3000, nt_hi=3, dead=0.1)
    nt = len(topics)
    msg_topics = rng.integers(0, nt, size=int(rng.integers(100, 1200))).astype(np.uint32)
    starts = rng.integers(0, 8, size=msg_topics.shape[0]).astype(np.uint32)
    exp = oracle_hops(topics, live)
    ref = None
    for pair, record in ((False, True), (True, True), (True, False)):
        st, kinds, hops, deliv, key = run(monkeypatch, pair, n, topics, live, msg_topics, starts, record=record)
        if pair:
            assert PE.K_PAIR in kinds
        if record:
            check_hops(hops, exp, msg_topics, f"pair={pair}")
        ref = ref or (key, [x.tolist() for x in deliv])
        assert (key, [x.tolist() for x in deliv]) == ref, (pair, record)


def test_pair_fanout_heavy(monkeypatch):
    """Fan-out up to 24 with one-word rows: a wave's run of up to 128 parents
    has hundreds of children, streamed 256 at a time; a dead child in every
    sibling group."""
    rng = np.random.default_rng(991)
    n = 30000
    topics = [(5, random_tree(rng, n, 5, 24)), (11, random_tree(rng, n, 11, 12))]
    live = (rng.random(n) > 0.05).astype(np.uint8)
    for r, _ in topics:
        live[r] = 1
    msg_topics = np.array([0] * 40 + [1] * 70, dtype=np.uint32)  # W = 1 and W = 2
    exp = oracle_hops(topics, live)
    ref = None
    for pair, record in ((False, True), (True, True), (True, False)):
        st, kinds, hops, _, key = run(monkeypatch, pair, n, topics, live, msg_topics, record=record)
        if pair:
            assert PE.K_PAIR in kinds
        if record:
            check_hops(hops, exp, msg_topics, f"pair={pair}")
        ref = ref or key
        assert key == ref


def test_pair_eager_seen(monkeypatch):
    """PS_F_NO_LAZY_SEEN (every row cleared and every generation stamped up
    front): the pair launch counts a dead parent's children as the separate
    launch's generation test would, and leaves the same state."""
    rng = np.random.default_rng(993)
    n, topics, live = make_case(rng, 1000, 3000, nt_hi=2, dead=0.2)
    msg_topics = rng.integers(0, len(topics), size=300).astype(np.uint32)
    exp = oracle_hops(topics, live)
    outs = []
    for pair in (False, True):
        st, kinds, hops, _, key = run(monkeypatch, pair, n, topics, live, msg_topics, flags=PE.F_NO_LAZY_SEEN)
        check_hops(hops, exp, msg_topics, f"eager pair={pair}")
        outs.append(key)
    assert outs[0] == outs[1]


def test_pair_rows_wider_than_stage(monkeypatch):
    """A topic whose rows exceed the LDS stage (70,000 messages: 1,094 words
    > 768) never pairs; a narrow topic beside it in the same window still
    gives the oracle's hops."""
    rng = np.random.default_rng(995)
    n = 600
    topics = [(0, random_tree(rng, n, 0, 3)), (1, random_tree(rng, n, 1, 4))]
    live = (rng.random(n) > 0.1).astype(np.uint8)
    live[0] = live[1] = 1
    msg_topics = np.concatenate([np.zeros(70000, dtype=np.uint32), np.ones(100, dtype=np.uint32)])
    exp = oracle_hops(topics, live)
    outs = []
    for pair in (False, True):
        st, kinds, hops, _, key = run(monkeypatch, pair, n, topics, live, msg_topics, record=False,
                                      msg_window=1 << 17)
        assert PE.K_PAIR not in kinds
        outs.append(key)
    assert outs[0] == outs[1]
    assert outs[0][0] == int((exp[0] != 0xFF).sum()) * 70000 + int((exp[1] != 0xFF).sum()) * 100


def test_pair_deep_chain_hops_past_255(monkeypatch):
    """A chain of 600 peers through pair launches only (PSAMD_FLOOD=0): 299
    pair launches of one node each; hops past 255 saturate at 254 as in the
    restatement."""
    n = 600
    parent = np.full(n, O.NONE, dtype=np.uint32)
    parent[1:] = np.arange(n - 1, dtype=np.uint32)
    live = np.ones(n, dtype=np.uint8)
    exp = oracle_hops([(0, parent)], live)[0]
    msg_topics = np.zeros(130, dtype=np.uint32)
    st, kinds, hops, _, key = run(monkeypatch, True, n, [(0, parent)], live, msg_topics)
    assert st.deliveries == 130 * (n - 1)
    assert kinds.count(PE.K_PAIR) >= 100
    for m in (0, 64, 129):
        assert np.array_equal(hops[m], exp)
    _, _, _, _, key0 = run(monkeypatch, False, n, [(0, parent)], live, msg_topics)
    assert key == key0


def test_pair_many_windows_and_drains(monkeypatch):
    """1,500 messages over two topics through 128-message windows (6+ windows,
    generations advancing per window) with start groups: pair launches give the oracle's
    hops, and each subscriber's drain (ps_read_peer_messages: its message ids
    in arrival order) equals the per-round launches'."""
    rng = np.random.default_rng(997)
    n, topics, live = make_case(rng, 1500, 2500, nt_hi=2, dead=0.08)
    msg_topics = rng.integers(0, len(topics), size=1500).astype(np.uint32)
    starts = rng.integers(0, 4, size=1500).astype(np.uint32)
    exp = oracle_hops(topics, live)
    peers = [int(p) for p in rng.integers(0, n, size=12)]
    outs = []
    for pair in (False, True):
        opts = {"chain_max": 2 if pair else 1, "chain_max_groups": 2 if pair else 1, "flood": 0}
        with PE.Engine(n, len(topics), record_hops=True, msg_window=128, plan=opts) as eng:
            for t, (root, parent) in enumerate(topics):
                eng.set_tree(t, root, parent)
            eng.set_live(live)
            first = eng.publish(msg_topics, starts)
            st = eng.run()
            assert st.windows >= 6  # (128 messages per topic per window)
            for m in range(0, 1500, 37):
                assert np.array_equal(eng.hops(first + m), exp[int(msg_topics[m])]), (pair, m)
            drains = [eng.peer_messages(t, p).tolist() for t in range(len(topics)) for p in peers]
            outs.append((st.deliveries, drains))
    assert outs[0] == outs[1]
