"""k_flood -- every round of a single-start tree window in one persistent
launch -- against the restatement (oracle/psoracle.c).

Round q delivers to BFS level q - s_t of each topic: a node receives its
parent's row of round q - 1 if the parent was reached this window and the
node is live (subtree.forwardMessage, subtree.go:319-354, the dead-child skip
at :326-331; client.processMessages, client.go:100-132).  k_flood orders the
rounds by per-task dependencies inside one launch; ps_plan_opts.flood = 0
runs one k_pull launch per round instead.  Both must give
the oracle's (peer, message, hop) exactly, the same per-round counters, and
the same final seen state -- recording and production instances alike.
"""
import numpy as np
import pytest

import oracle as O
import psengine as PE
from fullsize_common import cfg3_dead_mask as _cfg3_dead_mask
from psengine import workloads as WL

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


def run_mode(monkeypatch, flood, n, topics, live, msg_topics, record=True, starts=None, words=None, top=None):
    """One window; `top` (ps_plan_opts.flood_top_bytes): k_flood runs the
    leading rounds writing at most that many row bytes, k_pull the rest
    (default: 4 MB, every round of these small trees)."""
    # (deep windows plan no k_flood while the cross-window overlap is on)
    opts = {"flood": int(flood), "overlap": 0 if flood else 1, "flood_min_rounds": 1}
    if top is not None:
        opts["flood_top_bytes"] = top
    if words is not None:
        opts["flood_words"] = words
    with PE.Engine(n, len(topics), record_hops=record, plan=opts) as eng:
        for t, (root, parent) in enumerate(topics):
            eng.set_tree(t, root, parent)
        eng.set_live(live)
        first = eng.publish(msg_topics, starts)
        st = eng.run()
        assert st.expand_mode == (PE.MODE_FLOOD if flood else PE.MODE_LEVEL_PULL)
        if flood:
            assert 1 <= st.flood_rounds <= st.rounds
            if top is None:
                assert st.flood_rounds == st.rounds and st.expand_launches == 1
            elif st.rounds < PE.MAX_ROUNDS:  # k_pull rounds with rows, k_pull_pair round pairs
                k = list(st.round_kernel)
                assert st.expand_launches == 1 + sum(
                    1 for q in range(st.flood_rounds + 1, st.rounds + 1)
                    if (k[q] == PE.K_PULL and st.expand_bytes_per_round[q]) or k[q] in (PE.K_PAIR, PE.K_CHAIN))
        hops = [eng.hops(first + m) for m in range(len(msg_topics))] if record else None
        digest = eng.seen_digest()
    return st, hops, digest


def oracle_hops(topics, live):
    out = {}
    for t, (root, parent) in enumerate(topics):
        rp, cl = O.parents_to_csr(parent)
        _, oh, _ = O.disseminate(rp, cl, root, live, 1)
        out[t] = oh[0]
    return out


@pytest.mark.parametrize("seed", range(6))
def test_flood_parity(monkeypatch, seed):
    """Random trees (fan-out 2..8), several topics, ~15 % dead peers at every
    depth (a root's child included), ragged word counts: k_flood and the
    per-round launches both equal the oracle message by message."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(500, 4000))
    nt = int(rng.integers(1, 5))
    topics = []
    for t in range(nt):
        root = int(rng.integers(0, n))
        topics.append((root, random_tree(rng, n, root, fan=int(rng.integers(2, 9)))))
    live = (rng.random(n) > 0.15).astype(np.uint8)
    for root, parent in topics:
        live[root] = 1
        kids = np.nonzero(parent == root)[0]
        if len(kids):
            live[kids[0]] = 0
    n_msgs = int(rng.integers(1, 700))
    msg_topics = rng.integers(0, nt, size=n_msgs).astype(np.uint32)
    exp = oracle_hops(topics, live)
    total = sum(int((exp[t] != 0xFF).sum()) * int((msg_topics == t).sum()) for t in exp)
    ref = None
    # small tasks (64 words) force many tasks and cross-task waits per level;
    # top=2048: k_flood for the first rounds only, k_pull launches after it
    for flood, words, top in ((False, None, None), (True, None, None), (True, 64, None), (True, None, 2048)):
        st, hops, digest = run_mode(monkeypatch, flood, n, topics, live, msg_topics, words=words, top=top)
        assert st.deliveries == total, (flood, words, st.deliveries, total)
        assert st.duplicates == 0
        for m, t in enumerate(msg_topics):
            if not np.array_equal(hops[m], exp[int(t)]):
                bad = np.nonzero(hops[m] != exp[int(t)])[0][:8]
                raise AssertionError(f"flood={flood} words={words} msg {m}: peers {bad} got {hops[m][bad]} "
                                     f"want {exp[int(t)][bad]}")
        d = st.as_dict()
        key = (st.rounds, d["frontier_per_round"], d["deliveries_per_round"], digest)
        if ref is None:
            ref = key
        assert key == ref, (flood, words)


@pytest.mark.parametrize("seed", range(4))
def test_flood_production_instance(monkeypatch, seed):
    """The non-recording k_flood (its 16-B even-W stream and its odd-W pair
    stores with head and tail words) leaves the same seen state, deliveries
    and per-round counts as the recording instance and the per-round
    launches, for odd and even row widths (1..9 words, ragged last word)."""
    rng = np.random.default_rng(700 + seed)
    n = int(rng.integers(300, 3000))
    nt = int(rng.integers(1, 4))
    topics = []
    for t in range(nt):
        root = int(rng.integers(0, n))
        topics.append((root, random_tree(rng, n, root, fan=int(rng.integers(2, 9)))))
    live = (rng.random(n) > 0.05).astype(np.uint8)
    for root, _ in topics:
        live[root] = 1
    counts = [64 * int(rng.integers(0, 9)) + int(rng.integers(1, 65)) for _ in range(nt)]
    msg_topics = rng.permutation(np.repeat(np.arange(nt), counts)).astype(np.uint32)
    outs = []
    for flood, record, words, top in ((False, True, None, None), (True, True, None, None),
                                      (True, False, None, None), (True, False, 128, None),
                                      (True, False, None, 4096), (False, False, None, None)):
        st, _, digest = run_mode(monkeypatch, flood, n, topics, live, msg_topics, record=record, words=words,
                                 top=top)
        d = st.as_dict()
        outs.append((st.deliveries, st.duplicates, d["deliveries_per_round"], d["frontier_per_round"], digest))
    assert all(o == outs[0] for o in outs), (counts, outs)


def test_flood_topics_with_different_start_rounds(monkeypatch):
    """Each topic single-start, but at different rounds (ps_publish_at): one
    k_flood launch still; hops are relative to each message's start round."""
    rng = np.random.default_rng(31)
    n = 2500
    topics = [(0, random_tree(rng, n, 0, 3)), (7, random_tree(rng, n, 7, 5)), (9, random_tree(rng, n, 9, 2))]
    live = (rng.random(n) > 0.08).astype(np.uint8)
    for r, _ in topics:
        live[r] = 1
    msg_topics = rng.integers(0, 3, size=500).astype(np.uint32)
    starts = np.array([0, 3, 6], dtype=np.uint32)[msg_topics]
    exp = oracle_hops(topics, live)
    # top = round 1's row bytes: k_flood for the leading rounds that write no
    # more than that; the later topics start inside the k_pull launches, from
    # roots k_flood's launch seeded
    per_round = {}
    for t, (root, parent) in enumerate(topics):
        w = -(-int((msg_topics == t).sum()) // 64)
        depth = np.zeros(n, dtype=np.int64)
        for v in range(n):  # depth by walking up (n is small)
            d, u = 0, v
            while u != root:
                u, d = int(parent[u]), d + 1
            depth[v] = d
        for d, c in zip(*np.unique(depth[depth > 0], return_counts=True)):
            q = int(d) + int(starts[msg_topics == t][0])
            per_round[q] = per_round.get(q, 0) + int(c) * w * 8
    top1 = per_round[1]
    expect_fr = 0
    while per_round.get(expect_fr + 1, 0) <= top1 and expect_fr < max(per_round):
        expect_fr += 1
    assert expect_fr < 6  # topic 2 (start 6) begins inside the k_pull launches
    for flood, top in ((True, None), (True, top1), (False, None)):
        st, hops, _ = run_mode(monkeypatch, flood, n, topics, live, msg_topics, starts=starts, top=top)
        if top is not None:
            assert st.flood_rounds == expect_fr
        for m, t in enumerate(msg_topics):
            assert np.array_equal(hops[m], exp[int(t)]), (flood, top, m)
        assert st.deliveries == sum(int((exp[int(t)] != 0xFF).sum()) for t in msg_topics)


def test_flood_deep_chain(monkeypatch):
    """A chain of 600 peers: 599 rounds, one single-node task per round, each
    waiting on the previous one; hops past 255 saturate at 254 as in the
    restatement."""
    n = 600
    parent = np.full(n, O.NONE, dtype=np.uint32)
    parent[1:] = np.arange(n - 1, dtype=np.uint32)
    live = np.ones(n, dtype=np.uint8)
    exp = oracle_hops([(0, parent)], live)[0]
    st, hops, _ = run_mode(monkeypatch, True, n, [(0, parent)], live, np.zeros(130, dtype=np.uint32))
    assert st.deliveries == 130 * (n - 1)
    for m in (0, 64, 129):
        assert np.array_equal(hops[m], exp)


def test_flood_follows_live_changes(monkeypatch):
    """Kill and revive top-level peers between runs of one engine: every run
    decides reachability from its own window's generation stamps."""
    rng = np.random.default_rng(9)
    n = 3000
    parent = random_tree(rng, n, 0, fan=3)
    rp, cl = O.parents_to_csr(parent)
    live = np.ones(n, dtype=np.uint8)
    kids = np.nonzero(parent == 0)[0]
    grand = np.nonzero(np.isin(parent, kids))[0]
    with PE.Engine(n, 1, record_hops=True, plan={"flood": 1, "overlap": 0, "flood_min_rounds": 1}) as eng:
        eng.set_tree(0, 0, parent)
        for step, change in enumerate([None, kids[:1], grand[:3], None, "revive"]):
            if isinstance(change, str):
                live[:] = 1
            elif change is not None:
                live[change] = 0
            eng.set_live(live)
            first = eng.publish(np.zeros(70))
            st = eng.run()
            assert st.expand_mode == PE.MODE_FLOOD
            total, oh, _ = O.disseminate(rp, cl, 0, live, 1)
            assert st.deliveries == total * 70, step
            for m in (0, 69):
                assert np.array_equal(eng.hops(first + m), oh[0]), (step, m)


def test_cfg3_full_size_dead_mask_against_oracle():
    """BASELINE cfg3 at full size (1M peers, 64 Zipf topics, 100k messages)
    with ~2 % dead peers including top-level ones, production instance: the
    exact deliveries and per-round histogram of the restatement per topic,
    and for 16 sampled messages of a hot (0), a mid (8) and a cold (63)
    topic, the delivered peer set of or_disseminate."""
    wl = WL.cfg3()
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) as eng:
        WL.build_engine_topics(eng, wl)
        parents = [eng.parents(t) for t in range(len(wl.topics))]
        live = _cfg3_dead_mask(wl, parents)
        eng.set_live(live)
        first = eng.publish(wl.msg_topics)
        st = eng.run()
        # the default deep-window plan: chains from round 1, no k_flood
        assert st.expand_mode == PE.MODE_LEVEL_PULL and PE.K_CHAIN in set(st.round_kernel)
        cnt = np.bincount(wl.msg_topics, minlength=len(wl.topics))
        exp_total, exp_hist, reach = 0, np.zeros(64, dtype=np.int64), {}
        for t, ts in enumerate(wl.topics):
            rp, cl = O.parents_to_csr(parents[t])
            tot, oh, hist = O.disseminate(rp, cl, ts.root, live, 1, hist_len=64)
            exp_total += tot * int(cnt[t])
            exp_hist += hist.astype(np.int64) * int(cnt[t])
            reach[t] = oh[0] != 0xFF
        assert st.deliveries == exp_total
        assert st.duplicates == 0
        per = st.as_dict()["deliveries_per_round"]
        assert per[1:] == [int(x) for x in exp_hist[1:len(per)]]
        rng = np.random.default_rng(5)
        for t in (0, 8, 63):
            idx = np.nonzero(wl.msg_topics == t)[0]
            for m in rng.choice(idx, size=min(16, len(idx)), replace=False):
                got = eng.delivered(first + int(m))
                assert np.array_equal(got.astype(bool), reach[t]), (t, int(m))


@pytest.mark.parametrize("chain", [False, True])
def test_cfg3_topology_dead_mask_hops_record_instance(chain):
    """The cfg3 topology (1M peers, 64 topics) with the same dead mask, a
    1,200-message Zipf burst in recording mode: (peer, message, hop) of 16
    sampled messages per topic class equal or_disseminate's.  chain: the
    plan pinned to the production kernel -- flood = 0,
    k_pull_chain launches from round 1 (the recording variant of the
    headline's kernel at full topology size)."""
    wl = WL.cfg3()
    msgs = wl.msg_topics[:1200]
    plan = {"flood": 0} if chain else {}
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, record_hops=True, plan=plan) as eng:
        WL.build_engine_topics(eng, wl)
        parents = [eng.parents(t) for t in range(len(wl.topics))]
        live = _cfg3_dead_mask(wl, parents)
        eng.set_live(live)
        first = eng.publish(msgs)
        st = eng.run()
        if chain:
            kinds = list(st.round_kernel)
            assert st.expand_mode == PE.MODE_LEVEL_PULL and PE.K_FLOOD not in kinds
            assert kinds[1] == PE.K_CHAIN, kinds[:st.rounds + 1]  # chains from round 1
            assert sum(k == PE.K_CHAIN for k in kinds) >= 2  # more than one chain launch
        else:
            assert st.expand_mode == PE.MODE_FLOOD
        rng = np.random.default_rng(6)
        for t in (0, 8, 63):
            idx = np.nonzero(msgs == t)[0]
            if not len(idx):
                continue
            rp, cl = O.parents_to_csr(parents[t])
            _, oh, _ = O.disseminate(rp, cl, wl.topics[t].root, live, 1)
            for m in rng.choice(idx, size=min(16, len(idx)), replace=False):
                assert np.array_equal(eng.hops(first + int(m)), oh[0]), (t, int(m))


def test_flood_timeout_reruns_window_per_round(monkeypatch):
    """k_flood needs every wave resident; when they are not (another engine
    shares the GPU) a dependency wait times out.  flood_spin_ticks = 0
    forces that on a 40-level tree: the same window is re-run with per-round
    launches under a fresh generation (exact hops, counters and digest), and
    later windows keep the per-round launches.  An asynchronous run that times
    out reports PS_E_DEVICE from ps_wait and the next run is exact."""
    rng = np.random.default_rng(5)
    n = 3000
    parent = np.full(n, O.NONE, dtype=np.uint32)
    parent[1:] = np.maximum(0, np.arange(1, n) - 1 - rng.integers(0, 75, n - 1)).astype(np.uint32)
    live = (rng.random(n) > 0.03).astype(np.uint8)
    live[0] = 1
    rp, cl = O.parents_to_csr(parent)
    _, oh, _ = O.disseminate(rp, cl, 0, live, 1)
    n_msgs = 130
    opts = {"flood": 1, "overlap": 0, "flood_top_bytes": 1 << 40, "flood_spin_ticks": 0}
    with PE.Engine(n, 1, record_hops=True, plan=opts) as eng:
        eng.set_tree(0, 0, parent)
        eng.set_live(live)
        d0 = eng.depth(0)[0]
        assert d0 >= 20
        for rep in range(2):
            first = eng.publish(np.zeros(n_msgs))
            st = eng.run()
            assert st.expand_mode == PE.MODE_LEVEL_PULL, rep  # k_flood gave up
            assert st.windows == 1 and st.deliveries == n_msgs * int((oh[0][1:] != 0xFF).sum())
            for m in (0, 64, n_msgs - 1):
                assert np.array_equal(eng.hops(first + m), oh[0]), (rep, m)
    with PE.Engine(n, 1, plan={"flood_spin_ticks": 0}) as eng:
        eng.set_tree(0, 0, parent)
        eng.set_live(live)
        eng.publish(np.zeros(n_msgs))
        eng.run_async()
        with pytest.raises(PE.EngineError) as ei:
            eng.wait()
        assert "k_flood" in str(ei.value)
        first = eng.publish(np.zeros(n_msgs))
        st = eng.run()
        assert st.expand_mode == PE.MODE_LEVEL_PULL
        assert st.deliveries == n_msgs * int((oh[0][1:] != 0xFF).sum())
        got = eng.delivered(first + 7)
        assert np.array_equal(got.astype(bool), oh[0] != 0xFF)
