"""Start groups: tree windows whose messages enter at different rounds
(ps_publish_at, paced publishing as in pubsub_test.go:101-131) run level mode
-- one k_pull launch per round over each start group's word block -- and must
equal the restatement (oracle/psoracle.c) and the compaction path
(PS_F_COMPACT) exactly: hops, deliveries, per-round counts, seen digest and
the readbacks.

A message started at round s reaches a node of BFS level d in round s + d
(subtree.forwardMessage, subtree.go:319-354; client.processMessages,
client.go:100-132): each group is a single-start window of its own, laid out
as an even-length word block of every row of its topic.
"""
import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


def random_tree(rng, n, root, fan):
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


def run(level, n, topics, live, msg_topics, starts, record=True, plan=None):
    with PE.Engine(n, len(topics), record_hops=record, flags=0 if level else PE.F_COMPACT, plan=plan) as eng:
        for t, (root, parent) in enumerate(topics):
            eng.set_tree(t, root, parent)
        eng.set_live(live)
        first = eng.publish(msg_topics, starts)
        st = eng.run()
        if level:  # k_flood for the small leading rounds, k_pull after
            assert st.expand_mode in (PE.MODE_FLOOD, PE.MODE_LEVEL_PULL)
        else:
            assert st.expand_mode == PE.MODE_COMPACT
        hops = [eng.hops(first + m) for m in range(len(msg_topics))] if record else None
        deliv = [eng.delivered(first + m) for m in (0, len(msg_topics) // 2, len(msg_topics) - 1)]
        peer_msgs = [eng.peer_messages(t, (topics[t][0] + 1) % n).tolist() for t in range(len(topics))]
        return st, hops, deliv, peer_msgs, eng.seen_digest()


@pytest.mark.parametrize("seed", range(6))
def test_groups_match_oracle_and_compaction(monkeypatch, seed):
    """Several topics, start rounds 0..7 drawn per message (some topics with
    a single start), ~12 % dead peers: level mode with start groups and the
    compaction path both equal the oracle message by message, and leave the
    same counters, readbacks and seen digest."""
    rng = np.random.default_rng(300 + seed)
    n = int(rng.integers(400, 3000))
    nt = int(rng.integers(1, 5))
    topics = []
    for t in range(nt):
        root = int(rng.integers(0, n))
        topics.append((root, random_tree(rng, n, root, fan=int(rng.integers(2, 7)))))
    live = (rng.random(n) > 0.12).astype(np.uint8)
    for root, _ in topics:
        live[root] = 1
    n_msgs = int(rng.integers(2, 900))
    msg_topics = rng.integers(0, nt, size=n_msgs).astype(np.uint32)
    starts = rng.integers(0, 8, size=n_msgs).astype(np.uint32)
    if nt > 1:  # one topic single-start: a one-group topic beside grouped ones
        starts[msg_topics == nt - 1] = 3
    exp = {}
    for t, (root, parent) in enumerate(topics):
        rp, cl = O.parents_to_csr(parent)
        exp[t] = O.disseminate(rp, cl, root, live, 1)[1][0]
    outs = []
    # level mode: the default k_flood / k_pull split, every round in k_flood,
    # every round in k_pull -- level-aligned (the default, one launch
    # schedule over the BFS levels of every start group) and round by round
    # (align_groups 0); then the compaction path
    for level, opts in ((True, {}), (True, {"flood_top_bytes": 1 << 40}), (True, {"flood": 0}),
                        (True, {"align_groups": 0}), (True, {"align_groups": 0, "flood": 0}),
                        (True, {"chain_max": 1}), (True, {"chain_max": 2}), (False, {})):
        st, hops, deliv, pm, digest = run(level, n, topics, live, msg_topics, starts, plan=opts)
        for m, t in enumerate(msg_topics):
            if not np.array_equal(hops[m], exp[int(t)]):
                bad = np.nonzero(hops[m] != exp[int(t)])[0][:8]
                raise AssertionError(f"level={level} msg {m} start {starts[m]}: peers {bad} "
                                     f"got {hops[m][bad]} want {exp[int(t)][bad]}")
        assert st.duplicates == 0
        d = st.as_dict()
        outs.append((st.deliveries, st.rounds, d["deliveries_per_round"], digest,
                     [x.tobytes() for x in deliv], pm))
    assert all(o == outs[0] for o in outs)
    # per-round deliveries: message m reaches level d in round starts[m] + d
    per = np.zeros(64, dtype=np.int64)
    for m, t in enumerate(msg_topics):
        h = exp[int(t)]
        got = h[(h != 0xFF) & (h > 0)].astype(np.int64) + int(starts[m])
        np.add.at(per, got, 1)
    assert outs[0][2][1:] == [int(x) for x in per[1:len(outs[0][2])]]


def test_groups_production_instance_and_windows():
    """The non-recording instance, several windows per run (msg_window 200)
    and ragged group sizes (1..130 messages per start round): level mode and
    the compaction path leave the same deliveries, per-round counts and seen
    digest; delivered() readbacks equal the oracle."""
    rng = np.random.default_rng(77)
    n = 2500
    root = 11
    parent = random_tree(rng, n, root, fan=4)
    live = (rng.random(n) > 0.05).astype(np.uint8)
    live[root] = 1
    sizes = [1, 63, 64, 65, 130, 2, 127]
    starts = np.concatenate([np.full(k, s, dtype=np.uint32) for s, k in enumerate(sizes)])
    starts = starts[rng.permutation(len(starts))]
    msg_topics = np.zeros(len(starts), dtype=np.uint32)
    rp, cl = O.parents_to_csr(parent)
    exp = O.disseminate(rp, cl, root, live, 1)[1][0]
    outs = []
    for level, align in ((True, 1), (True, 0), (False, 1)):
        with PE.Engine(n, 1, msg_window=200, flags=0 if level else PE.F_COMPACT,
                       plan={"align_groups": align}) as eng:
            eng.set_tree(0, root, parent)
            eng.set_live(live)
            first = eng.publish(msg_topics, starts)
            st = eng.run()
            assert st.windows >= 2
            for m in (len(starts) - 1, len(starts) - 2, len(starts) - 50):  # the last window's
                assert np.array_equal(eng.delivered(first + m), ((exp != 0xFF) & (exp > 0)).astype(np.uint8))
            outs.append((st.deliveries, st.as_dict()["deliveries_per_round"], eng.seen_digest()))
    assert outs[0] == outs[1] == outs[2]
    assert outs[0][0] == len(starts) * int(((exp != 0xFF) & (exp > 0)).sum())


def test_cfg3_staggered_full_size():
    """BASELINE cfg3 at full size with start rounds uniform over 0..7 (the
    bench's general-path workload): level mode with start groups delivers
    exactly what the single-start window delivers, the per-round histogram
    is the single-start one shifted per group, and 16 sampled messages per
    topic class (hot 0, mid 8, cold 63) are delivered to exactly the tree.
    Level-aligned (the default: a deep window, chains from round 1, 21
    launch rounds for 28 rounds) and round by round (align_groups 0: k_flood
    for the leading rounds) leave the same counters and seen digest."""
    wl = WL.cfg3()
    starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(8)).astype(np.uint32)
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, plan={"align_groups": 0}) as eng:
        WL.build_engine_topics(eng, wl)
        eng.publish(wl.msg_topics, starts)
        st0 = eng.run()
        assert st0.expand_mode == PE.MODE_FLOOD and 0 < st0.flood_rounds < st0.rounds and not st0.level_aligned
        ref = (st0.deliveries, st0.rounds, st0.as_dict()["deliveries_per_round"], eng.seen_digest())
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) as eng:
        sizes = WL.build_engine_topics(eng, wl)
        first = eng.publish(wl.msg_topics, starts)
        st = eng.run()
        assert st.level_aligned and st.expand_mode == PE.MODE_LEVEL_PULL, (st.level_aligned, st.expand_mode)
        kinds = list(st.round_kernel)
        assert kinds[1] == PE.K_CHAIN and PE.K_FLOOD not in kinds, kinds[:30]
        assert (st.deliveries, st.rounds, st.as_dict()["deliveries_per_round"], eng.seen_digest()) == ref
        assert st.deliveries == wl.expected_deliveries(sizes) == 34_354_202_750
        assert st.duplicates == 0
        hist = np.zeros(80, dtype=np.int64)
        ones = np.ones(wl.n_peers, np.uint8)
        members = {}
        for t in (0, 8, 63):
            ts = wl.topics[t]
            members[t] = np.zeros(wl.n_peers, dtype=np.uint8)
            members[t][ts.join_order] = 1
        for t, ts in enumerate(wl.topics):
            rp, cl = O.parents_to_csr(eng.parents(t))
            _, _, h = O.disseminate(rp, cl, ts.root, ones, 1, want_hops=False, hist_len=64)
            for s0 in range(8):
                k = int(((wl.msg_topics == t) & (starts == s0)).sum())
                hist[s0:s0 + 64] += h.astype(np.int64) * k
        per = st.as_dict()["deliveries_per_round"]
        assert per[1:] == [int(x) for x in hist[1:len(per)]]
        for t in (0, 8, 63):
            ids = np.nonzero(wl.msg_topics == t)[0]
            for m in ids[np.linspace(0, len(ids) - 1, 16).astype(int)]:
                assert np.array_equal(eng.delivered(first + int(m)), members[t]), (t, m)
        # the compaction path (bench.py's general_path.compaction: arrival
        # extents for the 64..704-word rows of topics 0..6) on the same engine
        eng.set_flags(eng.flags | PE.F_COMPACT)
        first = eng.publish(wl.msg_topics, starts)
        st = eng.run()
        assert st.expand_mode == PE.MODE_COMPACT
        assert (st.deliveries, st.rounds, st.as_dict()["deliveries_per_round"], eng.seen_digest()) == ref
        for t in (0, 8):
            m = int(np.nonzero(wl.msg_topics == t)[0][-1])
            assert np.array_equal(eng.delivered(first + m), members[t]), (t, m)


@pytest.mark.parametrize("seed", range(4))
def test_compaction_extents_match_level(seed):
    """Compaction-path arrival extents (ExpandArgs::ext_cur): staggered tree
    topics whose rows are 64..704 words (each node receives one start group's
    block per round, so only that block of its arrival row is written and
    read), beside a narrow staggered topic, a single-start topic, a node with
    more than 64 children (the direct path consumes and produces extents) and
    dead peers; two windows per run.  Hops equal the oracle (recording
    instance) and the production instance leaves the same counters and seen
    digest as level mode."""
    rng = np.random.default_rng(900 + seed)
    n = int(rng.integers(1500, 3000))
    topics = []
    for t in range(3):
        root = int(rng.integers(0, n))
        parent = random_tree(rng, n, root, fan=int(rng.integers(2, 6)))
        if t == 0:  # a hub: > 64 children (deg > 64 entries take the direct path)
            hub = int(parent[int(rng.integers(0, n))])
            hub = hub if hub != O.NONE else root
            anc, x = set(), hub
            while x != O.NONE:
                anc.add(int(x))
                x = parent[x]
            movable = [v for v in rng.permutation(n) if int(v) not in anc][:90]
            parent[movable] = hub
        topics.append((root, parent))
    live = (rng.random(n) > 0.1).astype(np.uint8)
    for root, _ in topics:
        live[root] = 1
    # topic 0: 9000 messages over starts 0..7 (windows of 8000 messages: 8
    # groups of 12 or 8 words, W = 96 / 64); topic 1: 480 (W = 8 / 16);
    # topic 2: 4500 at one start
    msg_topics = np.concatenate([np.zeros(9000, np.uint32), np.ones(480, np.uint32),
                                 np.full(4500, 2, np.uint32)])
    starts = np.concatenate([rng.integers(0, 8, size=9480), np.full(4500, 2)]).astype(np.uint32)
    order = rng.permutation(len(msg_topics))
    msg_topics, starts = msg_topics[order], starts[order]
    exp = {}
    for t, (root, parent) in enumerate(topics):
        rp, cl = O.parents_to_csr(parent)
        exp[t] = O.disseminate(rp, cl, root, live, 1)[1][0]
    outs = []
    for level, record in ((True, False), (False, False), (False, True)):
        with PE.Engine(n, 3, record_hops=record, msg_window=8000, flags=0 if level else PE.F_COMPACT) as eng:
            for t, (root, parent) in enumerate(topics):
                eng.set_tree(t, root, parent)
            eng.set_live(live)
            first = eng.publish(msg_topics, starts)
            st = eng.run()
            assert st.windows >= 2 and st.duplicates == 0
            assert (st.expand_mode == PE.MODE_COMPACT) == (not level)
            if record:
                for m in list(rng.choice(len(msg_topics), 120, replace=False)) + [len(msg_topics) - 1]:
                    want = exp[int(msg_topics[m])]
                    got = eng.hops(first + int(m))
                    if not np.array_equal(got, want):
                        bad = np.nonzero(got != want)[0][:8]
                        raise AssertionError(f"msg {m} topic {msg_topics[m]} start {starts[m]}: peers {bad} "
                                             f"got {got[bad]} want {want[bad]}")
            outs.append((st.deliveries, st.as_dict()["deliveries_per_round"], eng.seen_digest()))
    assert outs[0] == outs[1] == outs[2]
    assert outs[0][0] == sum(int(((exp[int(t)] != 0xFF) & (exp[int(t)] > 0)).sum()) for t in msg_topics)
