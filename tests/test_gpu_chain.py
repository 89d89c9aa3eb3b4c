"""k_pull_chain -- rounds q .. q + L - 1 (L = 3 .. 6) of a level window in
one launch: each wave writes a run of level-d nodes (its parents' rows from
HBM, kept in its LDS stage) and then every descendant of the run level by
level, each node copying the stage row its parent holds --
against the restatement (oracle/psoracle.c) and against one k_pull launch per
round (ps_plan_opts.chain_max = 1) and pair launches (chain_max = 2).

Round q delivers to BFS level q - s of each topic: a node receives its
parent's row of round q - 1 if the parent was reached this window and the
node is live (subtree.forwardMessage, subtree.go:319-354, the dead-child skip
at :326-331; client.processMessages, client.go:100-132).  Every schedule must
give the oracle's (peer, message, hop) exactly and the same per-round
counters and final seen state: recording and production instances, single
starts and start groups (a group entering inside a chain starts its own run
there), lazy and eager seen, rows wider than the stage (column slices), and
subtrees wider than the level tables (the plan falls back to pairs).
"""
import numpy as np
import pytest

import oracle as O
import psengine as PE
from test_gpu_pair import check_hops, make_case, oracle_hops, random_tree

pytestmark = pytest.mark.gpu


def run(monkeypatch, chain, n, topics, live, msg_topics, starts=None, record=True, flood=False, flags=0,
        msg_window=65536, waves=12):
    opts = {"chain_max": chain, "chain_max_groups": chain, "flood": int(flood), "chain_waves": waves}
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


def sweep(monkeypatch, n, topics, live, msg_topics, starts=None, chains=(1, 2, 3, 4, 6), records=(True, False),
          expect_chain=True, **kw):
    exp = oracle_hops(topics, live)
    ref = None
    for chain in chains:
        for record in records:
            st, kinds, hops, deliv, key = run(monkeypatch, chain, n, topics, live, msg_topics, starts, record=record,
                                              **kw)
            if chain >= 3 and expect_chain:
                assert PE.K_CHAIN in kinds and PE.K_CHAIN2 in kinds, kinds
            if chain == 1:
                assert PE.K_CHAIN not in kinds and PE.K_PAIR not in kinds
            if record:
                check_hops(hops, exp, msg_topics, f"chain={chain}")
            cur = (key, [x.tolist() for x in deliv])
            ref = ref or cur
            assert cur == ref, (chain, record)
            if chain >= 3 and not record:
                # no residency cap (ps_plan_opts.chain_waves = 0): the same
                # rows, counters and digest
                _, _, _, deliv0, key0 = run(monkeypatch, chain, n, topics, live, msg_topics, starts, record=False,
                                            waves=0, **kw)
                assert (key0, [x.tolist() for x in deliv0]) == ref, (chain, "no residency cap")
    return ref


@pytest.mark.parametrize("seed", range(6))
def test_chain_parity(monkeypatch, seed):
    """Random trees, several topics, ~15 % dead peers at every depth (a dead
    child of each root), ragged word counts."""
    rng = np.random.default_rng(1900 + seed)
    n, topics, live = make_case(rng)
    msg_topics = rng.integers(0, len(topics), size=int(rng.integers(1, 900))).astype(np.uint32)
    exp = oracle_hops(topics, live)
    key, _ = sweep(monkeypatch, n, topics, live, msg_topics)
    assert key[0] == sum(int((exp[t] != 0xFF).sum()) * int((msg_topics == t).sum()) for t in exp)


@pytest.mark.parametrize("n_msgs", [21000, 52000])
def test_chain_column_slices(monkeypatch, n_msgs):
    """Whole rows of 330 words (the hot topic of cfg3), and rows of 814 words,
    wider than the 768-word stage: each run is then written by one wave per
    column slice; the slices tile every row exactly, and only the slice-0
    wave counts nodes."""
    rng = np.random.default_rng(1950 + n_msgs)
    n = 3000
    topics = [(0, random_tree(rng, n, 0, 3)), (7, random_tree(rng, n, 7, 5))]
    live = (rng.random(n) > 0.05).astype(np.uint8)
    live[0] = live[7] = 1
    msg_topics = np.concatenate([np.zeros(n_msgs, dtype=np.uint32), np.ones(150, dtype=np.uint32)])
    rng.shuffle(msg_topics)
    sweep(monkeypatch, n, topics, live, msg_topics, records=(False,), chains=(1, 2, 4, 6), msg_window=1 << 16)
    # hops of every message through a recording run of the same rows: at
    # 52,000 messages the hot rows (814 words) are column-sliced, so the
    # recording slice variant (k_pull_chain<record, slices>) is checked too
    # 
    exp = oracle_hops(topics, live)
    st, kinds, hops, _, _ = run(monkeypatch, 4, n, topics, live, msg_topics, msg_window=1 << 16)
    assert PE.K_CHAIN in kinds
    check_hops(hops, exp, msg_topics, "chain=4 record")


@pytest.mark.parametrize("seed", range(4))
def test_chain_start_groups(monkeypatch, seed):
    """Start rounds 0..7 per message (group-major blocks): groups entering
    inside a chain launch run their level 1 there (r0 > 0)."""
    rng = np.random.default_rng(1970 + seed)
    n, topics, live = make_case(rng, 800, 3000, nt_hi=3, dead=0.1)
    msg_topics = rng.integers(0, len(topics), size=int(rng.integers(100, 1200))).astype(np.uint32)
    starts = rng.integers(0, 8, size=msg_topics.shape[0]).astype(np.uint32)
    sweep(monkeypatch, n, topics, live, msg_topics, starts)


def test_chain_fanout_heavy(monkeypatch):
    """Fan-out up to 24: runs of one node, or no chain where even one node's
    subtree is expected wider than the level tables."""
    rng = np.random.default_rng(1991)
    n = 30000
    topics = [(5, random_tree(rng, n, 5, 24)), (11, random_tree(rng, n, 11, 12))]
    live = (rng.random(n) > 0.05).astype(np.uint8)
    for r, _ in topics:
        live[r] = 1
    msg_topics = np.array([0] * 40 + [1] * 70 + [0] * 3000, dtype=np.uint32)  # W = 48 and W = 2
    sweep(monkeypatch, n, topics, live, msg_topics, chains=(1, 3, 4), expect_chain=False)


def test_chain_range_overflow_falls_back(monkeypatch):
    """A broom: level 2 of 200 nodes, one of which has 2,000 children and the
    others one each (the planner's average growth sizes a chain of rounds 2-4
    into runs of ~46 nodes, so the run holding the heavy node overflows a
    1,024-node level table): k_chain_ranges flags the plan and the window runs
    on pairs, with the same results."""
    n = 4000
    parent = np.full(n, O.NONE, dtype=np.uint32)
    parent[1:3] = 0                          # level 1: peers 1, 2
    parent[3:203] = np.repeat([1, 2], 100)   # level 2: 200 peers
    parent[203:2203] = 57                    # level 3: 2,000 children of peer 57 ...
    parent[2203:2402] = [x for x in range(3, 203) if x != 57]  # ... and one of every other
    parent[2402:] = np.arange(2402, n) - 2000  # level 4: one child each for 1,598 of them
    live = np.ones(n, dtype=np.uint8)
    live[5] = 0
    msg_topics = np.zeros(500, dtype=np.uint32)
    sweep(monkeypatch, n, [(0, parent)], live, msg_topics, chains=(1, 2, 4), expect_chain=False)
    st, kinds, _, _, _ = run(monkeypatch, 4, n, [(0, parent)], live, msg_topics, record=False)
    assert PE.K_CHAIN not in kinds and PE.K_PAIR in kinds, kinds


def test_chain_eager_seen(monkeypatch):
    """PS_F_NO_LAZY_SEEN: every generation stamped up front, every parent
    counts as reached for the counters, the same state."""
    rng = np.random.default_rng(1993)
    n, topics, live = make_case(rng, 1000, 3000, nt_hi=2, dead=0.2)
    msg_topics = rng.integers(0, len(topics), size=300).astype(np.uint32)
    sweep(monkeypatch, n, topics, live, msg_topics, chains=(1, 4, 6), records=(True,), flags=PE.F_NO_LAZY_SEEN)


@pytest.mark.parametrize("seed", range(2))
def test_chain_after_flood(monkeypatch, seed):
    """The default schedule: k_flood for the leading rounds, chains after
    (when the flood's byte budget leaves rounds over)."""
    rng = np.random.default_rng(1950 + seed)
    n, topics, live = make_case(rng, 20000, 40000, nt_hi=3, fan_lo=2, fan_hi=4, dead=0.03)
    msg_topics = rng.integers(0, len(topics), size=int(rng.integers(300, 3000))).astype(np.uint32)
    sweep(monkeypatch, n, topics, live, msg_topics, chains=(1, 4), flood=True, expect_chain=False)


def test_chain_deep_path_hops_past_255(monkeypatch):
    """A 600-deep chain of peers: 4- and 6-round launches only (flood 0); hops
    past 255 saturate at 254 as in the restatement."""
    n = 600
    parent = np.full(n, O.NONE, dtype=np.uint32)
    parent[1:] = np.arange(n - 1, dtype=np.uint32)
    live = np.ones(n, dtype=np.uint8)
    msg_topics = np.zeros(130, dtype=np.uint32)
    sweep(monkeypatch, n, [(0, parent)], live, msg_topics, chains=(1, 4, 6))


def test_chain_many_windows_and_drains(monkeypatch):
    """1,500 messages over two topics in 128-message windows with start
    groups: each subscriber's drain equals the per-round launches'."""
    rng = np.random.default_rng(1997)
    n, topics, live = make_case(rng, 1500, 2500, nt_hi=2, dead=0.08)
    msg_topics = rng.integers(0, len(topics), size=1500).astype(np.uint32)
    starts = rng.integers(0, 4, size=1500).astype(np.uint32)
    peers = [int(p) for p in rng.integers(0, n, size=12)]
    outs = []
    for chain in (1, 4, 6):
        opts = {"chain_max": chain, "chain_max_groups": chain, "flood": 0}
        with PE.Engine(n, len(topics), record_hops=True, msg_window=128, plan=opts) as eng:
            for t, (root, parent) in enumerate(topics):
                eng.set_tree(t, root, parent)
            eng.set_live(live)
            eng.publish(msg_topics, starts)
            st = eng.run()
            assert st.windows >= 6
            drains = [eng.peer_messages(t, p).tolist() for t in range(len(topics)) for p in peers]
            outs.append((st.deliveries, drains))
    assert outs[0] == outs[1] == outs[2]


def test_chain_direct_level0_wide_parent_span(monkeypatch):
    """a chain run of <= 64 nodes whose parents span more
    than 65,535 ids, with a level below it.  Level 2 holds 140,000 nodes and
    only its first and last have children (2 each), so the chain of rounds
    3-5 has one run of 4 nodes whose parents' span takes the direct level-0
    path; its level-0 metadata slot shares a register with level 1's.  The
    relative parent index (139,999) must not spill into level 1's half: the
    second level-3 node is dead, and a spilled bit would hand its children
    the live fourth node's row.  (Rounds 1-2 pair: the level-1 -> 2 growth of
    700 is wider than a chain's level tables.)"""
    from test_plan_cpu import wide_span_tree

    parent, _, _, l3 = wide_span_tree()
    l4 = l3 + 4
    n = parent.shape[0]
    live = np.ones(n, dtype=np.uint8)
    live[l3 + 1] = 0
    msg_topics = np.zeros(100, dtype=np.uint32)
    sweep(monkeypatch, n, [(0, parent)], live, msg_topics, chains=(1, 3, 4))
    for record in (True, False):
        st, kinds, hops, _, _ = run(monkeypatch, 4, n, [(0, parent)], live, msg_topics, record=record)
        assert kinds[1] == PE.K_PAIR and kinds[3] == PE.K_CHAIN, kinds
    exp = oracle_hops([(0, parent)], live)[0]
    assert exp[l4 + 2] == exp[l4 + 3] == 0xFF and exp[l4 + 6] == 4
