"""GPU: the churn path (BASELINE cfg5) -- joins, graceful
leaves with the restated repair and abrupt drops between publish batches,
with the node space rebuilt on the GPU (gbuild.hip) or on the host.

Parity: every message's hop per peer equals the CPU restatement's
(oracle/psoracle.c Tree.message) on the same operation sequence; the GPU
rebuild and the host build give identical hops, per-round deliveries and
seen digests.
"""
import os

import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


def make_engine(n, gpu_build, n_topics=1, **kw):
    """An engine whose node space is rebuilt on the GPU (default) or host."""
    return PE.Engine(n, n_topics, plan={"gpu_build": int(gpu_build)}, **kw)


@pytest.mark.parametrize("gpu_build", [True, False])
def test_cfg5_scaled_batches_match_oracle(gpu_build):
    """cfg5 shape at 20k peers: 90 % members, per batch 1 % leaves + 1 % joins,
    then a burst; messages of every batch checked against the oracle."""
    wl = WL.cfg5(20_000, batches=6, per_batch=70)
    plan = WL.churn_plan(wl, 6)
    seed = wl.seed
    eng = make_engine(wl.n_peers, gpu_build, record_hops=True, seed=seed)
    ot = O.Tree(wl.n_peers, 0, 2, 5, PE.Engine.topic_seed(seed, 0))
    WL.build_engine_topics(eng, wl)
    ot.join_all(wl.topics[0].join_order)
    for b, (leave, join) in enumerate(plan):
        for p in leave:
            assert ot.leave(int(p)) in (0, -3)  # an orphaned peer cannot Part
        try:
            eng.leave(0, leave)
        except PE.EngineError:
            pass
        st = eng.join(0, join, check=False)
        for p, s in zip(join, st):
            assert ot.join(int(p)) == s, (b, p)
        first = eng.publish(np.zeros(wl.n_msgs))
        run = eng.run()
        exp = ot.message()  # Part'ed peers receive nothing; the prune changes no hop
        for m in (0, wl.n_msgs // 2, wl.n_msgs - 1):
            assert np.array_equal(eng.hops(first + m), exp), (b, m)
        assert run.deliveries == wl.n_msgs * int((exp != 0xFF).sum())
        assert np.array_equal(eng.parents(0), ot.parents()), b
    eng.close()


def test_cfg5_pipelined_churn_matches_oracle():
    """bench.py's cfg5 loop: batch b's leaves and joins run on the host while
    batch b - 1's propagation is still in flight (ps_run_async / ps_wait, no
    hop record so the windows defer); every batch's deliveries equal the
    oracle's reach on the tree of that batch, and the trees stay the oracle's."""
    wl = WL.cfg5(20_000, batches=8, per_batch=70)
    plan = WL.churn_plan(wl, 8)
    eng = make_engine(wl.n_peers, True, seed=wl.seed)
    ot = O.Tree(wl.n_peers, 0, 2, 5, PE.Engine.topic_seed(wl.seed, 0))
    WL.build_engine_topics(eng, wl)
    ot.join_all(wl.topics[0].join_order)
    want, got = [], []
    for b, (leave, join) in enumerate(plan):
        for p in leave:
            ot.leave(int(p))
        try:
            eng.leave(0, leave)
        except PE.EngineError:
            pass
        st = eng.join(0, join, check=False)
        for p, s in zip(join, st):
            assert ot.join(int(p)) == s, (b, p)
        eng.publish(np.zeros(wl.n_msgs))
        eng.run_async()
        want.append(wl.n_msgs * int((ot.message() != 0xFF).sum()))
        if b:
            got.append(eng.wait().deliveries)
        assert np.array_equal(eng.parents(0), ot.parents()), b
    got.append(eng.wait().deliveries)
    assert got == want
    eng.close()


def test_gpu_and_host_builds_agree_under_drops():
    """Joins, leaves and abrupt drops (failed-write repairs in BFS order)
    interleaved with publishes: GPU rebuild == host build, message by message
    and in the seen digest."""
    rng = np.random.default_rng(17)
    n = 3000
    engs = [make_engine(n, g, record_hops=True, seed=4) for g in (True, False)]
    for e in engs:
        e.topic_create(0, 0, 2, 5)
        e.join(0, np.arange(1, n, 2))
    members = set(range(1, n, 2))
    for step in range(25):
        op = rng.random()
        if op < 0.3:
            outs = [p for p in range(1, n) if p not in members]
            peers = rng.choice(outs, size=min(20, len(outs)), replace=False)
            sts = [e.join(0, peers, check=False) for e in engs]
            assert np.array_equal(sts[0], sts[1])
            members |= {int(p) for p, s in zip(peers, sts[0]) if s == 0}
        elif op < 0.5:
            peers = rng.choice(sorted(members), size=15, replace=False)
            for e in engs:
                try:
                    e.leave(0, peers)
                except PE.EngineError:
                    pass
            members -= {int(p) for p in peers}
        elif op < 0.6:
            p = int(rng.choice(sorted(members)))
            for e in engs:
                try:
                    e.drop(0, [p])
                except PE.EngineError:
                    pass
            members.discard(p)
        k = int(rng.integers(1, 5))
        firsts = [e.publish(np.zeros(k)) for e in engs]
        sts = [e.run() for e in engs]
        assert sts[0].deliveries == sts[1].deliveries, step
        for m in range(k):
            assert np.array_equal(engs[0].hops(firsts[0] + m), engs[1].hops(firsts[1] + m)), (step, m)
        assert engs[0].seen_digest() == engs[1].seen_digest(), step
        assert engs[0].depth(0) == engs[1].depth(0), step
    for e in engs:
        e.close()


def test_gpu_build_multi_topic_and_live_mask():
    """cfg3 shape (scaled, 16 topics) with a live mask: the GPU-built fused
    node space delivers exactly what the host-built one does, per round."""
    wl = WL.cfg3(30_000, 16, 2000)
    live = (np.random.default_rng(2).random(wl.n_peers) > 0.05).astype(np.uint8)
    out = []
    for g in (True, False):
        e = make_engine(wl.n_peers, g, n_topics=len(wl.topics), seed=wl.seed)
        WL.build_engine_topics(e, wl)
        e.set_live(live)
        e.publish(wl.msg_topics)
        st = e.run()
        out.append((st.deliveries, st.as_dict()["deliveries_per_round"], e.seen_digest(),
                    [e.depth(t) for t in range(len(wl.topics))]))
        e.close()
    assert out[0] == out[1]


def test_gpu_build_prune_queries_shared_peers():
    """Three Join topics over the same peers, Parts in every topic, then
    joins: the lazy prune asks the GPU which Part'ed parents each topic's
    message reached (asked with the rebuild, gbuild.hip k_reach_query), and
    a peer of several topics must be judged in each topic's own tree -- the
    GPU-built engine's trees and deliveries equal the host-built engine's
    (whose prune walks the host trees) after every batch."""
    rng = np.random.default_rng(23)
    n = 5000
    engs = [make_engine(n, g, n_topics=3, seed=12) for g in (True, False)]
    members = []
    for t in range(3):
        m = np.sort(rng.choice(np.arange(1, n), size=3500, replace=False))
        members.append(set(int(x) for x in m))
        for e in engs:
            e.topic_create(t, 0, 2, 5)
            e.join(t, m)
    for step in range(8):
        for t in range(3):
            cur = sorted(members[t])
            leave = rng.choice(cur, size=60, replace=False)
            for e in engs:
                try:
                    e.leave(t, leave)
                except PE.EngineError:
                    pass
            members[t] -= {int(x) for x in leave}
        msgs = np.repeat(np.arange(3, dtype=np.uint32), 40)
        sts = []
        for e in engs:
            e.publish(msgs)
            sts.append(e.run_async() or e.wait())
        assert sts[0].deliveries == sts[1].deliveries, step
        for t in range(3):
            outs = [p for p in range(1, n) if p not in members[t]]
            join = rng.choice(outs, size=50, replace=False)
            res = [e.join(t, join, check=False) for e in engs]
            assert np.array_equal(res[0], res[1]), (step, t)
            members[t] |= {int(p) for p, s in zip(join, res[0]) if s == 0}
            assert np.array_equal(engs[0].parents(t), engs[1].parents(t)), (step, t)
    for e in engs:
        e.close()


def test_cfg5_full_size_batches_match_oracle():
    """BASELINE cfg5 at its stated size: 1M peers, 90 % members joined by the
    restated protocol, then batches of 1 % graceful leaves (Part + repair,
    subtree.go:46-98,356-375), 1 % joins (subtree.go:100-194) and a
    1,000-message burst, the node space rebuilt on the GPU every batch.  Each
    batch: the tree equals the restatement's, and the hops of sampled messages
    equal oracle Tree.message()'s (peer by peer, 1M peers)."""
    wl = WL.cfg5()
    batches = 4
    plan = WL.churn_plan(wl, batches)
    eng = make_engine(wl.n_peers, True, record_hops=True, seed=wl.seed)
    ot = O.Tree(wl.n_peers, 0, 2, 5, PE.Engine.topic_seed(wl.seed, 0))
    WL.build_engine_topics(eng, wl)
    ot.join_all(wl.topics[0].join_order)
    for b, (leave, join) in enumerate(plan):
        for p in leave:
            assert ot.leave(int(p)) in (0, -3)  # an orphaned peer cannot Part
        try:
            eng.leave(0, leave)
        except PE.EngineError:
            pass
        st = eng.join(0, join, check=False)
        exp_st = np.array([ot.join(int(p)) for p in join], dtype=np.int32)
        assert np.array_equal(st, exp_st), b
        first = eng.publish(wl.msg_topics)
        run = eng.run()
        exp = ot.message()
        assert run.deliveries == wl.n_msgs * int((exp != 0xFF).sum()), b
        for m in (0, 63, 64, 500, wl.n_msgs - 1):
            got = eng.hops(first + m)
            if not np.array_equal(got, exp):
                bad = np.nonzero(got != exp)[0][:8]
                raise AssertionError(f"batch {b} msg {m}: peers {bad} got {got[bad]} want {exp[bad]}")
        assert np.array_equal(eng.parents(0), ot.parents()), b
    eng.close()
