"""GPU: twin windows -- a pipelined window whose plan is
already on the device runs entirely beside its predecessor, on the other of
two streams and into the other of two row sets.  Every batch must deliver
exactly what blocking ps_run (and the engine with twins off, PSAMD_TWIN=0)
delivers; readbacks right after ps_run_async, churn (a node-space rebuild
while a twin is in flight), live-mask changes and plan changes between twins
must order correctly behind the window on the other stream."""
import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


def stats_key(st):
    d = st.as_dict()
    return (st.deliveries, st.duplicates, st.rounds, st.windows, tuple(d["deliveries_per_round"]))


def make(wl, monkeypatch, twin):
    if not twin:
        monkeypatch.setenv("PSAMD_AB", "1")
        monkeypatch.setenv("PSAMD_TWIN", "0")
    e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, plan={"flood": 0})  # (k_flood windows run no twins)
    monkeypatch.delenv("PSAMD_AB", raising=False)
    monkeypatch.delenv("PSAMD_TWIN", raising=False)
    WL.build_engine_topics(e, wl)
    return e


def vary(msg_topics, i):
    """Batch i: each topic drops up to (n_t - 1) % 64 of its last messages (its
    row width -- and so the plan -- stays; the last word differs)."""
    keep = np.ones(msg_topics.shape[0], dtype=bool)
    for t in np.unique(msg_topics):
        idx = np.nonzero(msg_topics == t)[0]
        drop = (i * 5 + int(t)) % ((idx.shape[0] - 1) % 64 + 1)
        if drop:
            keep[idx[-drop:]] = False
    return msg_topics[keep]


@pytest.mark.parametrize("staggered", [False, True])
def test_twin_windows_equal_blocking(monkeypatch, staggered):
    """12 pipelined batches with the plan unchanged (twins from the third
    window on) against blocking runs and the engine with twins off:
    per-batch stats, the seen digest and 6 delivered sets of the last batch."""
    wl = WL.cfg3(60_000, 16, 4000)
    starts = None
    if staggered:
        starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(5)).astype(np.uint32)
    batches = [vary(wl.msg_topics, i) for i in range(12)]
    if staggered:
        batches = [(b, starts[: b.shape[0]]) for b in batches]
    else:
        batches = [(b, None) for b in batches]
    out = []
    for mode in ("blocking", "twin", "no_twin"):
        e = make(wl, monkeypatch, mode != "no_twin")
        res, over = [], 0
        first = None
        if mode == "blocking":
            for b, s in batches:
                first = e.publish(b, s)
                res.append(stats_key(e.run()))
        else:
            for i, (b, s) in enumerate(batches):
                first = e.publish(b, s)
                e.run_async()
                if i:
                    st = e.wait()
                    res.append(stats_key(st))
                    over += st.overlapped
            st = e.wait()
            res.append(stats_key(st))
            over += st.overlapped
        n_last = batches[-1][0].shape[0]
        sets = [e.delivered(first + int(m)).copy() for m in np.linspace(0, n_last - 1, 6).astype(int)]
        out.append((res, e.seen_digest(), sets))
        if mode == "twin":
            assert over >= 6, over  # windows ran as twins
        e.close()
    for k in (1, 2):
        assert out[k][0] == out[0][0]
        assert out[k][1] == out[0][1]
        for a, b in zip(out[k][2], out[0][2]):
            assert np.array_equal(a, b)


def test_twin_readback_and_live_changes():
    """A tree of 4000 peers, 130 messages per batch: ps_read_delivered right
    after ps_run_async (the window may be a twin on the other stream), a
    live-mask change every third batch (the node flags a twin in flight still
    reads), against the restatement's reach every batch."""
    rng = np.random.default_rng(8)
    n = 4000
    parent = np.full(n, O.NONE, dtype=np.uint32)
    perm = rng.permutation(np.arange(1, n))
    order = np.concatenate([[0], perm])
    for i in range(1, n):
        parent[order[i]] = order[rng.integers(0, i)]
    rp, cl = O.parents_to_csr(parent)
    with PE.Engine(n, 1, plan={"flood": 0}) as e:
        e.set_tree(0, 0, parent)
        live = np.ones(n, dtype=np.uint8)
        pending = []
        over = 0
        for b in range(15):
            if b % 3 == 2:
                live = (rng.random(n) > 0.05).astype(np.uint8)
                live[0] = 1
                e.set_live(live)
            _, oh, _ = O.disseminate(rp, cl, 0, live, 1)
            reach = oh[0] != 0xFF
            first = e.publish(np.zeros(130))
            e.run_async()
            got = e.delivered(first + 129).astype(bool)
            assert np.array_equal(got, reach), b
            pending.append(130 * int(reach[1:].sum()))
            if len(pending) == 2:
                st = e.wait()
                over += st.overlapped
                assert st.deliveries == pending.pop(0), b
        while pending:
            assert e.wait().deliveries == pending.pop(0)
        assert over >= 4, over


def test_twin_windows_with_churn():
    """Joins and leaves between pipelined batches (a node-space rebuild while
    the previous window may still run on the other stream), with batches of
    unchanged plan in between: deliveries per batch equal the oracle's reach
    on that batch's tree, and the trees stay the oracle's."""
    wl = WL.cfg5(20_000, batches=10, per_batch=70)
    plan = WL.churn_plan(wl, 10)
    with PE.Engine(wl.n_peers, 1, seed=wl.seed, plan={"flood": 0}) as eng:
        ot = O.Tree(wl.n_peers, 0, 2, 5, PE.Engine.topic_seed(wl.seed, 0))
        WL.build_engine_topics(eng, wl)
        ot.join_all(wl.topics[0].join_order)
        want, got = [], []
        for b, (leave, join) in enumerate(plan):
            if b % 2 == 0:  # churn every other batch: the batch after it may run as a twin
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
        got.append(eng.wait().deliveries)
        assert got == want
        assert np.array_equal(eng.parents(0), ot.parents())
