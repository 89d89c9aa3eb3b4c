"""GPU: pipelined runs (ps_run_async / ps_wait) deliver exactly what blocking
ps_run does, batch by batch; readbacks stay stream-ordered behind runs in
flight; the engine refuses the calls that would break the pairing."""
import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


def stats_key(st):
    d = st.as_dict()
    return (st.deliveries, st.duplicates, st.rounds, st.windows, st.expand_bytes,
            tuple(d["deliveries_per_round"]))


def test_pipelined_equals_blocking_multi_topic():
    wl = WL.cfg3(50_000, 16, 3000)
    rng = np.random.default_rng(3)
    batches = [rng.permutation(wl.msg_topics)[: 1000 + 300 * b] for b in range(6)]
    out = []
    for pipelined in (False, True):
        e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
        WL.build_engine_topics(e, wl)
        res = []
        if pipelined:
            for i, b in enumerate(batches):
                e.publish(b)
                e.run_async()
                if i:
                    res.append(stats_key(e.wait()))
            res.append(stats_key(e.wait()))
        else:
            for b in batches:
                e.publish(b)
                res.append(stats_key(e.run()))
        out.append((res, e.seen_digest()))
        e.close()
    assert out[0] == out[1]


def test_readback_behind_run_in_flight():
    """ps_read_delivered right after ps_run_async sees that run's result (the
    readback is stream-ordered behind the kernels)."""
    rng = np.random.default_rng(5)
    n, root = 3000, 0
    perm = rng.permutation(np.arange(1, n))
    parent = np.full(n, O.NONE, dtype=np.uint32)
    order = np.concatenate([[root], perm])
    for i in range(1, n):
        parent[order[i]] = order[rng.integers(0, i)]
    live = (rng.random(n) > 0.2).astype(np.uint8)
    rp, cl = O.parents_to_csr(parent)
    _, hops, _ = O.disseminate(rp, cl, root, live, 1)
    with PE.Engine(n, 1) as e:
        e.set_tree(0, root, parent)
        e.set_live(live)
        first = e.publish(np.zeros(100))
        e.run_async()
        got = e.delivered(first + 37)  # before ps_wait
        exp = (hops[0] != 0xFF).astype(np.uint8)
        assert np.array_equal(got, exp)
        st = e.wait()
        assert st.deliveries == 100 * int(exp.sum())


def test_pairing_rules():
    with PE.Engine(64, 1) as e:
        e.topic_create(0, 0)
        e.join(0, np.arange(1, 64))
        with pytest.raises(PE.EngineError):
            e.wait()  # nothing in flight
        e.publish(np.zeros(10))
        e.run_async()
        e.publish(np.zeros(10))
        e.run_async()
        with pytest.raises(PE.EngineError):
            e.run_async()  # two in flight already
        with pytest.raises(PE.EngineError):
            e.run()  # blocking run while runs are pending
        assert e.wait().deliveries == 630
        assert e.wait().deliveries == 630
        e.publish(np.zeros(3))
        assert e.run().deliveries == 189


def test_async_with_hop_record_and_churn():
    """Runs that cannot defer (hop record) or that prune after the message
    (Parts) stay exact through the asynchronous entry points."""
    n = 500
    with PE.Engine(n, 1, record_hops=True, seed=9) as e:
        ot = O.Tree(n, 0, 2, 5, PE.Engine.topic_seed(9, 0))
        e.topic_create(0, 0, 2, 5)
        e.join(0, np.arange(1, n))
        ot.join_all(range(1, n))
        for step in range(4):
            leave = np.arange(10 + step, n, 37)
            try:
                e.leave(0, leave)
            except PE.EngineError:
                pass
            for p in leave:
                ot.leave(int(p))
            first = e.publish(np.zeros(20))
            e.run_async()
            st = e.wait()
            exp = ot.message()
            assert np.array_equal(e.hops(first), exp), step
            assert st.deliveries == 20 * int((exp != 0xFF).sum())


def reached_per_topic(e, wl, live):
    """Peers each topic's messages reach on the engine's trees under `live`
    (the restatement's BFS, one message per topic)."""
    out = []
    for t, ts in enumerate(wl.topics):
        rp, cl = O.parents_to_csr(e.parents(t))
        tot, _, _ = O.disseminate(rp, cl, ts.root, live, 1, want_hops=False)
        out.append(int(tot))
    return np.array(out, dtype=np.int64)


def expected_deliveries(msg_topics, reach):
    """Every message reaches its topic's reached peers (trees: no duplicates)."""
    return int((np.bincount(msg_topics, minlength=reach.shape[0]).astype(np.int64) * reach).sum())


def vary_counts(msg_topics, i):
    """Window i's batch: each topic loses up to (n_t - 1) % 64 of its last
    messages, so its row width ceil(n_t / 64) -- and the plan -- stays, while
    its last row word differs from window to window."""
    keep = np.ones(msg_topics.shape[0], dtype=bool)
    for t in np.unique(msg_topics):
        idx = np.nonzero(msg_topics == t)[0]
        drop = (i * 7 + int(t)) % ((idx.shape[0] - 1) % 64 + 1)
        if drop:
            keep[idx[-drop:]] = False
    return msg_topics[keep]


@pytest.mark.parametrize("dead,full", [(0.0, False), (0.03, False), (0.02, True)])
def test_overlapped_windows_equal_blocking(monkeypatch, dead, full):
    """Deep windows pipelined with the same plan: each window's leading
    launches run beside the previous window's last ones.
    Every run's counters and the final rows equal blocking runs, and the
    overlap did happen.  Small cases lower the window-size floor of the
    overlap; the full-size cfg3 case keeps the default.  Consecutive windows
    carry different message counts per topic (the same row widths, so the
    same plan and the overlap still applies), so their rows differ in every
    topic's last word: a launch reading rows its successor had already
    rewritten would change its own window's counters."""
    wl = WL.cfg3() if full else WL.cfg3(200_000, 16, 5000)
    rng = np.random.default_rng(11)
    live = (rng.random(wl.n_peers) >= dead).astype(np.uint8)
    live[[ts.root for ts in wl.topics]] = 1
    batches = [vary_counts(wl.msg_topics, i) for i in range(8)]
    assert len({b.shape[0] for b in batches}) > 4
    plan = {} if full else {"overlap_min_bytes": 0}
    out = []
    for pipelined in (False, True):
        e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, plan=plan)
        WL.build_engine_topics(e, wl)
        e.set_live(live)
        res = []
        if pipelined:
            for i in range(8):
                e.publish(batches[i])
                e.run_async()
                if i:
                    res.append(stats_key(e.wait()))
            res.append(stats_key(e.wait()))
            assert e.overlapped_windows() >= 5
        else:
            reach = reached_per_topic(e, wl, live)
            for i in range(8):
                e.publish(batches[i])
                res.append(stats_key(e.run()))
                # exact: a window with fewer messages than the one before must
                # not keep the old ones' bits in its root rows (rows wider
                # than 256 words: cfg3's hot topic)
                assert res[-1][0] == expected_deliveries(batches[i], reach), i
            assert e.overlapped_windows() == 0
            assert res[-1][2] >= 12  # a deep window (rounds)
        out.append((res, e.seen_digest()))
        e.close()
    assert out[0][0] == out[1][0]
    assert out[0][1] == out[1][1]


def vary_group_counts(msg_topics, starts, i):
    """Window i's staggered batch: each topic loses up to (n_t - 1) % 64 of
    its last messages (of whatever start rounds), so its packed row width
    ceil(n_t / 64) -- and the plan -- stays, while its start groups' sizes
    and its last row word change from window to window."""
    keep = np.ones(msg_topics.shape[0], dtype=bool)
    for t in np.unique(msg_topics):
        idx = np.nonzero(msg_topics == t)[0]
        drop = (i * 7 + int(t)) % ((idx.shape[0] - 1) % 64 + 1)
        if drop:
            keep[idx[-drop:]] = False
    return msg_topics[keep], starts[keep]


@pytest.mark.parametrize("dead,full", [(0.03, False), (0.02, True)])
def test_overlapped_staggered_windows_equal_blocking(monkeypatch, dead, full):
    """Paced publishing (start rounds 0..7), pipelined: level-aligned start
    groups make a deep window whose leading launches run beside the previous
    window's last ones.  Eight windows with different
    counts per (topic, start) group -- the same packed row widths, so the
    same plan and the overlap applies -- equal blocking runs counter for counter
    and in the final rows, and the blocking round-by-round schedule
    (align_groups 0) too; the overlap did happen."""
    wl = WL.cfg3() if full else WL.cfg3(200_000, 16, 5000)
    rng = np.random.default_rng(12)
    live = (rng.random(wl.n_peers) >= dead).astype(np.uint8)
    live[[ts.root for ts in wl.topics]] = 1
    starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(8)).astype(np.uint32)
    batches = [vary_group_counts(wl.msg_topics, starts, i) for i in range(8)]
    assert len({b[0].shape[0] for b in batches}) > 4
    base = {} if full else {"overlap_min_bytes": 0}
    out = []
    for pipelined, align in ((False, 1), (True, 1), (False, 0)):
        e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, plan={**base, "align_groups": align})
        WL.build_engine_topics(e, wl)
        e.set_live(live)
        res = []
        if pipelined:
            for i in range(8):
                e.publish(*batches[i])
                e.run_async()
                if i:
                    res.append(stats_key(e.wait()))
            res.append(stats_key(e.wait()))
        else:
            reach = reached_per_topic(e, wl, live)
            for i in range(8):
                e.publish(*batches[i])
                st = e.run()
                assert bool(st.level_aligned) == bool(align)
                assert st.deliveries == expected_deliveries(batches[i][0], reach), i
                res.append(stats_key(st))
            assert e.overlapped_windows() == 0
        out.append((res, e.seen_digest()))
        if pipelined:
            assert e.overlapped_windows() >= 5
        e.close()
    assert out[0][1] == out[1][1] == out[2][1]
    assert out[0][0] == out[1][0]
    # (expand_bytes, key index 4, differ by schedule: compare the rest)
    assert [k[:4] + k[5:] for k in out[0][0]] == [k[:4] + k[5:] for k in out[2][0]]


@pytest.mark.parametrize("reuse", [1, 0])
def test_signalled_windows_equal_blocking(monkeypatch, reuse):
    """Small pipelined windows (under the overlap floor, one rank) end with
    a pinned completion flag raised by the reduce instead of an event, and
    reuse the device copies of uploads that repeat.  Runs
    whose batches alternate between repeating and changing (same plan, new
    seeds; a new plan) give the blocking runs' counters and final rows, and
    the flag's timestamps a positive run time.  reuse=0 stages every upload."""
    monkeypatch.setenv("PSAMD_AB", "1")
    monkeypatch.setenv("PSAMD_UPLOAD_REUSE", str(reuse))
    wl = WL.cfg3(60_000, 8, 4000)
    rng = np.random.default_rng(5)
    live = (rng.random(wl.n_peers) >= 0.03).astype(np.uint8)
    live[[ts.root for ts in wl.topics]] = 1
    base = wl.msg_topics
    batches = [base, base, vary_counts(base, 1), vary_counts(base, 1), base[: base.shape[0] // 2], base,
               vary_counts(base, 3), base]
    out = []
    for pipelined in (False, True):
        e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
        WL.build_engine_topics(e, wl)
        e.set_live(live)
        res, ms = [], []
        if pipelined:
            for i, b in enumerate(batches):
                e.publish(b)
                e.run_async()
                if i:
                    st = e.wait()
                    res.append(stats_key(st))
                    ms.append(st.run_ms)
            st = e.wait()
            res.append(stats_key(st))
            ms.append(st.run_ms)
            assert all(m > 0 for m in ms), ms
            assert e.overlapped_windows() == 0
        else:
            for b in batches:
                e.publish(b)
                res.append(stats_key(e.run()))
        out.append((res, e.seen_digest()))
        e.close()
    assert out[0][0] == out[1][0]
    assert out[0][1] == out[1][1]


@pytest.mark.parametrize("fuse", [1, 0])
def test_held_back_reduce_orderings(monkeypatch, fuse):
    """A signalled window's reduce waits for the next window's first launch
    (k_window_turn) or for ps_wait.  Every order of the
    entry points -- wait right away, two in flight, a live-mask change and a
    readback between them, one-topic batches (no sort) beside mixed ones,
    batches published in several calls -- gives the blocking runs' counters
    and rows.  fuse=0: the reduce launches with its own window."""
    monkeypatch.setenv("PSAMD_AB", "1")
    monkeypatch.setenv("PSAMD_FUSE_REDUCE", str(fuse))
    wl = WL.cfg3(40_000, 6, 3000)
    rng = np.random.default_rng(17)
    live0 = np.ones(wl.n_peers, dtype=np.uint8)
    live1 = (rng.random(wl.n_peers) >= 0.05).astype(np.uint8)
    live1[[ts.root for ts in wl.topics]] = 1
    base = wl.msg_topics
    one = np.full(700, 2, dtype=np.uint32)        # one topic: identity order, no sort
    one_b = np.full(300, 4, dtype=np.uint32)
    # (op, arg): publish / publish2 (two calls) / async / wait / live / read
    script = [("publish", base), ("async", None), ("wait", None),
              ("publish", one), ("async", None), ("publish", base), ("async", None), ("wait", None), ("wait", None),
              ("publish", one), ("async", None), ("live", live1), ("publish2", (one, one_b)), ("async", None),
              ("wait", None), ("read", None), ("wait", None),
              ("publish", base[:1000]), ("async", None), ("publish", one), ("async", None), ("wait", None),
              ("live", live0), ("publish", one), ("async", None), ("wait", None), ("wait", None)]
    out = []
    for pipelined in (False, True):
        e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
        WL.build_engine_topics(e, wl)
        res, reads = [], []
        first = 0
        for op, arg in script:
            if op == "publish":
                first = e.publish(arg)
            elif op == "publish2":
                first = e.publish(arg[0])
                e.publish(arg[1])
            elif op == "live":
                e.set_live(arg)
            elif op == "async":
                if pipelined:
                    e.run_async()
                else:
                    res.append(stats_key(e.run()))
            elif op == "wait":
                if pipelined:
                    res.append(stats_key(e.wait()))
            elif op == "read":
                reads.append(e.delivered(first).tobytes())
        out.append((res, reads, e.seen_digest()))
        e.close()
    assert out[0][0] == out[1][0]
    assert out[0][1] == out[1][1]
    assert out[0][2] == out[1][2]
    # the batch published in two one-topic calls ran as one mixed batch (run 5
    # of the script): the same as publishing it in one call
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) as e:
        WL.build_engine_topics(e, wl)
        e.set_live(live1)
        e.publish(np.concatenate([one, one_b]))
        assert stats_key(e.run()) == out[0][0][4]
