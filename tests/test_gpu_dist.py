"""GPU: the multi-GPU path (hash-partitioned nodes, per-round all-to-allv
exchange, apply kernel) on ONE GPU through the in-process loopback transport:
`world` engines in `world` threads, the real kernels and routing, device-to-
device copies in place of RCCL.  The union of the ranks' deliveries must equal
the CPU restatement's bit for bit."""
import threading

import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


def random_tree(rng, n, root=0):
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, O.NONE, dtype=np.uint32)
    for i in range(1, n):
        parent[perm[i]] = perm[rng.integers(0, i)]
    return parent


def run_ranks(engines):
    stats = [None] * len(engines)
    errs = []

    def go(r):
        try:
            stats[r] = engines[r].run()
        except Exception as ex:  # noqa: BLE001
            errs.append((r, ex))

    th = [threading.Thread(target=go, args=(r,)) for r in range(len(engines))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "rank thread hung"
    assert not errs, errs
    return stats


def make_ranks(world, n, n_topics, partition, split_depth=0, copy=False, **kw):
    """copy=True: the RCCL-shaped data path (PS_DIST_F_COPY: records through
    the receive buffer) instead of the zero-copy loopback reads; "inplace":
    no records below the roots, ghost-fed nodes read the owner's rows
    (PS_DIST_F_INPLACE)."""
    lb = PE.Loopback(world)
    engines = [PE.Engine(n, n_topics, record_hops=True, **kw) for _ in range(world)]
    for r, e in enumerate(engines):
        e.dist_init_loopback(lb, r, partition, split_depth, copy=copy is True, inplace=copy == "inplace")
    return lb, engines


def check_path(stats, copy):
    """Which transport path ran (ps_stats.xchg_path), on every rank."""
    want = PE.XCHG_COPY if copy is True else PE.XCHG_IN_PLACE if copy == "inplace" else PE.XCHG_ZERO_COPY
    assert all(st.xchg_rounds > 0 for st in stats), [st.xchg_rounds for st in stats]
    assert all(st.xchg_path == want for st in stats), [st.xchg_path for st in stats]


def merged_hops(engines, msg):
    h = np.stack([e.hops(msg) for e in engines])
    return h.min(axis=0)  # every peer is owned by exactly one rank per topic


@pytest.mark.parametrize("copy", [False, True, "inplace"])
@pytest.mark.parametrize("overlap", [0, 1])
@pytest.mark.parametrize("staggered", [True, False])
@pytest.mark.parametrize("world,partition", [(2, PE.PART_SUBTREE), (3, PE.PART_PEER),
                                             (4, PE.PART_SUBTREE), (4, PE.PART_PEER)])
def test_sharded_trees_match_oracle(world, partition, staggered, overlap, copy):
    """Level mode on N ranks, single start round and staggered starts (start
    groups: one word block per start round, each group's ghost records
    exchanged in its own rounds), with dead peers cutting subtrees across
    ranks; never the compaction path.  overlap=1: the
    exchange on its own stream beside the round's locally fed chunks, as RCCL
    runs it (the zero-copy loopback default is one stream).  copy: the records
    go through each receiver's buffer (PS_DIST_F_COPY) -- the RCCL transport's
    data path: send parts, receive buffer, exchange stream (VERDICT r3 item 1;
    subtree.go:333, client.go:103-131)."""
    rng = np.random.default_rng(world * 10 + partition + 100 * staggered)
    n, n_topics = 2500, 3
    lb, engines = make_ranks(world, n, n_topics, partition, copy=copy, plan={"xchg_overlap": overlap})
    trees = [random_tree(rng, n, int(rng.integers(0, n))) for _ in range(n_topics)]
    live = (rng.random(n) > 0.08).astype(np.uint8)
    topics = rng.integers(0, n_topics, size=150)
    starts = rng.integers(0, 4, size=150) if staggered else np.full(150, 2)
    for e in engines:
        for t in range(n_topics):
            e.set_tree(t, int(np.nonzero(trees[t] == O.NONE)[0][0]), trees[t])
        e.set_live(live)
    firsts = [e.publish(topics, starts) for e in engines]
    stats = run_ranks(engines)
    assert all(st.expand_mode == PE.MODE_LEVEL_PULL for st in stats), [st.expand_mode for st in stats]
    check_path(stats, copy)
    total = 0
    for t in range(n_topics):
        root = int(np.nonzero(trees[t] == O.NONE)[0][0])
        rp, cl = O.parents_to_csr(trees[t])
        idx = np.nonzero(topics == t)[0]
        tot, hops, _ = O.disseminate(rp, cl, root, live, len(idx))
        total += tot
        for k, m in enumerate(idx):
            assert np.array_equal(merged_hops(engines, firsts[0] + m), hops[k]), (t, m)
    assert sum(s.deliveries for s in stats) == total
    assert sum(s.duplicates for s in stats) == 0
    for e in engines:
        e.close()
    lb.close()


def test_sharded_join_trees_and_digest_sum():
    """cfg3-shaped (scaled): restated join trees on every rank, subtree
    partition; per-rank digests add up to the single-engine digest."""
    wl = WL.cfg3(20000, 8, 3000)
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) as one:
        sizes = WL.build_engine_topics(one, wl)
        one.publish(wl.msg_topics)
        st1 = one.run()
        d1 = one.seen_digest()
    world = 4
    lb = PE.Loopback(world)
    engines = [PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) for _ in range(world)]
    for r, e in enumerate(engines):
        e.dist_init_loopback(lb, r, PE.PART_SUBTREE)
        WL.build_engine_topics(e, wl)
        e.publish(wl.msg_topics)
    stats = run_ranks(engines)
    assert sum(s.deliveries for s in stats) == st1.deliveries == wl.expected_deliveries(sizes)
    assert sum(e.seen_digest() for e in engines) % (1 << 64) == d1
    for e in engines:
        e.close()
    lb.close()


def test_sharded_pipelined_batches():
    """Pipelined runs (ps_run_async / ps_wait) on 3 ranks: every batch's job
    total equals the single engine's, and the final digests add up."""
    wl = WL.cfg3(20000, 8, 2000)
    rng = np.random.default_rng(8)
    batches = [rng.permutation(wl.msg_topics)[: 500 + 250 * b] for b in range(5)]
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) as one:
        WL.build_engine_topics(one, wl)
        exp = []
        for b in batches:
            one.publish(b)
            exp.append(one.run().deliveries)
        d1 = one.seen_digest()
    world = 3
    lb = PE.Loopback(world)
    engines = [PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, msg_window=1 << 20)
               for _ in range(world)]
    for r, e in enumerate(engines):
        e.dist_init_loopback(lb, r, PE.PART_SUBTREE)
        WL.build_engine_topics(e, wl)
    got = [[] for _ in range(world)]
    errs = []

    def go(r):
        try:
            e = engines[r]
            for i, b in enumerate(batches):
                e.publish(b)
                e.run_async()
                if i:
                    got[r].append(e.wait().deliveries)
            got[r].append(e.wait().deliveries)
        except Exception as ex:  # noqa: BLE001
            errs.append((r, ex))

    th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "rank thread hung"
    assert not errs, errs
    assert [sum(g[i] for g in got) for i in range(len(batches))] == exp
    assert sum(e.seen_digest() for e in engines) % (1 << 64) == d1
    for e in engines:
        e.close()
    lb.close()


def test_sharded_churn_batches():
    """Joins and graceful leaves between batches on 2 ranks (host-built node
    space on every rank): per-batch job totals and digests equal the single
    engine's (GPU-built) on the same operation sequence."""
    wl = WL.cfg5(6000, batches=4, per_batch=90)
    plan = WL.churn_plan(wl, 4)

    def drive(e, b):
        leave, join = plan[b]
        try:
            e.leave(0, leave)
        except PE.EngineError:
            pass
        e.join(0, join, check=False)
        e.publish(np.zeros(wl.n_msgs))

    one = PE.Engine(wl.n_peers, 1, seed=wl.seed)
    WL.build_engine_topics(one, wl)
    exp = []
    for b in range(4):
        drive(one, b)
        exp.append((one.run().deliveries, one.seen_digest()))
    one.close()
    world = 2
    lb = PE.Loopback(world)
    engines = [PE.Engine(wl.n_peers, 1, seed=wl.seed) for _ in range(world)]
    for r, e in enumerate(engines):
        e.dist_init_loopback(lb, r, PE.PART_SUBTREE)
        WL.build_engine_topics(e, wl)
    for b in range(4):
        for e in engines:
            drive(e, b)
        stats = run_ranks(engines)
        got = (sum(s.deliveries for s in stats), sum(e.seen_digest() for e in engines) % (1 << 64))
        assert got == exp[b], b
    for e in engines:
        e.close()
    lb.close()


@pytest.mark.parametrize("copy", [False, True, "inplace"])
@pytest.mark.parametrize("world", [2, 4])
def test_cfg4_shaped_peer_partition(world, copy):
    """cfg4-shaped trees (TreeOpts{8,20} by the restated joins, scaled to
    200k peers) under the peer hash (the default partition),
    with ~3 % dead peers: every round ships ghost parents over the loopback
    transport; the ranks' deliveries and seen digests add up to the single
    engine's, and sampled messages' hops equal the restatement's."""
    wl = WL.cfg4(200_000, 300)
    rng = np.random.default_rng(40 + world)
    live = (rng.random(wl.n_peers) > 0.03).astype(np.uint8)
    live[0] = 1
    with PE.Engine(wl.n_peers, 1, seed=wl.seed) as one:
        WL.build_engine_topics(one, wl)
        par = one.parents(0)
        one.set_live(live)
        one.publish(wl.msg_topics)
        st1 = one.run()
        d1 = one.seen_digest()
    lb = PE.Loopback(world)
    engines = [PE.Engine(wl.n_peers, 1, seed=wl.seed, record_hops=True) for _ in range(world)]
    for r, e in enumerate(engines):
        e.dist_init_loopback(lb, r, copy=copy is True, inplace=copy == "inplace")  # PART_PEER by default
        WL.build_engine_topics(e, wl)
        e.set_live(live)
    firsts = [e.publish(wl.msg_topics) for e in engines]
    stats = run_ranks(engines)
    assert all(s.expand_mode == PE.MODE_LEVEL_PULL for s in stats)
    check_path(stats, copy)
    assert sum(s.deliveries for s in stats) == st1.deliveries
    assert sum(e.seen_digest() for e in engines) % (1 << 64) == d1
    rp, cl = O.parents_to_csr(par)
    _, hops, _ = O.disseminate(rp, cl, 0, live, 1)
    for m in (0, 150, 299):
        assert np.array_equal(merged_hops(engines, firsts[0] + m), hops[0]), m
    for e in engines:
        e.close()
    lb.close()


@pytest.mark.parametrize("world,partition", [(2, PE.PART_PEER), (4, PE.PART_PEER), (3, PE.PART_SUBTREE)])
def test_sharded_modes_agree(world, partition):
    """The same staggered batch on N ranks through level mode (start groups,
    the exchange beside the local chunks) and through the compaction path
    (PS_F_COMPACT): identical per-rank hops, deliveries and digests."""
    rng = np.random.default_rng(77 + world)
    n, n_topics = 4000, 2
    trees = [random_tree(rng, n, int(rng.integers(0, n))) for _ in range(n_topics)]
    live = (rng.random(n) > 0.05).astype(np.uint8)
    topics = rng.integers(0, n_topics, size=400)
    starts = rng.integers(0, 6, size=400)
    out = {}
    for flags in (0, PE.F_COMPACT):
        lb, engines = make_ranks(world, n, n_topics, partition, flags=flags)
        for e in engines:
            for t in range(n_topics):
                e.set_tree(t, int(np.nonzero(trees[t] == O.NONE)[0][0]), trees[t])
            e.set_live(live)
        firsts = [e.publish(topics, starts) for e in engines]
        stats = run_ranks(engines)
        assert all(st.expand_mode == (PE.MODE_COMPACT if flags else PE.MODE_LEVEL_PULL) for st in stats)
        out[flags] = ([merged_hops(engines, firsts[0] + m) for m in (0, 1, 199, 399)],
                      sum(st.deliveries for st in stats), sum(e.seen_digest() for e in engines) % (1 << 64))
        for e in engines:
            e.close()
        lb.close()
    a, b = out[0], out[PE.F_COMPACT]
    assert all(np.array_equal(x, y) for x, y in zip(a[0], b[0]))
    assert a[1:] == b[1:]
