"""GPU: BASELINE cfg2 and cfg4 at FULL size against the restatement with a
dead mask -- the single-rank production instance, and cfg4 (16,777,216 peers)
hash-sharded over 2, 4 and 8 loopback ranks under PS_PART_PEER, the north
star's 8-way split included, through the
zero-copy exchange and the RCCL-shaped copy path (PS_DIST_F_COPY).

A dead peer stops forwarding (subtree.go:324-337, the dead-child skip at
:326-331), so its subtree is cut: ~2 % dead peers, including a child of the
root and a grandchild, cut real subtrees out of the top levels.  Checked:

* the exact deliveries and the per-round histogram of or_disseminate
  (oracle/psoracle.c) times the message count -- every message of a
  single-start burst reaches the same peers at the same hops;
* the delivered peer sets of 16 sampled messages (ps_read_delivered, the
  union over ranks);
* the seen-state digest: the ranks' digests add up to the single engine's.
"""
import threading

import numpy as np
import pytest

import psengine as PE
from fullsize_common import check_run, dead_mask, oracle_reach, sampled
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfg4_tree(cfg4_full):
    return cfg4_full.astuple()


def test_cfg2_full_size_dead_mask_against_oracle():
    """cfg2 (100k peers, TreeOpts{8,20}, 10k burst) on the production
    instance: chain launches from round 1 (3 leading rounds are below
    ps_plan_opts.flood_min_rounds) at fan-out 8-20 with dead peers."""
    wl = WL.cfg2()
    with PE.Engine(wl.n_peers, 1, seed=wl.seed) as eng:
        WL.build_engine_topics(eng, wl)
        parent = eng.parents(0)
        live = dead_mask(parent, 0, wl.n_peers)
        tot, reach, hist = oracle_reach(parent, 0, live)
        eng.set_live(live)
        first = eng.publish(wl.msg_topics)
        st = eng.run()
        assert st.expand_mode == PE.MODE_LEVEL_PULL and PE.K_CHAIN in set(st.round_kernel)
        check_run([st], wl.n_msgs, tot, hist)
        for m in sampled(wl.n_msgs):
            assert np.array_equal(eng.delivered(first + int(m)).astype(bool), reach), int(m)


def test_cfg4_full_size_dead_mask_single_rank(cfg4_tree, cfg4_full):
    """cfg4 at full size on one rank, production instance, dead mask."""
    wl, parent, live, tot, reach, hist = cfg4_tree
    with PE.Engine(wl.n_peers, 1, seed=wl.seed) as eng:
        eng.set_tree(0, 0, parent)
        eng.set_live(live)
        first = eng.publish(wl.msg_topics)
        st = eng.run()
        assert st.expand_mode == PE.MODE_FLOOD
        assert {PE.K_PAIR, PE.K_CHAIN} & set(st.round_kernel)  # multi-round launches ran
        check_run([st], wl.n_msgs, tot, hist)
        for m in sampled(wl.n_msgs):
            assert np.array_equal(eng.delivered(first + int(m)).astype(bool), reach), int(m)
        assert eng.seen_digest() == cfg4_full.digest()


@pytest.mark.parametrize("world,copy", [(2, False), (2, True), (2, "inplace"), (4, False), (4, True), (4, "inplace"),
                                        (8, False), (8, True), (8, "inplace")])
def test_cfg4_full_size_ranks_peer_hash(cfg4_tree, cfg4_full, world, copy):
    """cfg4 at full size hash-sharded over `world` loopback ranks (owner(p) =
    splitmix64(p) mod world; 8 = the north star's split):
    every round ships ghost parent rows -- read in place, or (copy) through
    each receiver's buffer as RCCL moves them; deliveries, the per-round
    histogram, 16 sampled delivered sets (the union over the ranks) and the
    digest sum against the oracle and the single engine
    (subtree.go:324-337)."""
    wl, parent, live, tot, reach, hist = cfg4_tree
    lb = PE.Loopback(world)
    engines = [PE.Engine(wl.n_peers, 1, seed=wl.seed) for _ in range(world)]
    try:
        for r, e in enumerate(engines):
            e.dist_init_loopback(lb, r, PE.PART_PEER, copy=copy is True, inplace=copy == "inplace")
            e.set_tree(0, 0, parent)
            e.set_live(live)
        firsts = [e.publish(wl.msg_topics) for e in engines]
        stats = [None] * world
        errs = []

        def go(r):
            try:
                stats[r] = engines[r].run()
            except Exception as ex:  # noqa: BLE001
                errs.append((r, ex))

        th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in th), "rank thread hung"
        assert not errs, errs
        assert all(s.expand_mode == PE.MODE_LEVEL_PULL for s in stats)
        want = PE.XCHG_COPY if copy is True else PE.XCHG_IN_PLACE if copy == "inplace" else PE.XCHG_ZERO_COPY
        assert all(s.xchg_path == want and s.xchg_rounds > 0 for s in stats), [s.xchg_path for s in stats]
        check_run(stats, wl.n_msgs, tot, hist)
        own = PE.partition_owner(parent, 0, 0, world, PE.PART_PEER)
        for r in range(world):
            assert 0.9 / world < float((own == r).sum()) / float((own >= 0).sum()) < 1.1 / world
        for m in sampled(wl.n_msgs, seed=9):
            got = np.zeros(wl.n_peers, dtype=bool)
            for r, e in enumerate(engines):
                d = e.delivered(firsts[r] + int(m)).astype(bool)
                assert not (d & (own != r)).any()  # a rank reports its own nodes only
                got |= d
            assert np.array_equal(got, reach), int(m)
        digest = sum(e.seen_digest() for e in engines) % (1 << 64)
        assert digest == cfg4_full.digest()
    finally:
        for e in engines:
            e.close()
        lb.close()
