"""GPU parity: the HIP hot path against the CPU restatement (oracle/).

Every test drives the engine through the C ABI (libpsengine.so) and compares
which peer received which message at which hop with oracle/psoracle.c on the
same inputs: bit-exact, no tolerance (integer work).  Reference semantics:
subtree.forwardMessage (subtree.go:319-354), client.processMessages
(client.go:100-132), Topic.PublishMessage (pubsub.go:111-120).
"""
import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


def random_tree(rng, n, root=0):
    """Random recursive tree over peers 0..n-1 rooted at `root` (labels shuffled)."""
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, O.NONE, dtype=np.uint32)
    for i in range(1, n):
        parent[perm[i]] = perm[rng.integers(0, i)]
    return parent


def random_mesh(rng, n, max_out=4):
    """Random directed graph with cycles: every peer gets 0..max_out children."""
    deg = rng.integers(0, max_out + 1, size=n)
    row_ptr = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(deg, out=row_ptr[1:])
    col = rng.integers(0, n, size=int(row_ptr[-1])).astype(np.uint32)
    return row_ptr, col


def engine_hops(eng, first, n_msgs):
    return np.stack([eng.hops(first + m) for m in range(n_msgs)]) if n_msgs else None


def check_topic(eng, first, msg_idx, row_ptr, col, root, live):
    """Compare engine hops of messages `msg_idx` (run-relative) with the oracle."""
    total, ohops, _ = O.disseminate(row_ptr, col, root, live, len(msg_idx))
    for k, m in enumerate(msg_idx):
        got = eng.hops(first + m)
        exp = ohops[k]
        if not np.array_equal(got, exp):
            bad = np.nonzero(got != exp)[0][:10]
            raise AssertionError(f"msg {m}: peers {bad} engine {got[bad]} oracle {exp[bad]}")
    return total


@pytest.mark.parametrize("level", [True, False])
@pytest.mark.parametrize("eager", [False, True])
@pytest.mark.parametrize("seed", range(8))
def test_tree_parity_random(seed, eager, level):
    """Odd seeds publish at staggered start rounds: level mode runs them as
    start groups, PS_F_COMPACT through the compaction path."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 3000))
    root = int(rng.integers(0, n))
    parent = random_tree(rng, n, root)
    live = (rng.random(n) > 0.1).astype(np.uint8)
    n_msgs = int(rng.integers(1, 300))
    starts = rng.integers(0, 6, size=n_msgs) if seed % 2 else None
    flags = (PE.F_NO_LAZY_SEEN if eager else 0) | (0 if level else PE.F_COMPACT)
    with PE.Engine(n, 1, record_hops=True, flags=flags) as eng:
        eng.set_tree(0, root, parent)
        eng.set_live(live)
        first = eng.publish(np.zeros(n_msgs), starts)
        st = eng.run()
        if not level:
            assert st.expand_mode == PE.MODE_COMPACT
        rp, cl = O.parents_to_csr(parent)
        total = check_topic(eng, first, list(range(n_msgs)), rp, cl, root, live)
        assert st.deliveries == total
        assert st.duplicates == 0


@pytest.mark.parametrize("level", [True, False])
@pytest.mark.parametrize("staggered", [False, True])
def test_wide_rows_parity(staggered, level):
    """Rows wider than the expand kernel's LDS stage (W > 704 words): staged
    slice by slice (expand_wide, PS_F_COMPACT); single-start and staggered
    (level mode: three start groups of ~268 words)."""
    rng = np.random.default_rng(40 + staggered)
    n = 600
    parent = random_tree(rng, n, 3)
    live = (rng.random(n) > 0.1).astype(np.uint8)
    n_msgs = 64 * 800 + 17  # W = 801 words: two slices
    starts = rng.integers(0, 3, size=n_msgs) if staggered else None
    with PE.Engine(n, 1, record_hops=True, flags=0 if level else PE.F_COMPACT) as eng:
        eng.set_tree(0, 3, parent)
        eng.set_live(live)
        first = eng.publish(np.zeros(n_msgs), starts)
        st = eng.run()
        assert st.expand_mode != PE.MODE_COMPACT if level else st.expand_mode == PE.MODE_COMPACT
        rp, cl = O.parents_to_csr(parent)
        # every message floods the same tree: hop = depth below the root
        _, hops, _ = O.disseminate(rp, cl, 3, live, 1)
        for m in list(range(0, n_msgs, 97)) + [n_msgs - 1]:
            assert np.array_equal(eng.hops(first + m), hops[0]), m
        assert st.deliveries == n_msgs * int((hops[0] != 0xFF).sum())
        assert st.duplicates == 0


@pytest.mark.parametrize("seed", range(6))
def test_mesh_parity_dedup(seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(2, 2000))
    rp, cl = random_mesh(rng, n, 1 + seed % 4)
    root = int(rng.integers(0, n))
    live = (rng.random(n) > 0.15).astype(np.uint8)
    n_msgs = int(rng.integers(1, 200))
    starts = rng.integers(0, 4, size=n_msgs) if seed % 2 else None
    with PE.Engine(n, 1, record_hops=True) as eng:
        eng.set_children(0, root, rp, cl)
        eng.set_live(live)
        first = eng.publish(np.zeros(n_msgs), starts)
        st = eng.run()
        total = check_topic(eng, first, list(range(n_msgs)), rp, cl, root, live)
        assert st.deliveries == total


def test_multi_topic_fused_and_windows():
    """Several topics (trees and meshes) fused in one launch, several windows."""
    rng = np.random.default_rng(7)
    n = 1500
    n_topics = 6
    graphs = []
    with PE.Engine(n, n_topics, record_hops=True, msg_window=128) as eng:
        for t in range(n_topics):
            root = int(rng.integers(0, n))
            if t % 3 == 2:
                rp, cl = random_mesh(rng, n, 3)
                eng.set_children(t, root, rp, cl)
            else:
                par = random_tree(rng, n, root)
                rp, cl = O.parents_to_csr(par)
                eng.set_tree(t, root, par)
            graphs.append((rp, cl, root))
        live = (rng.random(n) > 0.05).astype(np.uint8)
        eng.set_live(live)
        topics = rng.integers(0, n_topics, size=900)
        starts = rng.integers(0, 3, size=900)
        first = eng.publish(topics, starts)
        st = eng.run()
        assert st.windows > 1
        total = 0
        for t in range(n_topics):
            idx = list(np.nonzero(topics == t)[0])
            if idx:
                total += check_topic(eng, first, idx, *graphs[t], live)
        assert st.deliveries == total


def test_join_tree_matches_oracle_and_disseminates():
    n = 5000
    seed = 11
    with PE.Engine(n, 2, record_hops=True, seed=seed) as eng:
        for t, (w, mw) in enumerate([(2, 5), (8, 20)]):
            eng.topic_create(t, t, w, mw)
            order = np.array([p for p in range(n) if p != t], dtype=np.uint32)
            eng.join(t, order)
            ot = O.Tree(n, t, w, mw, PE.Engine.topic_seed(seed, t))
            ot.join_all(order)
            assert np.array_equal(eng.parents(t), ot.parents())
        first = eng.publish([0, 1, 1, 0, 1])
        eng.run()
        for k, t in enumerate([0, 1, 1, 0, 1]):
            ot = O.Tree(n, t, *[(2, 5), (8, 20)][t], PE.Engine.topic_seed(seed, t))
            ot.join_all([p for p in range(n) if p != t])
            assert np.array_equal(eng.hops(first + k), ot.message())


def test_churn_sequence_matches_oracle():
    """join / leave / drop interleaved with publishes: the
    message that meets a failed host is lost below it, the parent repairs."""
    rng = np.random.default_rng(5)
    n = 400
    seed = 9
    with PE.Engine(n, 1, record_hops=True, seed=seed, tree_width=2, tree_max_width=5) as eng:
        eng.topic_create(0, 0)
        ot = O.Tree(n, 0, 2, 5, PE.Engine.topic_seed(seed, 0))
        out = set(range(1, n))
        for step in range(60):
            op = rng.random()
            if op < 0.5 and out:
                peers = rng.choice(sorted(out), size=min(len(out), int(rng.integers(1, 20))),
                                   replace=False)
                st = eng.join(0, peers, check=False)
                for p, s in zip(peers, st):
                    assert ot.join(int(p)) == s
            elif op < 0.65:
                ins = [p for p in range(1, n) if ot.state(p) == O.IN]
                if ins:
                    p = int(rng.choice(ins))
                    eng.leave(0, [p])
                    ot.leave(p)
            elif op < 0.75:
                ins = [p for p in range(1, n) if ot.state(p) == O.IN]
                if ins:
                    p = int(rng.choice(ins))
                    eng.drop(0, [p])
                    ot.drop(p)
            else:
                k = int(rng.integers(1, 4))
                first = eng.publish(np.zeros(k))
                eng.run()
                for m in range(k):
                    assert np.array_equal(eng.hops(first + m), ot.message()), (step, m)
            out = {p for p in range(1, n) if ot.state(p) == O.OUT}
            assert np.array_equal(eng.parents(0), ot.parents()), step


def test_delivered_readback_and_no_record_mode():
    rng = np.random.default_rng(3)
    n = 3000
    par = random_tree(rng, n, 0)
    live = (rng.random(n) > 0.2).astype(np.uint8)
    with PE.Engine(n, 1) as eng:
        eng.set_tree(0, 0, par)
        eng.set_live(live)
        first = eng.publish(np.zeros(70))
        st = eng.run()
        rp, cl = O.parents_to_csr(par)
        total, hops, _ = O.disseminate(rp, cl, 0, live, 70)
        assert st.deliveries == total
        for m in (0, 63, 64, 69):
            assert np.array_equal(eng.delivered(first + m), (hops[m] != 0xFF).astype(np.uint8))


def _digest_full_tree(peers_in_tree, topic, n_msgs):
    """Host digest of a topic whose every node holds every message."""
    W = (n_msgs + 63) // 64
    words = np.full(W, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    if n_msgs % 64:
        words[-1] = np.uint64((1 << (n_msgs % 64)) - 1)
    g = WL.GOLDEN
    with np.errstate(over="ignore"):
        hw = WL.mix64(words + g)
        key = (peers_in_tree.astype(np.uint64)[:, None] << np.uint64(32)) | \
            (np.uint64(topic) << np.uint64(16)) | np.arange(W, dtype=np.uint64)[None, :]
        return int(WL.mix64((key ^ hw[None, :]) + g).sum(dtype=np.uint64))


def test_cfg2_full_size_properties():
    """BASELINE cfg2 at full size (100k peers, TreeOpts{8,20}, 10k burst):
    size-independent properties -- exact delivery count, per-hop histogram
    equal to level sizes x messages, no duplicates, seen-state digest."""
    wl = WL.cfg2()
    with PE.Engine(wl.n_peers, 1, seed=wl.seed) as eng:
        WL.build_engine_topics(eng, wl)
        par = eng.parents(0)
        eng.publish(wl.msg_topics)
        st = eng.run()
        assert st.deliveries == (wl.n_peers - 1) * wl.n_msgs == 999_990_000
        assert st.duplicates == 0
        rp, cl = O.parents_to_csr(par)
        _, _, hist = O.disseminate(rp, cl, 0, np.ones(wl.n_peers, np.uint8), 1, want_hops=False)
        per = st.as_dict()["deliveries_per_round"]
        assert per[1:] == [int(h) * wl.n_msgs for h in hist[1:len(per)]]
        assert eng.seen_digest() == _digest_full_tree(np.arange(wl.n_peers), 0, wl.n_msgs)


def test_cfg3_full_size_properties():
    """BASELINE cfg3 at full size (1M peers, 64 Zipf topics fused in one node
    space, 100k messages): exact deliveries, per-round histogram equal to
    sum_t msgs_t x level_t(r), no duplicates, digest of the seen state."""
    wl = WL.cfg3()
    with PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed) as eng:
        sizes = WL.build_engine_topics(eng, wl)
        eng.publish(wl.msg_topics)
        st = eng.run()
        assert st.deliveries == wl.expected_deliveries(sizes) == 34_354_202_750
        assert st.duplicates == 0
        cnt = np.bincount(wl.msg_topics, minlength=len(wl.topics))
        exp = np.zeros(64, dtype=np.int64)
        digest = 0
        ones = np.ones(wl.n_peers, np.uint8)
        for t, ts in enumerate(wl.topics):
            rp, cl = O.parents_to_csr(eng.parents(t))
            _, _, hist = O.disseminate(rp, cl, ts.root, ones, 1, want_hops=False, hist_len=64)
            exp += hist.astype(np.int64) * int(cnt[t])
            members = np.concatenate([[ts.root], ts.join_order]).astype(np.uint32)
            digest = (digest + _digest_full_tree(members, t, int(cnt[t]))) % (1 << 64)
        per = st.as_dict()["deliveries_per_round"]
        assert per[1:] == [int(x) for x in exp[1:len(per)]]
        assert int(exp[len(per):].sum()) == 0
        assert eng.seen_digest() == digest


def test_cfg4_full_size_properties():
    """BASELINE cfg4 at full size on one GPU (16,777,216 peers, TreeOpts{8,20}
    built by the restated join protocol and rebuilt on the GPU, 1k burst):
    exact deliveries, per-hop histogram, no duplicates, seen-state digest
    (host side summed in slices to bound memory)."""
    wl = WL.cfg4()
    with PE.Engine(wl.n_peers, 1, seed=wl.seed) as eng:
        WL.build_engine_topics(eng, wl)
        eng.publish(wl.msg_topics)
        st = eng.run()
        assert st.deliveries == (wl.n_peers - 1) * wl.n_msgs == 16_777_215_000
        assert st.duplicates == 0
        rp, cl = O.parents_to_csr(eng.parents(0))
        _, _, hist = O.disseminate(rp, cl, 0, np.ones(wl.n_peers, np.uint8), 1, want_hops=False)
        per = st.as_dict()["deliveries_per_round"]
        assert per[1:] == [int(h) * wl.n_msgs for h in hist[1:len(per)]]
        digest = 0
        for lo in range(0, wl.n_peers, 1 << 21):
            part = np.arange(lo, min(wl.n_peers, lo + (1 << 21)))
            digest = (digest + _digest_full_tree(part, 0, wl.n_msgs)) % (1 << 64)
        assert eng.seen_digest() == digest


def test_many_windows_generation_wrap_and_reuse():
    """> 255 windows on one engine: generation bytes wrap, stale rows from
    older windows never leak into a new window (lazy seen reset)."""
    rng = np.random.default_rng(21)
    n = 700
    par = random_tree(rng, n, 0)
    rp, cl = O.parents_to_csr(par)
    live = (rng.random(n) > 0.1).astype(np.uint8)
    with PE.Engine(n, 2, record_hops=True, msg_window=64) as eng:
        eng.set_tree(0, 0, par)
        eng.set_tree(1, 5, random_tree(rng, n, 5))
        eng.set_live(live)
        _, hops, _ = O.disseminate(rp, cl, 0, live, 1)
        for rep in range(3):
            k = 64 * 100 + 7  # 101 windows of topic 0 per run
            first = eng.publish(np.zeros(k), rng.integers(0, 3, size=k))
            st = eng.run()
            assert st.windows == 101
            for m in (0, 63, 64, 5000, k - 1):
                assert np.array_equal(eng.hops(first + m), hops[0]), (rep, m)
            assert st.deliveries == k * int((hops[0] != 255).sum())
