"""GPU: edge cases of the hot path -- empty runs and topics, a lone root,
ragged and exact 64-message words, a dead mask, window boundaries, and the
error behaviour of the ABI (closed topics, ids out of range).  Everything is
checked against the CPU restatement (oracle/psoracle.c or_disseminate) or an
exact count."""
import numpy as np
import pytest

import oracle as O
import psengine as PE

pytestmark = pytest.mark.gpu


def chain_and_star(n):
    """Peer 0 roots a star of its first children, then chains below."""
    parent = np.full(n, O.NONE, dtype=np.uint32)
    for p in range(1, n):
        parent[p] = 0 if p < 4 else p - 3
    return parent


def check(eng, first, n_msgs, parent, root, live):
    rp, cl = O.parents_to_csr(parent)
    tot, hops, _ = O.disseminate(rp, cl, root, live, n_msgs)
    for m in range(n_msgs):
        assert np.array_equal(eng.hops(first + m), hops[m]), m
    return tot


def test_run_with_nothing_published():
    with PE.Engine(32, 2, record_hops=True) as e:
        e.topic_create(0, 0)
        e.join(0, np.arange(1, 32))
        st = e.run()
        assert (st.deliveries, st.rounds, st.windows) == (0, 0, 0)
        with pytest.raises(PE.EngineError):
            e.peer_messages(0, 3)  # no window ran
        first = e.publish(np.zeros(5))
        assert e.run().deliveries == 5 * 31
        assert e.run().deliveries == 0  # nothing new
        e.publish(np.zeros(2))
        assert e.run().deliveries == 62
        assert e.hops(first + 5)[0] == 0xFF  # the root is not a recipient


def test_lone_root_and_empty_topic():
    with PE.Engine(1, 1, record_hops=True) as e:  # a network of one host
        e.topic_create(0, 0)
        first = e.publish(np.zeros(7))
        st = e.run()
        assert st.deliveries == 0 and e.hops(first).tolist() == [0xFF]
    with PE.Engine(50, 3, record_hops=True) as e:
        e.topic_create(0, 0)  # no subscribers
        e.topic_create(2, 9)
        e.join(2, np.arange(10, 50))
        first = e.publish(np.array([0, 2, 0, 2, 2]))
        st = e.run()
        assert st.deliveries == 3 * 40
        assert (e.hops(first) == 0xFF).all()


@pytest.mark.parametrize("n_msgs", [1, 63, 64, 65, 127, 128, 129, 640, 641])
def test_ragged_and_exact_words(n_msgs):
    rng = np.random.default_rng(n_msgs)
    n = 700
    parent = chain_and_star(n)
    live = (rng.random(n) > 0.05).astype(np.uint8)
    live[0] = 1
    with PE.Engine(n, 1, record_hops=True) as e:
        e.set_tree(0, 0, parent)
        e.set_live(live)
        first = e.publish(np.zeros(n_msgs))
        st = e.run()
        assert st.deliveries == check(e, first, n_msgs, parent, 0, live)


def test_dead_mask_and_dead_root_children():
    n = 200
    parent = chain_and_star(n)
    with PE.Engine(n, 1, record_hops=True) as e:
        e.set_tree(0, 0, parent)
        e.set_live(np.zeros(n, dtype=np.uint8))  # the root forwards regardless
        e.publish(np.zeros(10))
        assert e.run().deliveries == 0
        live = np.ones(n, dtype=np.uint8)
        live[1:4] = 0  # every child of the root
        e.set_live(live)
        e.publish(np.zeros(10))
        assert e.run().deliveries == 0


@pytest.mark.parametrize("extra", [-1, 0, 1])
def test_window_boundary(extra):
    """msg_window - 1, msg_window and msg_window + 1 messages of one topic:
    one or two windows, every message exact (the last window is readable
    through ps_read_delivered, the hop record covers all)."""
    win = 256
    n = 300
    parent = chain_and_star(n)
    live = np.ones(n, dtype=np.uint8)
    k = win + extra
    with PE.Engine(n, 1, record_hops=True, msg_window=win) as e:
        e.set_tree(0, 0, parent)
        first = e.publish(np.zeros(k))
        st = e.run()
        assert st.windows == (2 if k > win else 1)
        assert st.deliveries == check(e, first, k, parent, 0, live)
        assert e.delivered(first + k - 1).sum() == n - 1
        if k > win:
            with pytest.raises(PE.EngineError):
                e.delivered(first)  # an earlier window: not resident any more


def test_abi_error_behaviour():
    with PE.Engine(20, 2) as e:
        e.topic_create(0, 0)
        with pytest.raises(PE.EngineError):
            e.topic_create(0, 1)  # exists
        with pytest.raises(PE.EngineError):
            e.topic_create(5, 0)  # slot out of range
        with pytest.raises(PE.EngineError):
            e.publish(np.array([1]))  # closed topic
        st = e.join(0, np.array([3, 3, 25 % 20]), check=False)
        assert st[0] == 0 and st[1] == -3  # joining twice: PS_E_STATE
        with pytest.raises(PE.EngineError):
            e.join(0, np.array([0]))  # the root
        e.topic_close(0)
        with pytest.raises(PE.EngineError):
            e.publish(np.array([0]))
        with pytest.raises(PE.EngineError):
            e.hops(0)  # no hop record on this engine


@pytest.mark.parametrize("n", [700, 5000])
@pytest.mark.parametrize("staggered", [False, True])
def test_deep_chain_beyond_255_hops(staggered, n):
    """Chains 700 and 5000 deep: more rounds than a hop byte holds and than
    the 4096 preallocated round rows.  Deliveries are exact; hops read back
    saturated at 254, as the restatement reports them; the host build takes
    over from the GPU rebuild (depth > 254)."""
    parent = np.full(n, O.NONE, dtype=np.uint32)
    parent[1:] = np.arange(n - 1)
    live = np.ones(n, dtype=np.uint8)
    k = 70
    starts = np.arange(k) % 3 if staggered else None
    with PE.Engine(n, 1, record_hops=True) as e:
        e.set_tree(0, 0, parent)
        first = e.publish(np.zeros(k), starts)
        st = e.run()
        assert st.deliveries == k * (n - 1)
        rp, cl = O.parents_to_csr(parent)
        _, hops, _ = O.disseminate(rp, cl, 0, live, 1)
        assert hops[0][300] == 254 and hops[0][200] == 200
        for m in (0, 1, k - 1):
            assert np.array_equal(e.hops(first + m), hops[0]), m
        assert e.depth(0) == (n - 1, n)


def test_wide_join_beyond_65535_children():
    """TreeWidth 70,000: the root takes every joiner directly
    (subtree.go:141-152).  The child count of a peer is a 32-bit field: a
    16-bit one wrapped at child 65,536 and dropped the spill list.
    The attached tree equals the oracle's restated joins, and a message reaches
    every member in one hop; a leave of the root's last child redistributes
    nothing (it has no children) and keeps the others."""
    n, w = 70_002, 70_000
    with PE.Engine(n, 1, record_hops=True, seed=3) as e:
        e.topic_create(0, 0, w, w)
        e.join(0, np.arange(1, n))
        par = e.parents(0)
        t = O.Tree(n, 0, w, w, PE.Engine.topic_seed(3, 0))
        t.join_all(range(1, n))
        assert np.array_equal(par, t.parents())
        assert (par[1:w + 1] == 0).all()
        first = e.publish(np.zeros(3))
        st = e.run()
        assert st.deliveries == 3 * (n - 1)
        assert np.array_equal(e.hops(first), t.message())
        e.leave(0, np.array([w]))
        t.leave(w)
        assert np.array_equal(e.parents(0), t.parents())
