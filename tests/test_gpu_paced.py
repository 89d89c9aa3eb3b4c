"""GPU: the PACED path at full size on a CUT tree.  Paced
publishing -- messages entering at start rounds 0..7, as pubsub_test.go's
publisher sleeps between publishes (/root/reference/pubsub_test.go:101-131)
-- is what bench.py's general_path times on cfg3.  Here it runs on BASELINE
cfg3 (1M peers, 64 Zipf topics) with ~2 % dead peers, including a child and a
grandchild of every root, so whole top subtrees are cut
(/root/reference/subtree.go:324-337: a dead child is skipped; its subtree
never hears the message), and is checked against the restatement
(oracle/psoracle.c or_disseminate), not against another schedule:

* the production instance, level-aligned start groups (the default plan):
  exact deliveries, the per-round histogram -- or_disseminate's per-topic
  histogram shifted by each message's start round -- and 16 sampled delivered
  sets per topic class (hot 0, mid 8, cold 63);
* the recording instance, 1,200 staggered messages, the plan pinned to
  level-aligned k_pull_chain launches: (peer, message, hop) of 16 sampled
  messages per class equal or_disseminate's (a hop counts from the message's
  own start, /root/reference/client.go:124-130);
* pipelined windows (ps_run_async, the next window's leading launches beside
  the previous window's last ones): every window's deliveries and histogram
  and the last window's sampled delivered sets against the oracle, and the
  overlap did happen.
"""
import numpy as np
import pytest

import psengine as PE
from fullsize_common import CLASSES, paced_starts
from psengine import workloads as WL

pytestmark = pytest.mark.gpu


def engine_on(wl, parents, live, **kw):
    eng = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed, **kw)
    for t, ts in enumerate(wl.topics):
        eng.set_tree(t, ts.root, parents[t])
    eng.set_live(live)
    return eng


def check_window(st, exp, msg_topics, starts):
    assert st.deliveries == exp.deliveries(msg_topics)
    assert st.duplicates == 0
    per = st.as_dict()["deliveries_per_round"]
    want = exp.per_round(msg_topics, starts, max(96, len(per)))
    assert per[1:] == [int(x) for x in want[1:len(per)]]
    assert int(want[len(per):].sum()) == 0


def sampled_ids(msg_topics, t, k=16, seed=5):
    idx = np.nonzero(msg_topics == t)[0]
    return np.random.default_rng(seed + t).choice(idx, size=min(k, len(idx)), replace=False)


def test_cfg3_paced_full_size_dead_mask(cfg3_cut):
    """Full cfg3, 100k messages over start rounds 0..7, production instance,
    the default level-aligned plan: deliveries, histogram and sampled
    delivered sets against the oracle."""
    wl, parents, live, exp = cfg3_cut
    starts = paced_starts(wl)
    with engine_on(wl, parents, live) as eng:
        first = eng.publish(wl.msg_topics, starts)
        st = eng.run()
        assert st.level_aligned and st.expand_mode == PE.MODE_LEVEL_PULL
        assert PE.K_CHAIN in set(st.round_kernel)
        check_window(st, exp, wl.msg_topics, starts)
        for t in CLASSES:
            for m in sampled_ids(wl.msg_topics, t):
                got = eng.delivered(first + int(m)).astype(bool)
                assert np.array_equal(got, exp.reach(t)), (t, int(m), int(starts[m]))


def test_cfg3_paced_recording_level_aligned_chains(cfg3_cut):
    """1,200 staggered messages in recording mode, the plan pinned to
    level-aligned chains (no k_flood): hops of 16 sampled messages per class
    equal or_disseminate's, hop counted from each message's start."""
    wl, parents, live, exp = cfg3_cut
    msgs = wl.msg_topics[:1200]
    starts = paced_starts(wl)[:1200]
    assert len(np.unique(starts)) == 8
    with engine_on(wl, parents, live, record_hops=True, plan={"align_groups": 1, "flood": 0}) as eng:
        first = eng.publish(msgs, starts)
        st = eng.run()
        kinds = list(st.round_kernel)
        assert st.level_aligned and PE.K_FLOOD not in kinds and PE.K_CHAIN in kinds, kinds[:40]
        check_window(st, exp, msgs, starts)
        for t in CLASSES:
            if not (msgs == t).any():
                continue
            for m in sampled_ids(msgs, t):
                got = eng.hops(first + int(m))
                if not np.array_equal(got, exp.hops[t]):
                    bad = np.nonzero(got != exp.hops[t])[0][:8]
                    raise AssertionError(f"topic {t} msg {m} start {starts[m]}: peers {bad} got {got[bad]} "
                                         f"want {exp.hops[t][bad]}")


def vary(msg_topics, starts, i):
    """Window i's batch: each topic drops a few of its last messages (the
    packed row widths, so the plan and the overlap, stay; group sizes and
    last row words change)."""
    keep = np.ones(msg_topics.shape[0], dtype=bool)
    for t in np.unique(msg_topics):
        idx = np.nonzero(msg_topics == t)[0]
        drop = (i * 7 + int(t)) % ((idx.shape[0] - 1) % 64 + 1)
        if drop:
            keep[idx[-drop:]] = False
    return msg_topics[keep], starts[keep]


def test_cfg3_paced_pipelined_windows_against_oracle(cfg3_cut):
    """Six pipelined paced windows (ps_run_async / ps_wait, the next window
    published and planned while the previous runs; level-aligned windows
    overlap their leading launches with the previous window's last): each
    window's deliveries and histogram, and the last window's sampled delivered
    sets, against the oracle -- not against a blocking run."""
    wl, parents, live, exp = cfg3_cut
    starts = paced_starts(wl)
    batches = [vary(wl.msg_topics, starts, i) for i in range(6)]
    with engine_on(wl, parents, live) as eng:
        out, firsts = [], []
        for i, (mt, st0) in enumerate(batches):
            firsts.append(eng.publish(mt, st0))
            eng.run_async()
            if i:
                out.append(eng.wait())
        out.append(eng.wait())
        for i, st in enumerate(out):
            assert st.level_aligned
            check_window(st, exp, *batches[i])
        assert eng.overlapped_windows() >= 3
        mt, _ = batches[-1]
        for t in CLASSES:
            for m in sampled_ids(mt, t, k=8):
                got = eng.delivered(firsts[-1] + int(m)).astype(bool)
                assert np.array_equal(got, exp.reach(t)), (t, int(m))
