"""Helpers of the full-size GPU tests (test_gpu_fullsize.py, test_gpu_ipc.py):
the cut-tree dead mask, the oracle's reach and per-round histogram, the
run checks, and cfg4's tree (16,777,216 peers, TreeOpts{8,20}) built once per
session (conftest.py's `cfg4_tree` fixture)."""
import numpy as np

import oracle as O
import psengine as PE
from psengine import workloads as WL


def dead_mask(parent, root, n, frac=0.02, seed=17):
    rng = np.random.default_rng(seed)
    live = (rng.random(n) > frac).astype(np.uint8)
    kids = np.nonzero(parent == root)[0]
    live[kids[0]] = 0  # a child of the root: a whole top subtree is cut
    grand = np.nonzero(parent == kids[-1])[0]
    live[grand[0]] = 0
    live[kids[-1]] = 1
    live[root] = 1
    return live


def oracle_reach(parent, root, live):
    rp, cl = O.parents_to_csr(parent)
    tot, oh, hist = O.disseminate(rp, cl, root, live, 1, hist_len=64)
    return tot, oh[0] != 0xFF, hist.astype(np.int64)


def check_run(stats, n_msgs, tot, hist):
    """Deliveries, duplicates and the per-round histogram summed over ranks."""
    assert sum(int(s.deliveries) for s in stats) == tot * n_msgs
    assert sum(int(s.duplicates) for s in stats) == 0
    per = np.zeros(PE.MAX_ROUNDS, dtype=np.int64)
    for s in stats:
        per += np.array(list(s.deliveries_per_round), dtype=np.int64)
    assert per[1:64].tolist() == (hist[1:64] * n_msgs).tolist()
    assert int(per[64:].sum()) == 0


def sampled(n_msgs, k=16, seed=5):
    return np.random.default_rng(seed).choice(n_msgs, size=min(k, n_msgs), replace=False)


def cfg3_dead_mask(wl, parents, frac=0.02, seed=17):
    """~2 % dead peers, plus two dead peers in the top levels of every topic
    (a child of the root and a grandchild), roots live."""
    rng = np.random.default_rng(seed)
    live = (rng.random(wl.n_peers) > frac).astype(np.uint8)
    for t, ts in enumerate(wl.topics):
        par = parents[t]
        kids = np.nonzero(par == ts.root)[0]
        if len(kids):
            live[kids[0]] = 0
            grand = np.nonzero(par == kids[-1])[0]
            if len(grand):
                live[grand[0]] = 0
    for ts in wl.topics:
        live[ts.root] = 1
    return live


CLASSES = (0, 8, 63)  # cfg3 topic classes the paced tests sample: hot, mid, cold


def paced_starts(wl):
    return (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(8)).astype(np.uint32)


class Expect:
    """or_disseminate per topic on the cut trees: reached-peer counts, hop
    histograms and, for the sampled classes, the hops themselves."""

    def __init__(self, wl, parents, live):
        self.tot = np.zeros(len(wl.topics), dtype=np.int64)
        self.hist = np.zeros((len(wl.topics), 64), dtype=np.int64)
        self.hops = {}
        for t, ts in enumerate(wl.topics):
            rp, cl = O.parents_to_csr(parents[t])
            tot, oh, h = O.disseminate(rp, cl, ts.root, live, 1, want_hops=t in CLASSES, hist_len=64)
            self.tot[t] = tot
            self.hist[t] = h.astype(np.int64)
            if t in CLASSES:
                self.hops[t] = oh[0].copy()

    def deliveries(self, msg_topics):
        return int((np.bincount(msg_topics, minlength=self.tot.shape[0]).astype(np.int64) * self.tot).sum())

    def per_round(self, msg_topics, starts, n=96):
        """Message m reaches BFS level d in round starts[m] + d."""
        per = np.zeros(n, dtype=np.int64)
        for s0 in np.unique(starts):
            sel = starts == s0
            cnt = np.bincount(msg_topics[sel], minlength=self.tot.shape[0]).astype(np.int64)
            per[int(s0):int(s0) + 64] += cnt @ self.hist
        return per

    def reach(self, t):
        return (self.hops[t] != 0xFF) & (self.hops[t] > 0)


class Cfg4Tree:
    """cfg4's tree (the restated joins of 16M - 1 peers in order), its dead
    mask and the oracle's reach; the single engine's seen digest on demand."""

    def __init__(self):
        self.wl = WL.cfg4()
        with PE.Engine(self.wl.n_peers, 1, seed=self.wl.seed) as eng:
            WL.build_engine_topics(eng, self.wl)
            self.parent = eng.parents(0)
        self.live = dead_mask(self.parent, 0, self.wl.n_peers)
        self.tot, self.reach, self.hist = oracle_reach(self.parent, 0, self.live)
        assert self.reach.sum() < self.wl.n_peers - 1 - 0.02 * self.wl.n_peers  # subtrees were cut
        self._digest = None

    def astuple(self):
        return self.wl, self.parent, self.live, self.tot, self.reach, self.hist

    def digest(self):
        if self._digest is None:
            with PE.Engine(self.wl.n_peers, 1, seed=self.wl.seed) as one:
                one.set_tree(0, 0, self.parent)
                one.set_live(self.live)
                one.publish(self.wl.msg_topics)
                one.run()
                self._digest = one.seen_digest()
        return self._digest
