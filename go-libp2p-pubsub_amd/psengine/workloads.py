"""Synthetic workloads of BASELINE.json's configs.

All randomness is counter-based SplitMix64 (value i of the stream seeded with
``seed`` is ``mix64(seed + (i+1) * golden)``), so numpy, C and the GPU can
regenerate the same draws independently.

cfg1  16 peers, 1 topic "foobar", W=2/MaxW=5, 1000 paced publishes (CPU plumbing)
cfg2  100k peers, 1 topic, TreeOpts{8,20}, join order 1..N-1, 10k-message burst
cfg3  1M peers, 64 topics, root_k = k, peer p subscribes to topic k with
      Bernoulli(1/(k+1)); 100k messages, topic ~ Zipf(alpha=1) over 64
cfg4  16M peers, 1 topic, W=8/MaxW=20, 1k messages
cfg5  1M peers, 1 topic, W=2/MaxW=5, 100 batches x 1000 msgs with 1% leave /
      1% join churn between batches
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def mix64(x: np.ndarray) -> np.ndarray:
    """SplitMix64 output function applied to state ``x`` (already advanced)."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64)
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def stream(seed: int, idx: np.ndarray) -> np.ndarray:
    """Values ``idx`` (0-based) of the SplitMix64 stream seeded with ``seed``."""
    with np.errstate(over="ignore"):
        i = np.asarray(idx, dtype=np.uint64) + np.uint64(1)
        return mix64(np.uint64(seed) + i * GOLDEN)


def uniform(seed: int, idx: np.ndarray) -> np.ndarray:
    return (stream(seed, idx) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def owner(peers: np.ndarray, n_shards: int) -> np.ndarray:
    """owner(p) = splitmix64(p) mod G."""
    return (mix64(np.asarray(peers, dtype=np.uint64) + GOLDEN) % np.uint64(n_shards)).astype(np.int64)


@dataclass
class TopicSpec:
    root: int
    width: int
    max_width: int
    join_order: np.ndarray  # peers, in subscription order


@dataclass
class Workload:
    name: str
    n_peers: int
    topics: list[TopicSpec]
    msg_topics: np.ndarray  # topic of every published message, publish order
    seed: int
    notes: dict = field(default_factory=dict)

    @property
    def n_msgs(self) -> int:
        return int(self.msg_topics.shape[0])

    def expected_deliveries(self, sizes: list[int]) -> int:
        """Deliveries on static trees where topic t reaches sizes[t] subscribers."""
        counts = np.bincount(self.msg_topics, minlength=len(self.topics))
        return int(sum(int(counts[t]) * int(sizes[t]) for t in range(len(self.topics))))


def cfg1() -> Workload:
    return Workload("cfg1", 16, [TopicSpec(0, 2, 5, np.arange(1, 16, dtype=np.uint32))],
                    np.zeros(1000, dtype=np.uint32), 1)


def cfg2(n_peers: int = 100_000, n_msgs: int = 10_000) -> Workload:
    return Workload("cfg2", n_peers,
                    [TopicSpec(0, 8, 20, np.arange(1, n_peers, dtype=np.uint32))],
                    np.zeros(n_msgs, dtype=np.uint32), 2)


def zipf_topics(seed: int, n_msgs: int, n_topics: int) -> np.ndarray:
    w = 1.0 / np.arange(1, n_topics + 1, dtype=np.float64)
    cdf = np.cumsum(w / w.sum())
    u = uniform(seed ^ 0x5EED, np.arange(n_msgs))
    return np.minimum(np.searchsorted(cdf, u, side="right"), n_topics - 1).astype(np.uint32)


def cfg3(n_peers: int = 1_000_000, n_topics: int = 64, n_msgs: int = 100_000,
         seed: int = 3) -> Workload:
    topics = []
    peers = np.arange(n_peers, dtype=np.uint64)
    for k in range(n_topics):
        u = uniform(seed, peers * np.uint64(n_topics) + np.uint64(k))
        sub = (u < 1.0 / (k + 1)) & (peers >= n_topics)  # roots are peers 0..63
        topics.append(TopicSpec(k, 2, 5, peers[sub].astype(np.uint32)))
    return Workload("cfg3", n_peers, topics, zipf_topics(seed, n_msgs, n_topics), seed)


def cfg4(n_peers: int = 1 << 24, n_msgs: int = 1000) -> Workload:
    return Workload("cfg4", n_peers,
                    [TopicSpec(0, 8, 20, np.arange(1, n_peers, dtype=np.uint32))],
                    np.zeros(n_msgs, dtype=np.uint32), 4)


def cfg5(n_peers: int = 1_000_000, batches: int = 100, per_batch: int = 1000,
         members: float = 0.9, churn: float = 0.01) -> Workload:
    """Churn workload: peers 1..N-1 subscribe with probability `members` (join
    order = peer order); then `batches` batches, each preceded by churn_plan's
    leaves (churn x N current members, graceful Part) and joins (churn x N
    current non-members)."""
    peers = np.arange(1, n_peers, dtype=np.uint64)
    sub = uniform(5, peers) < members
    w = Workload("cfg5", n_peers, [TopicSpec(0, 2, 5, peers[sub].astype(np.uint32))],
                 np.zeros(per_batch, dtype=np.uint32), 5)
    w.notes = {"batches": batches, "per_batch": per_batch, "churn": churn}
    return w


def churn_plan(wl: Workload, batches: int, seed: int = 5):
    """Leave / join sets before each batch, from the generator's own member set
    (a peer that leaves is a non-member from then on; a join makes a member).
    The engine may refuse some (a leave of an orphaned peer): the plan does not
    depend on that, so it is computed up front, outside any timed region."""
    rng = np.random.default_rng(seed)
    n = wl.n_peers
    k = max(1, int(round(n * wl.notes["churn"])))
    member = np.zeros(n, dtype=bool)
    member[wl.topics[0].join_order] = True
    plan = []
    for _ in range(batches):
        ins = np.nonzero(member)[0]
        outs = np.nonzero(~member)[0]
        outs = outs[outs != wl.topics[0].root]
        leave = np.sort(rng.choice(ins, size=min(k, ins.size), replace=False)).astype(np.uint32)
        join = np.sort(rng.choice(outs, size=min(k, outs.size), replace=False)).astype(np.uint32)
        member[leave] = False
        member[join] = True
        plan.append((leave, join))
    return plan


CONFIGS = {"cfg1": cfg1, "cfg2": cfg2, "cfg3": cfg3, "cfg4": cfg4, "cfg5": cfg5}


def scaled(name: str, scale: float) -> Workload:
    """A smaller instance of a config (tests): peers and messages scaled."""
    if name == "cfg2":
        return cfg2(max(16, int(100_000 * scale)), max(1, int(10_000 * scale)))
    if name == "cfg3":
        return cfg3(max(256, int(1_000_000 * scale)), 64, max(64, int(100_000 * scale)))
    if name == "cfg4":
        return cfg4(max(16, int((1 << 24) * scale)), max(1, int(1000 * scale)))
    if name == "cfg5":
        return cfg5(max(256, int(1_000_000 * scale)), 100, max(16, int(1000 * scale)))
    return CONFIGS[name]()


def build_engine_topics(engine, wl: Workload) -> list[int]:
    """Creates the workload's topics on an engine and subscribes every peer in
    join order through the restated join protocol.  Returns tree sizes."""
    sizes = []
    for t, ts in enumerate(wl.topics):
        engine.topic_create(t, ts.root, ts.width, ts.max_width)
        if ts.join_order.size:
            engine.join(t, ts.join_order)
        sizes.append(int(ts.join_order.size))
    return sizes
