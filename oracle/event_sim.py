"""Independent pure-Python restatement of go-libp2p-pubsub v0 (TEST INFRASTRUCTURE).

Only tests/, tests/golden/make_golden.py, ``__graft_entry__.smoke()`` and
bench.py's cpu_baseline leg may import this module.  It is the second, written-
from-scratch restatement used to cross-check ``oracle/psoracle.c`` and to emit
the committed fixtures under ``tests/golden/``.

It is deliberately shaped differently from the C restatement:

* the subscription tree is built by a message-level model of the join protocol
  -- ``handle_join`` answers with an ``Update`` whose ``peers`` field names the
  acceptor or the redirect target, and the joiner walks the redirects in
  ``join_parents`` exactly like subtree.go:241-307;
* dissemination is **asynchronous and event-driven**: every tree edge is a
  FIFO stream with a random per-message latency; a node delivers and then
  forwards (client.go:124-130).  Round-synchronous hop semantics (SURVEY.md F4:
  hop = depth, per-peer publish order) are therefore *checked*, not assumed.

Quiescent rules Q1-Q5 are the ones listed at the top of oracle/psoracle.c.
Parity of hop counts and tree shapes is unpinned by the reference itself (it has
no golden vectors); the reference's own test assertions are
restated in tests/golden/scenarios.json and checked against both restatements.
"""
from __future__ import annotations

import heapq
import random
from dataclasses import dataclass, field

MASK64 = (1 << 64) - 1
NONE = 0xFFFFFFFF

# MessageType, pubsub.go:138-145
DATA, JOIN, PART, UPDATE, STATE = range(5)


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & MASK64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & MASK64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)


@dataclass
class Child:
    """subtree.go:36-44 -- the parent's record of one child."""
    id: int
    size: int = 0
    children: list = field(default_factory=list)  # last State report
    dead: bool = False


@dataclass
class Subtree:
    """subtree.go:16-34 for one (host, topic)."""
    peer: int
    children: dict = field(default_factory=dict)  # insertion ordered, like Q2
    tree_width: int = 0
    tree_max_width: int = 0
    upstream: int | None = None  # the peer at the other end of `in`
    client_open: bool = True  # client.Close not called
    host_up: bool = True  # host.Close not called
    paused: bool = False


class Topic:
    """One topic tree rooted at ``root`` (TopicManager.NewTopic, pubsub.go:54-97)."""

    def __init__(self, n_peers: int, root: int, width: int = 2, max_width: int = 5,
                 seed: int = 1):
        self.n = n_peers
        self.root = root
        self.rng = SplitMix64(seed)
        self.subs: dict[int, Subtree] = {}
        r = Subtree(root, tree_width=width, tree_max_width=max_width)
        self.subs[root] = r
        self.orphans: set[int] = set()

    # -- join protocol ----------------------------------------------------
    def _handle_join(self, at: int, joiner: int, prio: bool) -> list[int]:
        """subtree.handleJoin: returns the Update's ``Peers`` field."""
        sub = self.subs[at]
        w = sub.tree_max_width if prio else sub.tree_width
        if len(sub.children) >= w:
            return self._redirect_join(sub)
        # welcome (subtree.go:121-132); child entry (149-152)
        sub.children[joiner] = Child(joiner)
        # State to our parent with NumPeers = sub.size = 0 (subtree.go:137-147)
        # a paused subscriber has dropped `in` (client.go:106) and sends no State
        if sub.upstream is not None and not sub.paused:
            parent = self.subs[sub.upstream]
            rec = parent.children.get(at)
            if rec is not None:
                rec.size = 0 + 1
                rec.children = [joiner]
        return [at]

    def _redirect_join(self, sub: Subtree) -> list[int]:
        """subtree.redirectJoin (subtree.go:156-194), ties per rule Q2."""
        if not sub.children:
            raise RuntimeError("called redirectJoin with no child peers")
        live = [c for c in sub.children.values() if not c.dead]
        if not live:
            raise RuntimeError("critical: failed to find child with minimum size")
        m = min(c.size for c in live)
        ties = [c for c in live if c.size == m]
        pick = ties[self.rng.next() % len(ties)] if len(ties) > 1 else ties[0]
        pick.size += 1
        return [pick.id]

    def _join_parents(self, joiner: int, talking_to: int, peers: list[int]) -> int:
        """subtree.joinParents (subtree.go:241-307); returns the new upstream."""
        for p in peers:
            if p == talking_to:
                return talking_to
            target = self.subs.get(p)
            if target is None or not target.host_up:
                raise ConnectionError("could not get connection to tree")
            welcome = self._handle_join(p, joiner, False)
            if not (len(welcome) == 1 and welcome[0] == p):
                return self._join_parents(joiner, p, welcome)
            return p
        raise ConnectionError("received zero parents from initiator")

    def subscribe(self, peer: int) -> None:
        """TopicManager.Subscribe (client.go:65-94)."""
        if peer == self.root or peer in self.subs:
            # still subscribed, orphaned, failed, or Part'ed but not yet pruned
            raise ValueError("already subscribed")
        rsub = self.subs[self.root]
        sub = Subtree(peer, tree_width=rsub.tree_width,
                      tree_max_width=rsub.tree_max_width)
        self.subs[peer] = sub
        try:
            reply = self._handle_join(self.root, peer, False)  # Topic.AddPeer
            sub.upstream = self._join_parents(peer, self.root, reply)
        except (ConnectionError, RuntimeError):
            del self.subs[peer]
            raise
        self.orphans.discard(peer)

    def _member(self, peer: int) -> bool:
        s = self.subs.get(peer)
        return s is not None and s.client_open and s.host_up

    # -- departures -------------------------------------------------------
    def _redistribute(self, at: int, gone: Child) -> None:
        """subtree.redistributeChildren (subtree.go:356-375), prio join."""
        gsub = self.subs.get(gone.id)
        rescued = gone.children[0] if gone.children else None
        if gsub is not None:
            for cid in list(gsub.children):
                if cid != rescued:
                    self._orphan(cid)
            gsub.children = {}
        if rescued is None:
            return
        rs = self.subs.get(rescued)
        if rs is None or not rs.client_open or not rs.host_up or rs.upstream != gone.id:
            return
        try:
            reply = self._handle_join(at, rescued, True)
            rs.upstream = self._join_parents(rescued, at, reply)
            rs.paused = False
        except (ConnectionError, RuntimeError):
            self._orphan(rescued)

    def _orphan(self, peer: int) -> None:
        s = self.subs.get(peer)
        if s is not None and s.client_open and s.host_up:
            s.paused = True
            self.orphans.add(peer)

    def leave(self, peer: int) -> None:
        """client.Close -> subtree.Close -> Part (client.go:30-34, subtree.go:78-98)."""
        sub = self.subs[peer]
        sub.client_open = False
        parent = self.subs.get(sub.upstream) if sub.upstream is not None else None
        # Part written to a closed host is lost (subtree.go:89-92)
        rec = parent.children.get(peer) if parent is not None and parent.host_up else None
        if rec is None:
            for cid in list(sub.children):
                self._orphan(cid)
            sub.children = {}
            return
        rec.dead = True  # handleChildMessages Part (subtree.go:62-70)
        self._redistribute(parent.peer, rec)

    def drop(self, peer: int) -> None:
        """host.Close(): abrupt, noticed at the parent's next write."""
        self.subs[peer].host_up = False

    # -- structure --------------------------------------------------------
    def _receives(self, peer: int) -> bool:
        s = self.subs[peer]
        return s.client_open and s.host_up and peer not in self.orphans

    def parents(self) -> list[int]:
        out = [NONE] * self.n
        stack = [self.root]
        while stack:
            p = stack.pop()
            for cid in self.subs[p].children:
                if self._receives(cid):
                    out[cid] = p
                    stack.append(cid)
        return out

    def child_lists(self) -> dict[int, list[int]]:
        return {p: list(s.children) for p, s in self.subs.items()}

    # -- dissemination ----------------------------------------------------
    def publish(self, payloads: list[bytes], rng: random.Random,
                pace: float = 0.0) -> list[list[tuple[int, int]]]:
        """Publish ``payloads`` (pace=0: burst) and run the asynchronous network
        to quiescence.  Returns, per peer, the list of (msg index, hop) in
        arrival order.  After each message's flood the lazy prune / repair of
        every forwarding node is applied (rule Q3)."""
        n = self.n
        got: list[list[tuple[int, int]]] = [[] for _ in range(n)]
        for mi, _payload in enumerate(payloads):
            events: list = []
            seq = 0
            busy: dict[tuple[int, int], float] = {}
            forwarded: list[int] = []

            def send(src, dst, t, hop):
                nonlocal seq
                # FIFO stream: never overtake the previous message on this edge
                at = max(t + rng.uniform(1.0, 10.0), busy.get((src, dst), 0.0) + 1e-9)
                busy[(src, dst)] = at
                heapq.heappush(events, (at, seq, dst, hop))
                seq += 1

            def forward(node, t, hop):  # subtree.forwardMessage
                forwarded.append(node)
                for cid, rec in self.subs[node].children.items():
                    cs = self.subs.get(cid)
                    if cs is None or not cs.host_up:
                        continue  # write fails (rule Q4)
                    if rec.dead or not cs.client_open or cid in self.orphans:
                        continue  # written into a closed client: not delivered
                    send(node, cid, t, hop + 1)

            forward(self.root, mi * pace, 0)
            while events:
                t, _, node, hop = heapq.heappop(events)
                got[node].append((mi, hop))  # cli.out <- m.Data (client.go:124)
                forward(node, t, hop)  # cli.sub.forwardMessage (client.go:130)
            self._after_message(forwarded)
        return got

    def _after_message(self, forwarded: list[int]) -> None:
        # BFS order of the forwarding nodes (rule Q3)
        order = self._bfs_order(set(forwarded))
        for p in order:
            sub = self.subs[p]
            failed = []
            for cid in list(sub.children):
                rec = sub.children[cid]
                if rec.dead:
                    del sub.children[cid]
                    gone = self.subs.get(cid)
                    if gone is not None and not gone.client_open:
                        del self.subs[cid]  # fully departed: may subscribe again
                    continue
                cs = self.subs.get(cid)
                if cs is not None and not cs.host_up:
                    del sub.children[cid]
                    failed.append(rec)
            for rec in failed:
                self._redistribute(p, rec)

    def _bfs_order(self, nodes: set[int]) -> list[int]:
        out = []
        q = [self.root]
        qi = 0
        seen = {self.root}
        while qi < len(q):
            p = q[qi]
            qi += 1
            if p in nodes:
                out.append(p)
            for cid in self.subs[p].children:
                if cid not in seen and cid in self.subs:
                    seen.add(cid)
                    q.append(cid)
        return out


def depths(parent: list[int], root: int) -> list[int]:
    """Hop of every attached peer (-1 = not attached)."""
    n = len(parent)
    d = [-1] * n
    d[root] = 0
    kids: dict[int, list[int]] = {}
    for c, p in enumerate(parent):
        if p != NONE:
            kids.setdefault(p, []).append(c)
    stack = [root]
    while stack:
        p = stack.pop()
        for c in kids.get(p, []):
            d[c] = d[p] + 1
            stack.append(c)
    return d


def build_join_tree(n_peers: int, root: int, width: int, max_width: int, seed: int,
                    order: list[int] | None = None) -> Topic:
    t = Topic(n_peers, root, width, max_width, seed)
    for p in (order if order is not None else [p for p in range(n_peers) if p != root]):
        t.subscribe(p)
    return t
