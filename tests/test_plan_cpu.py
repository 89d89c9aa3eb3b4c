"""CPU tests of the engine's launch planners through the host-only probe
(include/psengine_plan.h): the C++ planners build every rank's node space and
window plan exactly as ps_run does, and a Python emulator replays the level
mode from those tables alone -- chunks, round pairs, ghost records shipped by
the chunks that write the parents, root records packed, the per-round
all-to-allv regions, records read back by the ghost-fed nodes -- with the row
blocks as data.  The union of the ranks' deliveries must equal the CPU
restatement (oracle/psoracle.c), every node of every start group must be
written exactly once, and every reached node's block must equal its root's
(subtree.go:319-354, client.go:100-132).

The 2-rank case also runs in two gloo processes, the regions exchanged with
all_gather_object: the ghost layout tested on the CPU against a real
process boundary."""
import os
import socket

import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import plan as PL

MASK = (1 << 27) - 1
NONE = 0xFFFFFFFF
K_GROUPS = 8  # kTopicGroups


def random_tree(rng, n, root, fan=None):
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, O.NONE, dtype=np.uint32)
    kids = np.zeros(n, dtype=np.int64)
    for i in range(1, n):
        while True:
            p = perm[rng.integers(max(0, i - 40), i)] if fan else perm[rng.integers(0, i)]
            if not fan or kids[p] < fan:
                break
        parent[perm[i]] = p
        kids[p] += 1
    return parent


def root_block(t, gi, wn):
    r = np.random.default_rng(1000 * t + gi)
    b = r.integers(1, 1 << 63, size=wn, dtype=np.uint64)
    return b  # first word non-zero, as a group's first message bit is


class RankSim:
    """One rank of the level mode, driven by its plan tables only."""

    def __init__(self, plan: PL.Plan, live):
        self.p = plan
        self.info = plan.info()
        assert self.info["level"] == 1
        self.peer = plan.get(PL.NODES).astype(np.int64)
        self.parent = plan.get(PL.PARENT).astype(np.int64)
        self.gref = plan.get(PL.GHOST_REF).astype(np.int64)
        self.kind = plan.get(PL.ROUND_KIND).astype(np.int64)
        self.topics = [plan.topic(t) for t in range(plan.n_topics)]
        self.lay = [plan.layout(t) for t in range(plan.n_topics)]
        self.segs = plan.segs() if plan.world > 1 else []
        self.shipv = plan.ship() if plan.world > 1 else np.zeros((0, 2), np.int64)
        self.live = live
        wtot = 0
        for T, Ly in zip(self.topics, self.lay):
            wtot = max(wtot, Ly["wbase"] + T["n_nodes"] * Ly["W"])
        self.rows = np.zeros(wtot + 16, dtype=np.uint64)
        self.reached = np.zeros(self.info["nodes"], dtype=bool)
        self.writes = {}  # (node, group) -> times written
        self.send = np.zeros(3 * self.info["send_half"] + 16, dtype=np.uint64)  # kSendBufs parts
        self.recv = np.zeros(self.info["recv_words"] + 16, dtype=np.uint64)
        self.node_topic = np.zeros(self.info["nodes"], dtype=np.int64)
        self.level = np.zeros(self.info["nodes"], dtype=np.int64)
        for t, T in enumerate(self.topics):
            self.node_topic[T["nbase"]:T["nbase"] + T["n_nodes"]] = t
            lo = T["level_off"]
            for d in range(T["depth"] + 1):
                self.level[T["nbase"] + lo[d]:T["nbase"] + lo[d + 1]] = d
        # seeds: every owned root's blocks
        for t, (T, Ly) in enumerate(zip(self.topics, self.lay)):
            if T["root_local"] and T["n_nodes"] and Ly["W"]:
                self.reached[T["nbase"]] = True
                for gi, (_, w0, wn) in enumerate(Ly["groups"]):
                    r0 = self.block_row0(t, gi)
                    self.rows[r0:r0 + wn] = root_block(t, gi, wn)

    def block_row0(self, t, gi):
        Ly, T = self.lay[t], self.topics[t]
        _, w0, wn = Ly["groups"][gi]
        return Ly["wbase"] + (T["n_nodes"] * w0 if Ly["flags"] & K_GROUPS else 0)

    def row(self, c, u):
        nbase = self.topics[c["topic"]]["nbase"]
        a = c["row0"] + (u - nbase) * c["W"]
        return a, a + c["W"]

    def pack(self, q):
        for ps in self.p.pack(q):
            seg = self.segs[ps["gseg"]]
            for e in range(ps["e0"], ps["e1"]):
                _, dst = self.shipv[e]
                b, k = dst >> 27, dst & MASK
                a = seg["sbase"][b] + k * ps["W"]
                self.send[a:a + ps["W"]] = self.rows[ps["row"]:ps["row"] + ps["W"]]

    def regions_out(self, q):
        """{dest rank: words} of round q's send regions."""
        x = self.p.xchg(q)
        if not x["any"]:
            return {}
        half = (q % 3) * self.info["send_half"]
        out = {}
        for b in range(self.p.world):
            if b != self.p.rank:
                s0 = half + x["s_off"][b] // 8
                out[b] = self.send[s0:s0 + x["s_len"][b] // 8].copy()
        return out

    def regions_in(self, q, got):
        """got: {source rank: words}"""
        x = self.p.xchg(q)
        for a, w in got.items():
            assert w.shape[0] * 8 == x["r_len"][a], (q, a, w.shape[0] * 8, x["r_len"][a])
            r0 = x["r_off"][a] // 8
            self.recv[r0:r0 + w.shape[0]] = w

    def node_step(self, c, u, gin, cols=None):
        """Node u of chunk c receives its parent's block (columns cols =
        (w0, S) of it, chains; default the whole block): True if reached."""
        w0, S = cols if cols else (0, c["W"])
        p = self.parent[u]
        if p != NONE:
            pa, _ = self.row(c, p)
            up, src = self.reached[p], self.rows[pa + w0:pa + w0 + S]
        else:
            g = self.gref[u]
            assert g != NONE and gin != NONE, (u, g, gin)
            seg = self.segs[gin]
            assert seg["rw"] == c["W"]
            a = seg["rbase"][g >> 27] + (g & MASK) * c["W"]
            src = self.recv[a + w0:a + w0 + S]
            up = self.recv[a] != 0
        ok = bool(up and self.live[self.peer[u]])
        self.writes.setdefault((u, c["group"]), []).append((w0, S))
        if ok:
            ra, _ = self.row(c, u)
            self.rows[ra + w0:ra + w0 + S] = src
        if self.reached[u]:
            assert ok, u  # reach is the same for every start group (and column slice) of a tree
        self.reached[u] |= ok
        return ok

    def run_chain(self, q):
        """A k_pull_chain launch: per chunk its run (level d, round q + r0),
        then each level's children of the level above, column slice [w0, w0 + S)."""
        n, chunks = self.p.chain(q)
        assert n >= 3
        for c in chunks:
            L, S = c["levels"], c["S"]
            n0 = c["node_end"] - c["node_begin"]
            assert 1 <= L <= PL.CHAIN_LEVELS and c["r0"] + L <= n and 1 <= n0 <= 128
            assert S % 2 == 0 or S == c["W"]
            assert n0 * S <= 768, (n0, S, L)  # the LDS stage holds the run's rows (slices)
            assert c["first"][0] == self.topics[c["topic"]]["nbase"] + self.topics[c["topic"]]["level_off"][
                self.level[c["node_begin"]]]
            win_nodes = list(range(c["node_begin"], c["node_end"]))
            for u in win_nodes:
                self.node_step(c, u, NONE, (c["w0"], S))
            for k in range(1, L):
                kids = np.nonzero(np.isin(self.parent, np.asarray(win_nodes)))[0]
                if kids.shape[0]:
                    assert np.array_equal(kids, np.arange(kids[0], kids[-1] + 1)), "children not consecutive"
                    assert c["first"][k] <= kids[0] and kids[-1] < c["first"][k + 1]
                    # the kernel's range from row_ptr: the kids of the nodes of level k - 1 before this window
                    before = np.isin(self.parent, np.arange(c["first"][k - 1], win_nodes[0])).sum()
                    assert kids[0] == c["first"][k] + before
                for v in kids:
                    self.node_step(c, int(v), NONE, (c["w0"], S))
                win_nodes = [int(v) for v in kids]

    def ship(self, c, oks):
        if c["gout"] == NONE:
            assert c["e_lo"] == c["e_hi"] or self.p.world == 1
            return
        seg = self.segs[c["gout"]]
        for e in range(c["e_lo"], c["e_hi"]):
            node, dst = self.shipv[e]
            assert c["node_begin"] <= node < c["node_end"]
            b, k = dst >> 27, dst & MASK
            a = seg["sbase"][b] + k * c["W"]
            if oks[node]:
                ra, rb = self.row(c, node)
                self.send[a:a + c["W"]] = self.rows[ra:rb]
            else:
                self.send[a] = 0

    def chunks_of(self, q):
        k = self.kind[q] if q < self.kind.shape[0] else 0
        if k in (PE.K_PAIR2, PE.K_CHAIN2):
            return None
        return self.p.chunks(PL.PAIR if k == PE.K_PAIR else PL.PULL, q), k == PE.K_PAIR

    def run_round(self, q, part):
        """The chunks of round q: part 0 = locally fed, 1 = ghost-fed."""
        k = self.kind[q] if q < self.kind.shape[0] else 0
        if k == PE.K_CHAIN:
            if part == 0:
                self.run_chain(q)
            return
        r = self.chunks_of(q)
        if r is None:
            return
        (lo, split, hi, ch), pair = r
        sel = ch[:split - lo] if part == 0 else ch[split - lo:]
        for c in sel:
            oks = {}
            nodes = range(c["node_begin"], c["node_end"])
            if part == 0 and not pair:
                assert all(self.parent[u] != NONE or self.gref[u] == NONE for u in nodes)
            for u in nodes:
                oks[u] = self.node_step(c, u, c["gin"])
            if not pair:
                self.ship(c, oks)
                continue
            assert c["gout"] == NONE and c["e_lo"] == c["e_hi"]
            if c["c_lo"] == NONE:
                continue  # a level-1 run of the second round: no children in this launch
            # phase B: every child of the run, consecutive ids, from the run's rows
            kids = np.nonzero(np.isin(self.parent, np.arange(c["node_begin"], c["node_end"])))[0]
            if kids.shape[0]:
                assert np.array_equal(kids, np.arange(kids[0], kids[-1] + 1)), "children not consecutive"
            for v in kids:
                self.node_step(c, int(v), NONE)


def emulate(sims, q_max, exchange):
    for q in range(1, q_max + 1):
        for s in sims:
            s.pack(q)
        exchange(q)
        for part in (0, 1):
            for s in sims:
                s.run_round(q, part)


def in_process_exchange(sims):
    def go(q):
        outs = [s.regions_out(q) for s in sims]
        for b, s in enumerate(sims):
            if s.p.xchg(q)["any"]:
                s.regions_in(q, {a: outs[a][b] for a in range(len(sims)) if a != b})
    return go


def check(sims, trees, roots, live, n_groups):
    """Deliveries equal the restatement's; every node written once per group;
    every reached block equals its root's."""
    n = live.shape[0]
    for t, (par, root) in enumerate(zip(trees, roots)):
        rp, cl = O.parents_to_csr(par)
        _, oh, _ = O.disseminate(rp, cl, root, live, 1)
        exp = oh[0] != 0xFF
        got = np.zeros(n, dtype=bool)
        for s in sims:
            T = s.topics[t]
            Ly = s.lay[t]
            if not T["n_nodes"] or not Ly["W"]:
                continue
            for u in range(T["nbase"], T["nbase"] + T["n_nodes"]):
                if s.level[u] == 0:
                    continue
                for gi, (_, _, wn) in enumerate(Ly["groups"]):
                    cols = sorted(s.writes.get((u, gi), []))  # the column slices written: tile [0, W) once
                    pos = 0
                    for w0, S in cols:
                        assert w0 == pos, (t, u, gi, cols)
                        pos += S
                    assert pos == (wn if Ly["flags"] & K_GROUPS else Ly["W"]), (t, u, gi, cols)
                if s.reached[u]:
                    got[s.peer[u]] = True
                    for gi, (_, w0, wn) in enumerate(Ly["groups"]):
                        r0 = s.block_row0(t, gi) + (u - T["nbase"]) * wn
                        assert np.array_equal(s.rows[r0:r0 + wn], root_block(t, gi, wn)), (t, u, gi)
        assert np.array_equal(got, exp), (t, int((got != exp).sum()))
        if sims[0].info["aligned"]:  # level-aligned: one packed block, the start groups over its bits
            assert len(Ly["groups"]) == 1 and (len(Ly["aligned_groups"]) == n_groups[t] or not Ly["W"])
        else:
            assert len(Ly["groups"]) == n_groups[t] or not Ly["W"]


def build(world, partition, n=1500, n_topics=2, seed=0, fan=None):
    rng = np.random.default_rng(seed)
    roots = [int(x) for x in rng.choice(n, size=n_topics, replace=False)]
    trees = [random_tree(rng, n, r, fan) for r in roots]
    live = (rng.random(n) > 0.08).astype(np.uint8)
    for r in roots:
        live[r] = 1
    return rng, trees, roots, live


@pytest.mark.parametrize("chain", [2, 4, 6])
@pytest.mark.parametrize("staggered", [False, True])
@pytest.mark.parametrize("world,partition", [(1, PE.PART_PEER), (2, PE.PART_PEER), (3, PE.PART_PEER),
                                             (4, PE.PART_SUBTREE), (4, PE.PART_PEER)])
def test_plans_replay_to_the_oracle(world, partition, staggered, chain):
    """ps_plan_opts.chain_max: 2 = round pairs, 4 = chains of up to four
    rounds where nothing is exchanged inside (and no k_flood launch for the
    leading rounds, so the chains start at round 1)."""
    opts = {"chain_max": chain, "chain_max_groups": chain}
    if chain > 2:
        opts["flood"] = 0
    rng, trees, roots, live = build(world, partition, seed=world * 7 + partition + 3 * staggered, fan=4)
    n_msgs = 300
    topics = rng.integers(0, len(trees), size=n_msgs)
    starts = rng.integers(0, 4, size=n_msgs) if staggered else None
    plans = [PL.Plan(np.stack(trees), roots, world, r, partition, plan=opts) for r in range(world)]
    for p in plans:
        p.window(topics, starts)
    info = [p.info() for p in plans]
    assert len({i["rounds"] for i in info}) == 1  # every rank plans the same rounds
    for q in range(1, info[0]["rounds"] + 1):  # ... and the same exchange rounds and region sizes
        xs = [p.xchg(q) for p in plans]
        assert len({x["any"] for x in xs}) == 1
        if xs[0]["any"]:
            for a in range(world):
                for b in range(world):
                    if a != b:
                        assert xs[a]["s_len"][b] == xs[b]["r_len"][a]
                        assert xs[a]["s_len"][b] % 128 == 0 and xs[a]["s_off"][b] % 128 == 0
    sims = [RankSim(p, live) for p in plans]
    emulate(sims, info[0]["rounds"], in_process_exchange(sims))
    n_groups = [len(np.unique(starts[topics == t])) if staggered else 1 for t in range(len(trees))]
    check(sims, trees, roots, live, n_groups)
    kinds = set(int(k) for p in plans for k in p.get(PL.ROUND_KIND))
    if chain == 2:
        assert PE.K_CHAIN not in kinds
    elif world == 1 or partition == PE.PART_SUBTREE:
        assert PE.K_CHAIN in kinds, kinds
    if world > 1 and partition == PE.PART_SUBTREE:
        # the subtree partition exchanges in one round per (topic, group) only
        ex = sum(plans[0].xchg(q)["any"] for q in range(1, info[0]["rounds"] + 1))
        assert ex <= len(trees) * max(n_groups)


def test_local_chunks_precede_ghost_chunks():
    """Per round, the locally fed nodes of a level come first (their chunks run
    while the exchange is in flight); the ghost-fed ones follow, grouped by
    source rank and ordered by record index (sequential reads of the receive
    buffer)."""
    _, trees, roots, live = build(4, PE.PART_PEER, n=3000, n_topics=1, seed=11, fan=6)
    p = PL.Plan(np.stack(trees), roots, 4, 1, PE.PART_PEER)
    p.window(np.zeros(200, dtype=np.uint32))
    gref = p.get(PL.GHOST_REF).astype(np.int64)
    T = p.topic(0)
    lo, ll = T["level_off"], T["level_local"]
    for d in range(1, T["depth"] + 1):
        a, b = T["nbase"] + lo[d], T["nbase"] + lo[d + 1]
        loc = T["nbase"] + lo[d] + ll[d]
        assert (gref[a:loc] == NONE).all() and (gref[loc:b] != NONE).all()
        g = gref[loc:b]
        key = (g >> 27) * (1 << 27) + (g & MASK)
        assert (np.diff(key) >= 0).all()
    for q in range(1, p.info()["rounds"] + 1):
        k = p.get(PL.ROUND_KIND)[q]
        if k != PE.K_PULL:
            continue
        lo_c, split, hi_c, ch = p.chunks(PL.PULL, q)
        assert all((gref[c["node_begin"]:c["node_end"]] == NONE).all() for c in ch[:split - lo_c])
        assert all((gref[c["node_begin"]:c["node_end"]] != NONE).all() for c in ch[split - lo_c:])


def test_multi_rank_pairs_only_without_exchange():
    """N ranks pair rounds (k_pull_pair) only where round q + 1 and q + 2
    exchange nothing: under the subtree partition, every round but the split
    level's neighbourhood."""
    _, trees, roots, live = build(2, PE.PART_SUBTREE, n=20000, n_topics=1, seed=5)
    plans = [PL.Plan(np.stack(trees), roots, 2, r, PE.PART_SUBTREE) for r in range(2)]
    for p in plans:
        p.window(np.zeros(600, dtype=np.uint32))
    for p in plans:
        kind = p.get(PL.ROUND_KIND)
        rounds = p.info()["rounds"]
        anyx = [False] + [p.xchg(q)["any"] for q in range(1, rounds + 1)] + [False, False]
        assert sum(anyx) == 1
        assert any(k in (PE.K_PAIR, PE.K_CHAIN) for k in kind)  # (a tail chain may take the pair's place)
        for q in range(1, rounds + 1):
            if kind[q] in (PE.K_PAIR, PE.K_CHAIN):
                assert not anyx[q + 1] and not anyx[q + 2]
    sims = [RankSim(p, live) for p in plans]
    emulate(sims, plans[0].info()["rounds"], in_process_exchange(sims))
    check(sims, trees, roots, live, [1])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, staggered, out):
    import torch.distributed as tdist

    from psengine import dist as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist = D.init("gloo")
    try:
        rng, trees, roots, live = build(world, PE.PART_PEER, n=1200, n_topics=2, seed=31 + staggered, fan=5)
        topics = rng.integers(0, 2, size=200)
        starts = rng.integers(0, 3, size=200) if staggered else None
        p = PL.Plan(np.stack(trees), roots, world, rank, PE.PART_PEER)
        p.window(topics, starts)
        sim = RankSim(p, live)

        def exchange(q):
            mine = sim.regions_out(q)
            allr = [None] * world
            tdist.all_gather_object(allr, mine)
            if p.xchg(q)["any"]:
                sim.regions_in(q, {a: allr[a][rank] for a in range(world) if a != rank})

        rounds = p.info()["rounds"]
        for q in range(1, rounds + 1):
            sim.pack(q)
            exchange(q)
            for part in (0, 1):
                sim.run_round(q, part)
        reached = sorted((int(sim.node_topic[u]), int(sim.peer[u])) for u in np.nonzero(sim.reached)[0]
                         if sim.level[u] != 0)
        allr = [None] * world
        tdist.all_gather_object(allr, (reached, [len(sim.writes[k]) for k in sorted(sim.writes)]))
        if rank == 0:
            out[staggered] = allr
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("staggered", [0, 1])
def test_gloo_world2_replays_the_plans(staggered):
    import torch.multiprocessing as mp

    world = 2
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_gloo_worker, args=(world, _free_port(), staggered, out), nprocs=world, join=True)
    rng, trees, roots, live = build(world, PE.PART_PEER, n=1200, n_topics=2, seed=31 + staggered, fan=5)
    got = set()
    for reached, writes in out[staggered]:
        got |= {tuple(x) for x in reached}
        assert all(w == 1 for w in writes)
    exp = set()
    for t, (par, root) in enumerate(zip(trees, roots)):
        rp, cl = O.parents_to_csr(par)
        _, oh, _ = O.disseminate(rp, cl, root, live, 1)
        exp |= {(t, int(x)) for x in np.nonzero(oh[0] != 0xFF)[0]}
    assert got == exp


@pytest.mark.parametrize("chain", [2, 4])
def test_wide_rows_plan(chain):
    """Rows wider than the 768-word LDS stage (52,000 messages of one topic in
    a window: 814 words): they cannot pair, so with pairs only (chain_max 2)
    those rounds get one k_pull launch each; chains cut the rows into column
    slices of the stage width, in the launch's slice segment, and the replay
    still tiles every row exactly."""
    rng, trees, roots, live = build(1, PE.PART_PEER, n=1200, n_topics=1, seed=5, fan=3)
    topics = np.zeros(52000, dtype=np.uint32)
    p = PL.Plan(np.stack(trees), roots, plan={"chain_max": chain, "chain_max_groups": chain, "flood": 0})
    p.window(topics)
    assert p.layout(0)["W"] == 814
    kinds = [int(k) for k in p.get(PL.ROUND_KIND)]
    rounds = p.info()["rounds"]
    if chain == 2:
        assert PE.K_PAIR not in kinds and PE.K_CHAIN not in kinds
        assert all(k in (PE.K_PULL, 0) for k in kinds[1:rounds + 1])
    else:
        assert PE.K_CHAIN in kinds
        for q in range(1, rounds + 1):
            n, ch = p.chain(q)
            for c in ch:
                assert (c["w0"], c["S"]) in ((0, 768), (768, 46)), c
                assert c["node_end"] - c["node_begin"] == 1
    sims = [RankSim(p, live)]
    emulate(sims, rounds, in_process_exchange(sims))
    check(sims, trees, roots, live, [1])


@pytest.mark.parametrize("overlap", [0, 1])
def test_deep_window_plan(overlap):
    """A deep single-start window (>= 12 rounds) plans chains from round 1 and
    no k_flood while the cross-window overlap is on (this
    window's 2.3 MB of rows pass the byte floor only with it lowered to 0);
    the chain that ends at the last round may take one round more than
    chain_max (chain_tail).  With the overlap off, k_flood takes the leading
    rounds again.  Either plan replays to the oracle."""
    rng = np.random.default_rng(17)
    n = 6000
    parent = np.full(n, NONE, dtype=np.uint32)
    parent[1:] = (np.arange(1, n) - 1) // 2  # a complete binary tree: 13 levels
    live = (rng.random(n) > 0.05).astype(np.uint8)
    live[0] = 1
    p = PL.Plan(parent[None, :], [0], plan={"overlap": overlap, "overlap_min_bytes": 0})
    p.window(np.zeros(3000, dtype=np.uint32))
    kinds = [int(k) for k in p.get(PL.ROUND_KIND)]
    rounds = p.info()["rounds"]
    last = max(q for q in range(1, rounds + 1) if kinds[q] != 0)
    if overlap:
        assert PE.K_FLOOD not in kinds and kinds[1] == PE.K_CHAIN, kinds
        starts = [q for q in range(1, rounds + 1) if kinds[q] == PE.K_CHAIN]
        n_last, _ = p.chain(starts[-1])
        assert starts[-1] + n_last - 1 == last and n_last == 5, (kinds, n_last)  # chain_max 4, + 1 at the tail
    else:
        assert kinds[1] == PE.K_FLOOD, kinds
    sims = [RankSim(p, live)]
    emulate(sims, rounds, in_process_exchange(sims))
    check(sims, [parent], [0], live, [1])


@pytest.mark.parametrize("align", [0, 1])
def test_aligned_start_groups_plan(align):
    """Paced publishing on one rank (start rounds 0..7): with align_groups the
    window plans exactly like the burst -- one packed node-major row per
    topic, its bits sorted by start round, launch round q writing BFS level
    q, chains from round 1 as a deep window -- and the start groups are bit
    ranges of that row (start, first bit, messages); without it, one
    group-major block per start round over start + depth rounds.  Both
    replay to the oracle."""
    rng = np.random.default_rng(23)
    n = 6000
    parent = np.full(n, NONE, dtype=np.uint32)
    parent[1:] = (np.arange(1, n) - 1) // 2  # 13 levels
    live = (rng.random(n) > 0.05).astype(np.uint8)
    live[0] = 1
    p = PL.Plan(parent[None, :], [0], plan={"align_groups": align, "overlap_min_bytes": 0})
    msgs = np.zeros(3000, dtype=np.uint32)
    starts = (np.arange(3000) % 8).astype(np.uint32)
    p.window(msgs, starts)
    info = p.info()
    lay = p.layout(0)
    kinds = [int(k) for k in p.get(PL.ROUND_KIND)]
    burst = PL.Plan(parent[None, :], [0], plan={"overlap_min_bytes": 0})
    burst.window(msgs)
    if align:
        assert info["aligned"] == 1 and info["rounds"] == 13, info
        assert lay["W"] == 48 and lay["groups"] == [(0, 0, 48)], lay  # ceil(3000 / 64) = 47, padded even
        assert lay["aligned_groups"] == [(s0, 375 * s0, 375) for s0 in range(8)], lay["aligned_groups"]
        assert kinds == [int(k) for k in burst.get(PL.ROUND_KIND)] and kinds[1] == PE.K_CHAIN, kinds
    else:
        assert info["aligned"] == 0 and info["rounds"] == 13 + 7, info
        assert [g[0] for g in lay["groups"]] == list(range(8)) and not lay["aligned_groups"]
    sims = [RankSim(p, live)]
    emulate(sims, info["rounds"], in_process_exchange(sims))
    check(sims, [parent], [0], live, [8])


def test_small_deep_window_keeps_flood():
    """A deep window below the overlap byte floor (512 MB of rows by default)
    can never overlap its predecessor, so it keeps the latency-optimal k_flood
    for its leading rounds instead of the deep-window chains."""
    n = 6000
    parent = np.full(n, NONE, dtype=np.uint32)
    parent[1:] = (np.arange(1, n) - 1) // 2  # 13 levels
    p = PL.Plan(parent[None, :], [0])
    assert p.set_plan()["overlap"] == 1  # (the default)
    p.window(np.zeros(3000, dtype=np.uint32))
    kinds = [int(k) for k in p.get(PL.ROUND_KIND)]
    assert kinds[1] == PE.K_FLOOD, kinds


def test_wide_rows_past_u16_columns():
    """Rows wider than 65,535 words (msg_window above 4.19M messages): the
    chain chunks' column offsets w0 are 32-bit (a u16 w0 wrapped
    and the slices rewrote the wrong columns).  Every slice of a 66,600-word
    row keeps its true offset and the slices tile the row exactly."""
    n = 40
    parent = np.full(n, NONE, dtype=np.uint32)
    parent[1:] = (np.arange(1, n) - 1) // 3
    p = PL.Plan(parent[None, :], [0], plan={"flood": 0, "chain_max": 4})
    p.set_msg_window(66600 * 64)
    p.window(np.zeros(66600 * 64 - 10, dtype=np.uint32))
    W = p.layout(0)["W"]
    assert W == 66600, W
    kinds = [int(k) for k in p.get(PL.ROUND_KIND)]
    assert PE.K_CHAIN in kinds, kinds
    for q in range(1, p.info()["rounds"] + 1):
        n_r, ch = p.chain(q)
        by_run = {}
        for c in ch:
            by_run.setdefault(c["node_begin"], []).append((c["w0"], c["S"]))
        for cols in by_run.values():
            cols.sort()
            assert cols[0][0] == 0 and cols[-1][0] > 65535, cols[-3:]
            for (a, sa), (b, _) in zip(cols, cols[1:]):
                assert a + sa == b
            assert cols[-1][0] + cols[-1][1] == W


def test_plan_opts_defaults_pinned():
    """The production plan is pinned by ps_plan_opts defaults, not by the
    environment: a stray PSAMD_* variable changes nothing unless the A/B
    switch PSAMD_AB=1 is set too."""
    d = PE.default_plan_opts()
    assert d == {"flood_top_bytes": 4 << 20, "overlap_min_bytes": 512 << 20, "launch_bytes": 16_000_000,
                 "flood": 1, "chain_max": 4, "chain_max_groups": 6, "chain_tail": 1, "chain_words": 4096,
                 "flood_words": 2048, "pad_words": 16, "overlap": 1, "overlap_min_rounds": 12,
                 "xchg_overlap": -1, "gpu_build": 1, "flood_spin_ticks": 200_000_000, "chain_nt": 1,
                 "chain_waves": 12, "flood_min_rounds": 4, "align_groups": 1}, d
    parent = np.full(64, NONE, dtype=np.uint32)
    parent[1:] = (np.arange(1, 64) - 1) // 2
    env = dict(os.environ)
    try:
        os.environ["PSAMD_CHAIN"] = "2"
        os.environ["PSAMD_FLOOD"] = "0"
        os.environ.pop("PSAMD_AB", None)
        assert PL.Plan(parent[None, :], [0]).set_plan() == {**d, "gpu_build": 0}  # ignored (a probe builds on the host)
        os.environ["PSAMD_AB"] = "1"
        ab = PL.Plan(parent[None, :], [0]).set_plan()
        assert ab["chain_max"] == 2 and ab["flood"] == 0  # the A/B tools' override
    finally:
        os.environ.clear()
        os.environ.update(env)
    with pytest.raises(PE.EngineError):
        PL.Plan(parent[None, :], [0]).set_plan(chain_max=7)


def wide_span_tree():
    """Level 1: 200 nodes; level 2: 700 children each (140,000 nodes), of
    which only the first and the last have children (2 each); levels 4 and 5
    double.  Peer ids are BFS numbers.  Returns (parent, first level-2 id,
    last level-2 id, first level-3 id)."""
    parent = [NONE] + [0] * 200 + list(np.repeat(np.arange(1, 201), 700))
    l2_first, l2_last = 201, 140200
    parent += [l2_first, l2_first, l2_last, l2_last]
    l3 = 140201
    parent += [l3 + j // 2 for j in range(8)]
    parent += [l3 + 4 + j // 2 for j in range(16)]
    return np.array(parent, dtype=np.uint32), l2_first, l2_last, l3


def test_chain_run_with_wide_parent_span_plan():
    """The plan behind test_gpu_chain.py::test_chain_direct_level0_wide_parent_span
    (ADVICE r4): rounds 1-2 pair (level 2 grows 700x, wider than a chain's
    level tables), rounds 3-5 chain, and that chain's one run of level-3
    nodes has parents 139,999 ids apart -- the direct level-0 path whose
    metadata slot must not spill into level 1's."""
    parent, l2_first, l2_last, l3 = wide_span_tree()
    p = PL.Plan(parent[None, :], [0], plan={"flood": 0, "chain_max": 4})
    p.window(np.zeros(100, dtype=np.uint32))
    kinds = [int(k) for k in p.get(PL.ROUND_KIND)]
    assert kinds[1] == PE.K_PAIR and kinds[3] == PE.K_CHAIN, kinds
    n_r, ch = p.chain(3)
    assert n_r == 3 and len(ch) == 1, (n_r, ch)
    c = ch[0]
    assert (c["node_begin"], c["node_end"]) == (l3, l3 + 4)
    assert parent[c["node_end"] - 1] - parent[c["node_begin"]] == l2_last - l2_first > 65535
