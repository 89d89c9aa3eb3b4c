#!/usr/bin/env python3
"""Randomised differential run of the HIP path against the CPU restatement
(oracle/psoracle.c), wider than the pytest suite: random trees and meshes,
live masks, staggered or single start rounds, several topics, small windows
(many windows per run), eager / lazy seen, pipelined runs, churn sequences
on restated join trees, 2-4 ranks on the loopback transport, per-subscriber
drains, and every execution mode on the same inputs (k_flood with random
k_flood / k_pull splits and task sizes, per-round k_pull, pairs, chains of
3-6 rounds with random run sizes, start groups, the compaction path): identical deliveries, per-round counts and seen digests
on the production (non-recording) instance.  Every case is bit-exact or the
script reports it (seed and case) and exits non-zero.

    python tools/fuzz_gpu.py [--cases 300] [--seed 0] [--max-peers 4000]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle as O  # noqa: E402

# the fuzzer draws plan options through the environment (read at ps_create
# only with the A/B switch on)
os.environ["PSAMD_AB"] = "1"
import psengine as PE  # noqa: E402


def random_tree(rng, n, root):
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, O.NONE, dtype=np.uint32)
    shape = rng.integers(0, 3)
    for i in range(1, n):
        if shape == 0:  # random recursive tree
            j = rng.integers(0, i)
        elif shape == 1:  # deep: mostly the previous few
            j = max(0, i - 1 - int(rng.integers(0, 3)))
        else:  # wide: bounded fan-out levels
            j = (i - 1) // int(rng.integers(2, 9))
        parent[perm[i]] = perm[j]
    return parent


def random_mesh(rng, n, max_out):
    deg = rng.integers(0, max_out + 1, size=n)
    row_ptr = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(deg, out=row_ptr[1:])
    col = rng.integers(0, n, size=int(row_ptr[-1])).astype(np.uint32)
    return row_ptr, col


def case_topology(rng, max_peers):
    n = int(rng.integers(2, max_peers))
    n_topics = int(rng.integers(1, 5))
    live = (rng.random(n) > rng.choice([0.0, 0.05, 0.3])).astype(np.uint8)
    n_msgs = int(rng.integers(1, 700))
    staggered = rng.random() < 0.4
    starts = rng.integers(0, 5, size=n_msgs) if staggered else None
    topics = rng.integers(0, n_topics, size=n_msgs)
    window = int(rng.choice([64, 200, 65536]))
    flags = (PE.F_NO_LAZY_SEEN if rng.random() < 0.2 else 0) | (PE.F_COMPACT if rng.random() < 0.2 else 0)
    if staggered and rng.random() < 0.5:
        starts = rng.integers(0, 9, size=n_msgs)
    set_modes(rng)
    record = True
    pipelined = rng.random() < 0.3
    with PE.Engine(n, n_topics, record_hops=record, msg_window=window, flags=flags) as e:
        graphs = []
        for t in range(n_topics):
            root = int(rng.integers(0, n))
            if rng.random() < 0.25:
                rp, cl = random_mesh(rng, n, int(rng.integers(1, 5)))
                e.set_children(t, root, rp, cl)
            else:
                par = random_tree(rng, n, root)
                e.set_tree(t, root, par)
                rp, cl = O.parents_to_csr(par)
            graphs.append((rp, cl, root))
        e.set_live(live)
        first = e.publish(topics, starts)
        if pipelined:
            e.run_async()
            st = e.wait()
        else:
            st = e.run()
        total = 0
        for t, (rp, cl, root) in enumerate(graphs):
            idx = np.nonzero(topics == t)[0]
            if not len(idx):
                continue
            # the oracle floods each message from its start round; hops are
            # relative to it, so one call per distinct start suffices
            tot, hops, _ = O.disseminate(rp, cl, root, live, 1)
            total += tot * len(idx)
            for m in idx[: 40]:
                got = e.hops(first + int(m))
                if not np.array_equal(got, hops[0]):
                    bad = np.nonzero(got != hops[0])[0][:8]
                    return f"topic {t} msg {m}: peers {bad} engine {got[bad]} oracle {hops[0][bad]}"
        if st.deliveries != total:
            return f"deliveries {st.deliveries} != oracle {total}"
    return None


MODE_ENV = ("PSAMD_FLOOD", "PSAMD_FLOOD_TOP_BYTES", "PSAMD_FLOOD_WORDS", "PSAMD_PULL_PAIR", "PSAMD_CHAIN",
            "PSAMD_CHAIN_WORDS", "PSAMD_OVERLAP_BYTES", "PSAMD_OVERLAP_ROUNDS")


def set_modes(rng):
    """Random execution-mode switches for the next engine (read at creation)."""
    for k in MODE_ENV:
        os.environ.pop(k, None)
    if rng.random() < 0.2:
        os.environ["PSAMD_FLOOD"] = "0"
    if rng.random() < 0.4:
        os.environ["PSAMD_FLOOD_TOP_BYTES"] = str(int(rng.choice([0, 256, 4096, 65536])))
    if rng.random() < 0.3:
        os.environ["PSAMD_FLOOD_WORDS"] = str(int(rng.choice([64, 256, 4096])))
    if rng.random() < 0.3:
        os.environ["PSAMD_PULL_PAIR"] = "0"
    if rng.random() < 0.5:  # launches of at most 2 (pairs) .. 6 rounds (chains)
        os.environ["PSAMD_CHAIN"] = str(int(rng.integers(2, 7)))
    if rng.random() < 0.3:  # chain runs sized for fewer / more row words per wave
        os.environ["PSAMD_CHAIN_WORDS"] = str(int(rng.choice([256, 1024, 32768])))


def case_modes(rng, max_peers):
    """One set of trees, live mask and publishes (single or staggered
    starts) through every mode, production instances: the same deliveries,
    per-round deliveries and seen digest, and the oracle's deliveries."""
    n = int(rng.integers(2, max_peers))
    n_topics = int(rng.integers(1, 5))
    live = (rng.random(n) > rng.choice([0.0, 0.05, 0.3])).astype(np.uint8)
    n_msgs = int(rng.integers(1, 900))
    starts = rng.integers(0, int(rng.integers(1, 9)), size=n_msgs) if rng.random() < 0.6 else None
    topics = rng.integers(0, n_topics, size=n_msgs)
    trees = []
    for _ in range(n_topics):
        root = int(rng.integers(0, n))
        trees.append((root, random_tree(rng, n, root)))
    total = 0
    for t, (root, par) in enumerate(trees):
        rp, cl = O.parents_to_csr(par)
        tot, _, _ = O.disseminate(rp, cl, root, live, 1, want_hops=False)
        total += tot * int((topics == t).sum())
    ref = None
    window = int(rng.choice([128, 65536]))
    modes = [({}, 0), ({}, PE.F_COMPACT), ({"PSAMD_FLOOD": "0"}, 0),
             ({"PSAMD_FLOOD": "0", "PSAMD_PULL_PAIR": "0"}, 0),
             ({"PSAMD_FLOOD": "0", "PSAMD_CHAIN": "2"}, 0),
             ({"PSAMD_FLOOD": "0", "PSAMD_CHAIN": str(int(rng.integers(3, 7))),
               "PSAMD_CHAIN_WORDS": str(int(rng.choice([256, 8192])))}, 0),
             ({"PSAMD_FLOOD_TOP_BYTES": str(int(rng.choice([0, 512, 1 << 30])))}, 0),
             ({"PSAMD_FLOOD_WORDS": "64"}, 0), ({}, PE.F_NO_LAZY_SEEN)]
    for env, flags in modes:
        for k in MODE_ENV:
            os.environ.pop(k, None)
        os.environ.update(env)
        with PE.Engine(n, n_topics, flags=flags, msg_window=window) as e:
            for t, (root, par) in enumerate(trees):
                e.set_tree(t, root, par)
            e.set_live(live)
            e.publish(topics, starts)
            st = e.run()
            key = (st.deliveries, st.duplicates, st.as_dict()["deliveries_per_round"], e.seen_digest())
        if st.deliveries != total:
            return f"mode {env} flags {flags}: deliveries {st.deliveries} != oracle {total}"
        if ref is None:
            ref = key
        elif key != ref:
            return f"mode {env} flags {flags}: counters or digest differ from the default mode"
    for k in MODE_ENV:
        os.environ.pop(k, None)
    return None


def case_churn(rng, max_peers):
    n = int(rng.integers(20, max_peers))
    seed = int(rng.integers(1, 1 << 30))
    w, mw = int(rng.integers(1, 5)), int(rng.integers(5, 9))
    with PE.Engine(n, 1, record_hops=True, seed=seed) as e:
        ot = O.Tree(n, 0, w, mw, PE.Engine.topic_seed(seed, 0))
        e.topic_create(0, 0, w, mw)
        members = set()
        for step in range(12):
            op = rng.random()
            if op < 0.5 or not members:
                outs = [p for p in range(1, n) if p not in members]
                if outs:
                    peers = rng.choice(outs, size=min(len(outs), int(rng.integers(1, 30))), replace=False)
                    st = e.join(0, peers, check=False)
                    for p, s in zip(peers, st):
                        if ot.join(int(p)) != s:
                            return f"join status differs at step {step} peer {p}"
                        if s == 0:
                            members.add(int(p))
            elif op < 0.8:
                peers = rng.choice(sorted(members), size=min(len(members), int(rng.integers(1, 10))), replace=False)
                try:
                    e.leave(0, peers)
                except PE.EngineError:
                    pass
                for p in peers:
                    ot.leave(int(p))
                    members.discard(int(p))
            else:
                p = int(rng.choice(sorted(members)))
                try:
                    e.drop(0, [p])
                except PE.EngineError:
                    pass
                ot.drop(p)
                members.discard(p)
            k = int(rng.integers(1, 4))
            first = e.publish(np.zeros(k))
            e.run()
            for m in range(k):
                exp = ot.message()
                got = e.hops(first + m)
                if not np.array_equal(got, exp):
                    bad = np.nonzero(got != exp)[0][:8]
                    return f"churn step {step} msg {m}: peers {bad} engine {got[bad]} oracle {exp[bad]}"
    return None


MAX_WORLD = 4  # --max-world


def case_dist(rng, max_peers):
    """world 2..MAX_WORLD engines on the loopback transport (one thread
    each), random trees, live masks, single or staggered starts, either
    partition: the union of the ranks' hops equals the oracle's."""
    import threading
    world = int(rng.integers(2, MAX_WORLD + 1))
    n = int(rng.integers(world + 2, max(world + 3, max_peers // 2)))
    n_topics = int(rng.integers(1, 4))
    part = int(rng.integers(0, 2))
    live = (rng.random(n) > rng.choice([0.0, 0.1])).astype(np.uint8)
    n_msgs = int(rng.integers(1, 300))
    starts = rng.integers(0, 4, size=n_msgs) if rng.random() < 0.4 else None
    topics = rng.integers(0, n_topics, size=n_msgs)
    trees = []
    for _ in range(n_topics):
        root = int(rng.integers(0, n))
        trees.append((random_tree(rng, n, root), root))
    lb = PE.Loopback(world)
    engines = [PE.Engine(n, n_topics, record_hops=True) for _ in range(world)]
    try:
        for r, e in enumerate(engines):
            e.dist_init_loopback(lb, r, part)
            for t, (par, root) in enumerate(trees):
                e.set_tree(t, root, par)
            e.set_live(live)
        firsts = [e.publish(topics, starts) for e in engines]
        stats, errs = [None] * world, []

        def go(r):
            try:
                stats[r] = engines[r].run()
            except Exception as ex:  # noqa: BLE001
                errs.append(ex)

        th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=120)
        if any(x.is_alive() for x in th):
            return "rank thread hung"
        if errs:
            return "rank errors: " + " | ".join(str(x) for x in errs)
        total = 0
        for t, (par, root) in enumerate(trees):
            idx = np.nonzero(topics == t)[0]
            if not len(idx):
                continue
            rp, cl = O.parents_to_csr(par)
            tot, hops, _ = O.disseminate(rp, cl, root, live, 1)
            total += tot * len(idx)
            for m in idx[:20]:
                got = np.stack([e.hops(firsts[0] + int(m)) for e in engines]).min(axis=0)
                if not np.array_equal(got, hops[0]):
                    bad = np.nonzero(got != hops[0])[0][:8]
                    return f"world {world} part {part} topic {t} msg {m}: peers {bad} {got[bad]} vs {hops[0][bad]}"
        if sum(st.deliveries for st in stats) != total:
            return f"world {world}: deliveries {sum(st.deliveries for st in stats)} != {total}"
    finally:
        for e in engines:
            e.close()
        lb.close()
    return None


def case_drain(rng, max_peers):
    """ps_read_peer_messages against the hops: a peer's drain is exactly the
    messages that reached it, ordered by (start round, publish order)."""
    n = int(rng.integers(2, max_peers))
    n_topics = int(rng.integers(1, 4))
    live = (rng.random(n) > 0.1).astype(np.uint8)
    n_msgs = int(rng.integers(1, 400))
    starts = rng.integers(0, 6, size=n_msgs) if rng.random() < 0.5 else np.zeros(n_msgs, dtype=np.int64)
    topics = rng.integers(0, n_topics, size=n_msgs)
    with PE.Engine(n, n_topics, record_hops=True) as e:
        for t in range(n_topics):
            root = int(rng.integers(0, n))
            e.set_tree(t, root, random_tree(rng, n, root))
        e.set_live(live)
        first = e.publish(topics, starts)
        e.run()
        hops = np.stack([e.hops(first + m) for m in range(n_msgs)])  # [msg][peer]
        for p in rng.choice(n, size=min(n, 12), replace=False):
            for t in range(n_topics):
                ids = [m for m in range(n_msgs) if topics[m] == t and hops[m, p] != 0xFF]
                exp = [first + m for m in sorted(ids, key=lambda m: (int(starts[m]), m))]
                got = e.peer_messages(t, int(p)).tolist()
                if got != exp:
                    return f"peer {p} topic {t}: drain {got[:6]}... != {exp[:6]}..."
    return None


def case_pipeline(rng, max_peers):
    """Pipelined runs with the cross-window overlap forced on small windows
    (PSAMD_OVERLAP_BYTES=0, random depth floor, random launch modes) or off
    (signalled windows, the reduce held back into the next window's first
    launch or not: PSAMD_FUSE_REDUCE), each run a random prefix of the batch
    published in one or two calls: every run's deliveries equal the oracle's,
    the last run's delivered sets of sampled messages equal the oracle's
    reach, and the rows' digest equals a blocking engine's on the same inputs."""
    n = int(rng.integers(64, max_peers))
    n_topics = int(rng.integers(1, 4))
    live = (rng.random(n) > rng.choice([0.0, 0.05, 0.2])).astype(np.uint8)
    n_msgs = int(rng.integers(1, 600))
    topics = rng.integers(0, n_topics, size=n_msgs)
    roots = [int(rng.integers(0, n)) for _ in range(n_topics)]
    pars = [random_tree(rng, n, r) for r in roots]
    runs = int(rng.integers(3, 7))
    set_modes(rng)
    os.environ["PSAMD_OVERLAP_BYTES"] = str(rng.choice([0, 4_000_000_000]))
    os.environ["PSAMD_OVERLAP_ROUNDS"] = str(int(rng.choice([2, 4, 8, 12])))
    os.environ["PSAMD_FUSE_REDUCE"] = str(int(rng.integers(0, 2)))
    per_topic, reach = [], []
    for t in range(n_topics):
        rp, cl = O.parents_to_csr(pars[t])
        tot, hops, _ = O.disseminate(rp, cl, roots[t], live, 1)
        per_topic.append(tot)
        reach.append(hops[0] != 0xFF)
    cuts = [int(rng.integers(1, n_msgs + 1)) for _ in range(runs)]
    splits = [int(rng.integers(0, c + 1)) for c in cuts]
    digests = []
    for pipelined in (True, False):
        with PE.Engine(n, n_topics) as e:
            for t in range(n_topics):
                e.set_tree(t, roots[t], pars[t])
            e.set_live(live)
            sts = []
            for i in range(runs):
                b = topics[: cuts[i]]
                first = e.publish(b[: splits[i]]) if splits[i] else None
                f2 = e.publish(b[splits[i]:]) if splits[i] < cuts[i] else None
                first = f2 if first is None else first
                if pipelined:
                    e.run_async()
                    if i:
                        sts.append(e.wait())
                else:
                    sts.append(e.run())
            if pipelined:
                sts.append(e.wait())
            for i, st in enumerate(sts):
                exp = sum(per_topic[int(t)] for t in topics[: cuts[i]])
                if st.deliveries != exp:
                    return f"pipelined={pipelined} run {i}: deliveries {st.deliveries} != oracle {exp}"
            last = cuts[-1]
            for m in rng.choice(last, size=min(last, 12), replace=False):
                got = e.delivered(first + int(m)).astype(bool)
                if not np.array_equal(got, reach[int(topics[m])]):
                    return f"pipelined={pipelined} msg {m}: delivered set differs from the oracle"
            digests.append(e.seen_digest())
    if digests[0] != digests[1]:
        return f"digest pipelined {digests[0]:#x} != blocking {digests[1]:#x}"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=300)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max-peers", type=int, default=4000)
    ap.add_argument("--only", type=int, nargs="*", help="run just these case numbers (reproduce a failure)")
    ap.add_argument("--max-world", type=int, default=4, help="most loopback ranks of a dist case")
    ap.add_argument("--kinds", nargs="*", help="only these case kinds (topology churn dist drain modes pipeline)")
    args = ap.parse_args()
    global MAX_WORLD
    MAX_WORLD = args.max_world
    fails = 0
    t0 = time.time()
    for c in (args.only if args.only else range(args.cases)):
        rng = np.random.default_rng([args.seed, c])
        kind = ("topology", "churn", "dist", "topology", "drain", "modes", "pipeline")[c % 7]
        if args.kinds and kind not in args.kinds:
            continue
        fn = {"topology": case_topology, "churn": case_churn, "dist": case_dist, "drain": case_drain,
              "modes": case_modes, "pipeline": case_pipeline}[kind]
        try:
            err = fn(rng, args.max_peers)
        except PE.EngineError as ex:
            err = f"engine error: {ex}"
        for k in MODE_ENV:
            os.environ.pop(k, None)
        if err:
            fails += 1
            print(f"FAIL case {c} ({kind}, seed {args.seed}): {err}", flush=True)
        if c % 25 == 0:
            print(f"[fuzz] {c + 1}/{args.cases} cases, {fails} failures, {time.time() - t0:.0f} s", flush=True)
    print(f"[fuzz] done: {args.cases} cases, {fails} failures, {time.time() - t0:.0f} s", flush=True)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
