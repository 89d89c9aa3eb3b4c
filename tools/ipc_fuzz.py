#!/usr/bin/env python3
"""Randomised differential runs of the multi-process IPC path: each case
starts 2-4 worker processes (tests/ipc_worker.py) on random multi-topic trees
with dead peers and staggered starts, under a random partition, data path
(zero copy, copy, in place), windows and pipelining, and checks the union of
the ranks' hops, their summed deliveries and digests against one engine on the
same inputs (itself oracle-checked bit-exact by the GPU suite).

    python tools/ipc_fuzz.py [--cases 40] [--seed 0]
"""
import argparse
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))  # (tests/fullsize_common imports the checker)

import psengine as PE  # noqa: E402
from test_gpu_ipc import random_tree, run_ranks  # noqa: E402


def one_case(rng, tmp):
    world = int(rng.integers(2, 5))
    mode = str(rng.choice(["zc", "copy", "inplace"]))
    partition = int(rng.choice([PE.PART_PEER, PE.PART_SUBTREE]))
    n = int(rng.integers(300, 6000))
    nt = int(rng.integers(1, 5))
    nm = int(rng.integers(1, 400))
    roots = [int(r) for r in rng.choice(n, size=nt, replace=False)]
    trees = np.stack([random_tree(rng, n, roots[t]) for t in range(nt)])
    live = (rng.random(n) > rng.uniform(0.0, 0.15)).astype(np.uint8)
    live[roots] = 1
    topics = rng.integers(0, nt, size=nm).astype(np.uint32)
    starts = rng.integers(0, int(rng.integers(1, 6)), size=nm).astype(np.uint32)
    windows = int(rng.integers(1, 4))
    pipelined = bool(rng.integers(0, 2))
    got = run_ranks(tmp, world, mode, partition, n, roots, trees, live, topics, starts, np.arange(nm),
                    record=True, windows=windows, pipelined=pipelined)
    with PE.Engine(n, nt, record_hops=True) as one:
        for t in range(nt):
            one.set_tree(t, roots[t], trees[t])
        one.set_live(live)
        for _ in range(windows):
            first = one.publish(topics, starts)
            st1 = one.run()
        hops1 = np.stack([one.hops(first + m) for m in range(nm)])
        digest1 = one.seen_digest()
    union = np.stack([g["hops"] for g in got]).min(axis=0)
    ok = (np.array_equal(union, hops1) and sum(int(g["deliveries"]) for g in got) == st1.deliveries
          and sum(int(g["duplicates"]) for g in got) == 0
          and sum(int(g["digest"]) for g in got) % (1 << 64) == digest1)
    return ok, dict(world=world, mode=mode, partition=partition, n=n, nt=nt, nm=nm, windows=windows,
                    pipelined=pipelined)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=40)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    t0 = time.time()
    bad = 0
    for c in range(args.cases):
        rng = np.random.default_rng([args.seed, c])
        with tempfile.TemporaryDirectory() as tmp:
            ok, desc = one_case(rng, tmp)
        if not ok:
            bad += 1
            print(f"[ipc-fuzz] case {c} FAILED: {desc}", flush=True)
        print(f"[ipc-fuzz] {c + 1}/{args.cases} cases, {bad} failures, {time.time() - t0:.0f} s  {desc}", flush=True)
    print(f"[ipc-fuzz] done: {args.cases} cases, {bad} failures", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
