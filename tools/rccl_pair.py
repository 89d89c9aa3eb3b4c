#!/usr/bin/env python3
"""Two ranks over real RCCL (ps_dist_init), launched by torch.distributed.run:
each rank owns a partition of three random trees (8 % dead peers), both run
the same publishes, and rank 0 checks the union of the ranks' hops, the
summed deliveries and the summed seen digests against a single engine.  On a
one-GPU box both ranks share device 0.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29613 tools/rccl_pair.py --partition peer [--staggered]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
import psengine as PE  # noqa: E402


def random_tree(rng, n, root):
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, 0xFFFFFFFF, dtype=np.uint32)
    for i in range(1, n):
        parent[perm[i]] = perm[rng.integers(max(0, i - 12), i)]
    return parent


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--partition", default="peer", choices=["peer", "subtree"])
    ap.add_argument("--staggered", action="store_true")
    args = ap.parse_args()
    PE.load()  # (the engine's /opt/rocm runtime before torch's bundled copies: psengine/dist.py)
    import torch.distributed as dist

    dist.init_process_group("gloo")  # bootstrap only: the exchange is RCCL inside the engine
    rank, world = dist.get_rank(), dist.get_world_size()
    ndev = int(os.environ.get("PSAMD_DEVICES", "1"))
    dev = rank % ndev
    part = PE.PART_PEER if args.partition == "peer" else PE.PART_SUBTREE
    rng = np.random.default_rng(4242)
    n, nt, nm = 3000, 3, 300
    roots = [int(r) for r in rng.integers(0, n, size=nt)]
    trees = [random_tree(rng, n, roots[t]) for t in range(nt)]
    live = (rng.random(n) > 0.08).astype(np.uint8)
    live[roots] = 1
    topics = rng.integers(0, nt, size=nm).astype(np.uint32)
    starts = rng.integers(0, 4, size=nm).astype(np.uint32) if args.staggered else None

    def build(e):
        for t in range(nt):
            e.set_tree(t, roots[t], trees[t])
        e.set_live(live)
        first = e.publish(topics, starts)
        st = e.run()
        hops = np.stack([e.hops(first + m) for m in range(nm)])
        return st, hops, e.seen_digest()

    obj = [PE.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    eng = PE.Engine(n, nt, record_hops=True, device=dev)
    eng.dist_init(rank, world, obj[0], part)
    st, hops, digest = build(eng)
    mine = (int(st.deliveries), int(st.duplicates), hops, int(digest), int(st.expand_mode))
    got = [None] * world
    dist.all_gather_object(got, mine)
    eng.close()
    if rank == 0:
        with PE.Engine(n, nt, record_hops=True, device=dev) as one:
            st1, hops1, digest1 = build(one)
        union = np.stack([g[2] for g in got]).min(axis=0)
        assert np.array_equal(union, hops1), "hops differ from the single engine"
        assert sum(g[0] for g in got) == st1.deliveries, (sum(g[0] for g in got), st1.deliveries)
        assert sum(g[1] for g in got) == 0
        assert sum(g[3] for g in got) % (1 << 64) == digest1, "digests do not add up"
        print(f"RCCL_PAIR OK partition={args.partition} staggered={args.staggered} "
              f"deliveries={st1.deliveries} modes={[g[4] for g in got]}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
