"""CPU tests of the multi-GPU path (no GPU): the partition function of the
engine (ps_partition_owner, host-only C ABI) and the bootstrap / reduction
helpers of psengine/dist.py under a world_size-2 gloo process group, plus a
2-rank replay of the per-round exchange protocol (ghost parents: a frontier
row crosses once per remote rank owning a child, via all_to_all) whose union
must equal the single-process restatement."""
import os
import socket

import numpy as np
import pytest

import oracle as O
import psengine as PE
from psengine import workloads as WL


def random_tree(rng, n, root=0):
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, O.NONE, dtype=np.uint32)
    for i in range(1, n):
        parent[perm[i]] = perm[rng.integers(0, i)]
    return parent


def depths(parent, root):
    n = len(parent)
    d = np.full(n, -1, np.int64)
    d[root] = 0
    rp, cl = O.parents_to_csr(parent)
    stack = [root]
    while stack:
        p = stack.pop()
        for c in cl[rp[p]:rp[p + 1]]:
            d[c] = d[p] + 1
            stack.append(int(c))
    return d, rp, cl


def test_peer_partition_is_splitmix_mod_world(oracle_lib):
    rng = np.random.default_rng(1)
    par = random_tree(rng, 3000)
    for world in (2, 3, 8):
        own = PE.partition_owner(par, 0, 0, world, PE.PART_PEER)
        assert np.array_equal(own, WL.owner(np.arange(3000), world))


def test_subtree_partition_keeps_subtrees_whole(oracle_lib):
    rng = np.random.default_rng(2)
    n = 20000
    par = random_tree(rng, n)
    d, rp, cl = depths(par, 0)
    for world in (2, 4, 8):
        own = PE.partition_owner(par, 0, 7, world, PE.PART_SUBTREE)
        assert own.min() >= 0 and own.max() < world
        # automatic split level: first level with >= 64*world nodes
        cnt = np.bincount(d[d >= 0])
        L = int(np.nonzero(cnt >= 64 * world)[0][0])
        cross = [(p, c) for p in range(n) for c in cl[rp[p]:rp[p + 1]] if own[p] != own[c]]
        # only edges into the level-L subtrees cross ranks; the levels above
        # L stay with the root's owner
        assert all(d[p] == L - 1 for p, _ in cross)
        assert len(set(own[d < L].tolist())) == 1
        share = np.bincount(own, minlength=world) / n
        # >= 64*world subtrees dealt largest first to the least-loaded rank
        assert share.min() > 0.9 / world and share.max() < 1.1 / world, share


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch.distributed as tdist

    from psengine import dist as D

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    dist = D.init("gloo")
    try:
        # bootstrap: rank 0's bytes reach every rank (the RCCL id path)
        uid = D.share_bytes(dist, lambda: bytes(range(128)), rank)
        assert uid == bytes(range(128))
        # the replayed protocol: each round, a rank ships the
        # row of every frontier parent it owns once to every other rank that
        # owns one of that parent's children (a ghost parent, with its reach
        # flag); the children read their parent's row locally or from the
        # ghosts received -- rows of 128 message bits, as on the GPU
        rng = np.random.default_rng(11)
        n = 1500
        par = random_tree(rng, n)
        live = (rng.random(n) > 0.1).astype(np.uint8)
        rp, cl = O.parents_to_csr(par)
        full = np.array([~0, ~0], dtype=np.int64)
        for part in (PE.PART_PEER, PE.PART_SUBTREE):
            own = PE.partition_owner(par, 0, 0, world, part)
            hop = np.full(n, 255, np.int64)
            rows = {0: full} if own[0] == rank else {}  # this rank's frontier: node -> row
            shipped = 0
            r = 0
            while True:
                r += 1
                outbox = [[] for _ in range(world)]
                for p, row in rows.items():
                    dests = sorted({int(own[c]) for c in cl[rp[p]:rp[p + 1]]} - {rank})
                    for b in dests:
                        outbox[b].append((p, row.tolist(), 1))  # reached: flag 1
                        shipped += 1
                gathered = [None] * world
                tdist.all_gather_object(gathered, outbox)
                ghosts = {p: np.array(row, np.int64) for s in range(world) for p, row, f in gathered[s][rank] if f}
                nxt = {}
                for src in (rows, ghosts):
                    for p, row in src.items():
                        for c in cl[rp[p]:rp[p + 1]]:
                            c = int(c)
                            if own[c] == rank and live[c] and hop[c] == 255:
                                hop[c] = r
                                nxt[c] = row  # new = row(parent) & ~seen(c), seen empty
                rows = nxt
                alive = [len(rows)]
                tot = [None] * world
                tdist.all_gather_object(tot, alive)
                if sum(t[0] for t in tot) == 0:
                    break
            gathered = [None] * world
            tdist.all_gather_object(gathered, hop.tolist())
            sh = [None] * world
            tdist.all_gather_object(sh, [shipped])
            if rank == 0:
                out[part] = np.min(np.array(gathered), axis=0)
                out[(part, "shipped")] = sum(x[0] for x in sh)
        # job totals: max time, summed counts
        t, c = D.job_totals(dist, 1.0 + rank, 10 * (rank + 1))
        assert t == float(world) and c == 10 * world * (world + 1) // 2
    finally:
        tdist.destroy_process_group()


def test_gloo_world2_protocol_matches_single_process(oracle_lib):
    import torch.multiprocessing as mp

    world = 2
    port = _free_port()
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    rng = np.random.default_rng(11)
    n = 1500
    par = random_tree(rng, n)
    live = (rng.random(n) > 0.1).astype(np.uint8)
    rp, cl = O.parents_to_csr(par)
    _, hops, _ = O.disseminate(rp, cl, 0, live, 1)
    own_peer = PE.partition_owner(par, 0, 0, world, PE.PART_PEER)
    for part in (PE.PART_PEER, PE.PART_SUBTREE):
        assert np.array_equal(np.asarray(out[part]).astype(np.uint8), hops[0]), part
    # one ghost row per (reached parent, remote rank owning a child): never
    # more than the cross edges, and the subtree partition ships far fewer
    reached = hops[0] != 255
    reached[0] = True
    cross = {(int(p), int(own_peer[c])) for p in range(n) if reached[p]
             for c in cl[rp[p]:rp[p + 1]] if own_peer[c] != own_peer[p]}
    assert out[(PE.PART_PEER, "shipped")] == len(cross)
    assert out[(PE.PART_SUBTREE, "shipped")] < out[(PE.PART_PEER, "shipped")] / 4
