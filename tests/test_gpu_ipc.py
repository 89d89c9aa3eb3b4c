"""GPU: the multi-GPU path with one PROCESS per rank: the
IPC transport (ps_dist_init_ipc) -- every rank a separate process
(tests/ipc_worker.py), several sharing this box's one GPU, device memory
mapped across processes with hipIpcGetMemHandle / hipIpcOpenMemHandle, each
round ordered by device flags in IPC-mapped memory -- through its three data
paths: the sender's records read in place (zero copy), copied into the
receive buffer (the RCCL data path), and the owners' rows read in place
(PS_DIST_F_INPLACE: no records below the roots).  This replaces the
reference's cross-host child write (/root/reference/subtree.go:333) and the
per-hop read (/root/reference/client.go:104) between ranks.

* Random multi-topic trees with dead peers and staggered starts, 2-3 ranks,
  both partitions, level and compaction mode, blocking and pipelined
  windows: the union of the ranks' hops, their summed deliveries and seen
  digests equal a single engine's (itself oracle-checked bit-exact in
  test_gpu_parity.py).
* cfg4 at FULL size (16,777,216 peers, TreeOpts{8,20}, 1,000 messages, 2 %
  dead peers cutting top subtrees) under the peer hash on 2 and 4 processes:
  exact deliveries and per-round histogram of or_disseminate
  (oracle/psoracle.c), 16 sampled delivered sets (the union over ranks; a
  rank reports its own nodes only) against the oracle's reach, and the
  digest sum against the single engine.
"""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import psengine as PE
from fullsize_common import CLASSES, check_run, paced_starts, sampled

pytestmark = pytest.mark.gpu
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ipc_worker.py")


class _St:  # a worker's stats, shaped like PE.Stats for check_run
    def __init__(self, z):
        self.deliveries = int(z["deliveries"])
        self.duplicates = int(z["duplicates"])
        self.deliveries_per_round = z["per_round"]
        self.xchg_path = int(z["xchg_path"])
        self.xchg_rounds = int(z["xchg_rounds"])
        self.expand_mode = int(z["expand_mode"])


def run_ranks(tmp, world, mode, partition, n, roots, parents, live, topics, starts=None, samples=(),
              record=False, windows=1, pipelined=False, flags=0, seed=1, timeout=150):
    """Starts `world` worker processes on one job and returns their results
    (every worker is killed if any fails or the job overruns)."""
    ppath = os.path.join(tmp, "parents.npy")
    np.save(ppath, np.ascontiguousarray(parents, dtype=np.uint32))
    gid = PE.ipc_group_id()
    job = os.path.join(tmp, "job.npz")
    np.savez(job, world=world, mode=mode, record=record, n_peers=n, roots=np.asarray(roots, dtype=np.int64),
             parents_path=ppath, live=np.asarray(live, dtype=np.uint8), topics=np.asarray(topics, dtype=np.uint32),
             starts=np.zeros(0, np.uint32) if starts is None else np.asarray(starts, dtype=np.uint32),
             samples=np.asarray(samples, dtype=np.int64), gid=np.frombuffer(gid, dtype=np.uint8),
             partition=partition, seed=seed, windows=windows, pipelined=pipelined, flags=flags)
    outs = [os.path.join(tmp, f"out{r}.npz") for r in range(world)]
    procs = [subprocess.Popen([sys.executable, WORKER, job, str(r), outs[r]], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    t0 = time.monotonic()
    logs = [""] * world
    try:
        for r, p in enumerate(procs):
            logs[r] = p.communicate(timeout=max(1.0, timeout - (time.monotonic() - t0)))[0]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    bad = [r for r, p in enumerate(procs) if p.returncode != 0]
    assert not bad, "\n".join(f"rank {r} rc={procs[r].returncode}:\n{logs[r][-3000:]}" for r in bad)
    return [np.load(o) for o in outs]


def random_tree(rng, n, root):
    perm = rng.permutation(n)
    perm = np.concatenate([[root], perm[perm != root]])
    parent = np.full(n, 0xFFFFFFFF, dtype=np.uint32)
    for i in range(1, n):
        parent[perm[i]] = perm[rng.integers(max(0, i - 12), i)]
    return parent


@pytest.mark.parametrize("world,mode,partition,compact,pipelined", [
    (2, "zc", PE.PART_PEER, False, False),
    (2, "copy", PE.PART_SUBTREE, False, True),
    (2, "inplace", PE.PART_PEER, False, True),
    (3, "inplace", PE.PART_SUBTREE, False, False),
    (3, "zc", PE.PART_PEER, False, True),
    (3, "copy", PE.PART_PEER, False, False),
    (2, "copy", PE.PART_PEER, True, False),
])
def test_random_trees_processes_match_single_engine(tmp_path, world, mode, partition, compact, pipelined):
    rng = np.random.default_rng(4242 + world)
    n, nt, nm = 3000, 3, 300
    roots = [int(r) for r in rng.integers(0, n, size=nt)]
    trees = np.stack([random_tree(rng, n, roots[t]) for t in range(nt)])
    live = (rng.random(n) > 0.08).astype(np.uint8)
    live[roots] = 1
    topics = rng.integers(0, nt, size=nm).astype(np.uint32)
    starts = rng.integers(0, 4, size=nm).astype(np.uint32)
    samples = np.arange(nm)
    flags = PE.F_COMPACT if compact else 0
    got = run_ranks(str(tmp_path), world, mode, partition, n, roots, trees, live, topics, starts, samples,
                    record=True, windows=3, pipelined=pipelined, flags=flags)
    with PE.Engine(n, nt, record_hops=True, flags=flags) as one:
        for t in range(nt):
            one.set_tree(t, roots[t], trees[t])
        one.set_live(live)
        for _ in range(3):
            first = one.publish(topics, starts)
            st1 = one.run()
        hops1 = np.stack([one.hops(first + m) for m in range(nm)])
        digest1 = one.seen_digest()
    union = np.stack([g["hops"] for g in got]).min(axis=0)
    assert np.array_equal(union, hops1), "hops differ from the single engine"
    assert sum(int(g["deliveries"]) for g in got) == st1.deliveries
    assert sum(int(g["duplicates"]) for g in got) == 0
    assert sum(int(g["digest"]) for g in got) % (1 << 64) == digest1, "digests do not add up"
    want_mode = PE.MODE_COMPACT if compact else None
    if want_mode is not None:
        assert all(int(g["expand_mode"]) == want_mode for g in got)
    else:
        want = {"zc": PE.XCHG_ZERO_COPY, "copy": PE.XCHG_COPY, "inplace": PE.XCHG_IN_PLACE}[mode]
        paths = [int(g["xchg_path"]) for g in got]
        assert all(p in (want, PE.XCHG_NONE) for p in paths) and want in paths, paths


@pytest.mark.parametrize("world,mode", [(2, "inplace"), (4, "inplace"), (4, "zc"), (2, "copy")])
def test_cfg4_full_size_processes_peer_hash(tmp_path, cfg4_full, world, mode):
    """cfg4 at full size, one process per rank under the peer hash (owner(p) =
    splitmix64(p) mod world), against the oracle."""
    wl, parent, live, tot, reach, hist = cfg4_full.astuple()
    samples = sampled(wl.n_msgs, seed=9)
    got = run_ranks(str(tmp_path), world, mode, PE.PART_PEER, wl.n_peers, [0], parent[None, :], live,
                    wl.msg_topics, samples=samples, seed=wl.seed)
    stats = [_St(g) for g in got]
    assert all(s.expand_mode == PE.MODE_LEVEL_PULL for s in stats)
    want = {"zc": PE.XCHG_ZERO_COPY, "copy": PE.XCHG_COPY, "inplace": PE.XCHG_IN_PLACE}[mode]
    assert all(s.xchg_path == want and s.xchg_rounds > 0 for s in stats), [s.xchg_path for s in stats]
    check_run(stats, wl.n_msgs, tot, hist)
    own = PE.partition_owner(parent, 0, 0, world, PE.PART_PEER)
    for k in range(len(samples)):
        u = np.zeros(wl.n_peers, dtype=bool)
        for r, g in enumerate(got):
            d = np.unpackbits(g["delivered"][k])[: wl.n_peers].astype(bool)
            assert not (d & (own != r)).any()  # a rank reports its own nodes only
            u |= d
        assert np.array_equal(u, reach), int(samples[k])
    assert sum(int(g["digest"]) for g in got) % (1 << 64) == cfg4_full.digest()


def test_bench_two_processes_on_one_gpu():
    """`bench.py --gpus 2` on this pool's one-GPU boxes: two ranks (one process
    each, torch.distributed.run) share the GPU over the IPC transport; the
    line reports the job's deliveries (asserted inside against the expected
    total) and the ratio to one rank doing the same messages alone."""
    import json

    if PE.device_count() >= 2:
        pytest.skip("every rank has a GPU of its own: bench.py takes RCCL")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--workload", "cfg4", "--scale", "0.05",
           "--steps", "3", "--warmup", "1", "--no-cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=repo)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert "IPC transport" in line["config"]["parallelism"]
    assert line["shared_gpu"]["ranks_per_gpu"] == 2 and line["shared_gpu"]["ratio_vs_one_rank"] > 0


def test_cfg3_paced_processes_cut_tree(tmp_path, cfg3_cut):
    """BASELINE cfg3 at full size (1M peers, 64 Zipf topics, 100k messages
    over start rounds 0..7) on a cut tree, two processes under the peer hash,
    owners' rows read in place: the summed deliveries and per-round histogram
    equal or_disseminate's shifted per start group, and 8 sampled delivered
    sets per topic class (the union over the ranks) equal the oracle's reach."""
    wl, parents, live, exp = cfg3_cut
    starts = paced_starts(wl)
    samples = np.concatenate([np.random.default_rng(7 + t).choice(np.nonzero(wl.msg_topics == t)[0], 8,
                                                                   replace=False) for t in CLASSES])
    got = run_ranks(str(tmp_path), 2, "inplace", PE.PART_PEER, wl.n_peers, [ts.root for ts in wl.topics],
                    np.stack(parents), live, wl.msg_topics, starts=starts, samples=samples, seed=wl.seed,
                    timeout=170)
    assert sum(int(g["deliveries"]) for g in got) == exp.deliveries(wl.msg_topics)
    assert sum(int(g["duplicates"]) for g in got) == 0
    per = sum(g["per_round"].astype(np.int64) for g in got)
    want = exp.per_round(wl.msg_topics, starts, max(96, per.shape[0]))
    assert per[1:].tolist() == want[1:per.shape[0]].tolist()
    assert all(int(g["xchg_path"]) == PE.XCHG_IN_PLACE for g in got)
    for k, m in enumerate(samples):
        t = int(wl.msg_topics[m])
        u = np.zeros(wl.n_peers, dtype=bool)
        for g in got:
            u |= np.unpackbits(g["delivered"][k])[: wl.n_peers].astype(bool)
        assert np.array_equal(u, exp.reach(t)), (t, int(m))
