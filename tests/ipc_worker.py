#!/usr/bin/env python3
"""One rank of a process-per-rank run over the IPC transport (ps_dist_init_ipc),
started by tests/test_gpu_ipc.py (several of these share the box's one GPU).

    python tests/ipc_worker.py <job.npz> <rank> <out.npz>

The job file holds the topology (per-topic roots and parent arrays), the live
mask, the publish schedule, the transport mode and the group id; every rank
builds the same topics and publishes the same messages, owns its partition of
every tree, and writes its stats, seen digest and -- for the sampled messages
-- its hops (recording mode) or delivered bitmaps (production instance) for
the parent to check against the oracle.  No oracle here: this is the product
path, run as a separate process per rank.
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
import psengine as PE  # noqa: E402


def main():
    job, rank, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    j = np.load(job, allow_pickle=False)
    world = int(j["world"])
    mode = str(j["mode"])
    record = bool(j["record"])
    n = int(j["n_peers"])
    roots = j["roots"].astype(np.int64)
    nt = len(roots)
    parents = np.load(str(j["parents_path"]), mmap_mode="r", allow_pickle=False)
    t0 = time.perf_counter()
    eng = PE.Engine(n, nt, record_hops=record, seed=int(j["seed"]), flags=int(j["flags"]))
    try:
        eng.dist_init_ipc(rank, world, bytes(j["gid"]), int(j["partition"]), copy=mode == "copy",
                          inplace=mode == "inplace")
        for t in range(nt):
            eng.set_tree(t, int(roots[t]), np.ascontiguousarray(parents[t]))
        eng.set_live(j["live"])
        starts = j["starts"] if j["starts"].size else None
        res = {}
        windows = int(j["windows"])
        if bool(j["pipelined"]):  # window k + 1 enqueued (its exchanges included) while k runs
            for w in range(windows):
                first = eng.publish(j["topics"], starts)
                eng.run_async()
                if w:
                    eng.wait()
            st = eng.wait()
        else:
            for w in range(windows):
                first = eng.publish(j["topics"], starts)
                st = eng.run()
        # the last window's stats and sampled messages (windows repeat the schedule)
        samples = j["samples"]
        if record:
            res["hops"] = np.stack([eng.hops(first + int(m)) for m in samples]) if len(samples) else np.zeros(0)
        else:
            res["delivered"] = (np.stack([np.packbits(eng.delivered(first + int(m)).astype(bool)) for m in samples])
                                if len(samples) else np.zeros(0))
        res.update(deliveries=st.deliveries, duplicates=st.duplicates, rounds=st.rounds,
                   per_round=np.array(list(st.deliveries_per_round), dtype=np.int64),
                   xchg_path=st.xchg_path, xchg_rounds=st.xchg_rounds, expand_mode=st.expand_mode,
                   digest=np.uint64(eng.seen_digest()), seconds=time.perf_counter() - t0)
        np.savez(out, **res)
        print(f"[ipc_worker] rank {rank}/{world} {mode}: {st.deliveries} deliveries, {st.rounds} rounds, "
              f"{time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    finally:
        eng.close()


if __name__ == "__main__":
    main()
