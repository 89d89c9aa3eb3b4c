"""Multi-GPU driver for bench.py: one process per GPU, torch.distributed (gloo,
host tensors) for bootstrap, barriers and the max-over-ranks clock; the
frontier exchange itself runs inside the engine -- over its own RCCL
communicator (ps_dist_init) when every rank has a GPU, or over the IPC
transport (ps_dist_init_ipc) when ranks share GPUs.  torch.cuda is never used:
the engine's calls block until their windows are done, and only the engine's
HIP runtime (/opt/rocm) initialises the GPU.

Every rank builds the same topics (the restated joins are deterministic) and
publishes the same messages; each owns a hash partition of every topic's tree
nodes (PART_PEER by default: owner(p) = splitmix64(p) mod N; PART_SUBTREE:
level-L subtrees).
The job's deliveries are the sum over ranks; its time is the slowest rank's.

Scaling: "weak" (default) keeps the per-GPU work of the N=1
workload: the same topology, N x the messages (each rank holds 1/N of every
tree, so it moves as many row words as one GPU does at N=1); "strong" runs
the N=1 workload unchanged.

Beside the partitioned run (the JSON line's value), two legs time SURVEY.md
§8e's other decompositions on the same ranks: the other partition
(`subtree_partition` beside the peer-hash headline: cross edges only above
level L, so almost no exchange) and `message_sharded`: every rank holds the
whole topology (a replicated CSR) and disseminates its own share of the
messages -- messages are independent on a churn-free batch, so no exchange
is needed.
"""
from __future__ import annotations

import json
import os
import sys
import time

from . import MODE_KERNEL, PART_PEER, PART_SUBTREE, Engine, device_count, ipc_group_id, load, unique_id
from . import workloads as WL


def env_ranks():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init(backend: str):
    """Initialises the default process group (rendezvous on 127.0.0.1)."""
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    os.environ.setdefault("RANK", "0")  # a single process (bench.py --force-dist)
    os.environ.setdefault("WORLD_SIZE", "1")
    if not dist.is_initialized():
        dist.init_process_group(backend)
    return dist


def share_bytes(dist, make, rank: int) -> bytes:
    """Rank 0 makes a byte string (the RCCL unique id); every rank gets it."""
    obj = [make() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def job_totals(dist, elapsed_s: float, local_count: int, device=None):
    """(max elapsed over ranks, sum of counts over ranks), over gloo."""
    import torch

    del device  # (host tensors)
    t = torch.tensor([elapsed_s], dtype=torch.float64)
    c = torch.tensor([float(local_count)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), int(round(c.item()))


def workload(args, world: int):
    """The bench workload at `world` ranks (weak scaling: N x the messages)."""
    wl = WL.CONFIGS[args.workload]() if args.scale == 1.0 else WL.scaled(args.workload, args.scale)
    if getattr(args, "scaling", "weak") == "weak" and world > 1:
        import numpy as np

        wl.msg_topics = np.tile(wl.msg_topics, world)
    return wl


def pick_transport(requested: str, world: int, ndev: int) -> str:
    """The exchange transport of a `world`-rank run on `ndev` visible GPUs:
    RCCL (value's transport) when every rank has a GPU of its
    own; ranks that share GPUs (this pool's one-GPU boxes) take the IPC
    transport -- RCCL refuses two ranks on one device."""
    shared = world > max(1, ndev)
    if requested == "auto":
        return "ipc" if shared else "rccl"
    if requested == "rccl" and shared:
        raise SystemExit(f"[bench] {world} ranks on {ndev} GPU(s): RCCL refuses two ranks "
                         "on one device; use --transport ipc")
    if requested not in ("rccl", "ipc"):
        raise SystemExit(f"[bench] unknown transport {requested!r}")
    return requested


def bench_main(args, descr: dict, metric: str):
    rank, world, local = env_ranks()
    gpus = getattr(args, "gpus", world)
    if world != gpus:
        raise SystemExit(f"[bench] rank {rank}: WORLD_SIZE={world} but --gpus {gpus}; "
                         "the line would report the wrong n_gpus")
    # The engine's HIP/HSA/RCCL runtime (/opt/rocm, which libpsengine.so is
    # built against) is bound before torch loads its bundled ROCm 7.0 copies,
    # and torch.cuda is never touched, so only the engine's runtime initialises
    # the GPU.  (With torch imported first the engine bound torch's copies,
    # whose hipIpcOpenMemHandle of a >= 2 GiB allocation spins forever;
    # initialising both copies fails ps_create: profiles/r06/ipc/NOTES.md.)
    load()
    ndev = max(1, device_count())
    # RCCL prints its version banner on stdout when a communicator comes up:
    # keep stdout for the one JSON line (rank 0), everything else to stderr
    json_fd = os.dup(1)
    os.dup2(2, 1)
    local = local % ndev
    dist = init("gloo")
    if getattr(args, "message_only", False):
        # the message-sharded leg alone (no exchange)
        ms = message_sharded(args, dist, local, rank, world, descr)
        if rank == 0:
            sys.stdout.flush()
            os.write(json_fd, (json.dumps({"metric": metric + " [message-sharded leg only]", "n_gpus": world,
                                           "message_sharded": ms}) + "\n").encode())
        dist.barrier()
        dist.destroy_process_group()
        return
    shared = world > ndev
    transport = pick_transport(getattr(args, "transport", "auto"), world, ndev)
    dev = local
    tdev = None
    part = PART_SUBTREE if getattr(args, "partition", "peer") == "subtree" else PART_PEER
    ipc_mode = getattr(args, "ipc_mode", "inplace")
    out = partitioned(args, dist, dev, rank, world, descr, metric, part, transport, ipc_mode, tdev)
    if shared and world > 1:
        # N ranks sharing one GPU against one rank doing the same N x messages
        # alone: the cost of the partition and its exchange on one device
        one = one_rank_reference(args, dev, world) if rank == 0 else None
        if rank == 0:
            out["shared_gpu"] = {"ranks_per_gpu": world, "one_rank_ms_per_step": one,
                                 "ratio_vs_one_rank": out["ms_per_step"] / one,
                                 "note": f"{world} processes on one GPU, each owning 1/{world} of every tree, "
                                         f"against one engine disseminating the same {world} x messages alone"}
        dist.barrier()
    if world > 1 and not shared and transport == "rccl" and getattr(args, "ipc_leg", False):
        # the same partition with the owners' rows read in place over xGMI peer
        # mappings (IPC transport, PS_DIST_F_INPLACE): no records shipped
        # (opt-in: never run across separate GPUs on this pool's one-GPU boxes)
        try:
            leg = partitioned(args, dist, dev, rank, world, descr, metric, part, "ipc", "inplace", tdev)
            if rank == 0:
                out["ipc_in_place"] = {k: leg[k] for k in ("value", "unit", "ms_per_step", "roofline", "config")}
        except Exception as exc:  # noqa: BLE001
            print(f"[bench] rank {rank}: ipc_in_place leg failed: {exc!r}", file=sys.stderr, flush=True)
            if rank == 0:
                out["ipc_in_place"] = {"error": repr(exc)}
    if world > 1 and not shared and not getattr(args, "no_message_leg", False):
        # the decompositions SURVEY.md §8e allows beside the mandated peer hash,
        # on the same ranks: level-L subtrees (cross edges only above level L)
        # and message sharding (replicated topology, no exchange)
        # (a leg that fails on every rank alike -- memory, a communicator --
        # is reported in the line instead of losing the headline run above)
        other = PART_PEER if part == PART_SUBTREE else PART_SUBTREE
        key = "peer_partition" if other == PART_PEER else "subtree_partition"
        try:
            leg = partitioned(args, dist, dev, rank, world, descr, metric, other, transport, ipc_mode, tdev)
            if rank == 0:
                keep = ("value", "unit", "ms_per_step", "roofline", "config")
                out[key] = {k: leg[k] for k in keep}
        except Exception as exc:  # noqa: BLE001
            print(f"[bench] rank {rank}: {key} leg failed: {exc!r}", file=sys.stderr, flush=True)
            if rank == 0:
                out[key] = {"error": repr(exc)}
        try:
            ms = message_sharded(args, dist, dev, rank, world, descr, totals_dev=tdev)
            if rank == 0:
                out["message_sharded"] = ms
        except Exception as exc:  # noqa: BLE001
            print(f"[bench] rank {rank}: message_sharded leg failed: {exc!r}", file=sys.stderr, flush=True)
            if rank == 0:
                out["message_sharded"] = {"error": repr(exc)}
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    dist.barrier()
    dist.destroy_process_group()


def partitioned(args, dist, dev, rank: int, world: int, descr: dict, metric: str, part: int,
                transport: str = "rccl", ipc_mode: str = "inplace", tdev=None):
    """The node-partitioned run: every rank owns a hash (PART_PEER) or
    subtree (PART_SUBTREE) share of every tree; the frontier rows that cross
    ranks are exchanged each round over the engine's RCCL communicator, or
    (transport "ipc", one process per rank on one node) read through IPC
    mappings of the other ranks' buffers: the owners' rows in place
    (ipc_mode "inplace"), the senders' records in place ("zc") or copied
    ("copy").  Returns the bench JSON object on rank 0 (None elsewhere)."""
    local = int(dev)
    wl = workload(args, world)
    scaling = getattr(args, "scaling", "weak") if world > 1 else "weak"
    uid = share_bytes(dist, ipc_group_id if transport == "ipc" else unique_id, rank)
    t0 = time.perf_counter()
    # one window per topic (pull kernels take rows of any width)
    eng = Engine(wl.n_peers, len(wl.topics), device=local, seed=wl.seed, msg_window=1 << 20)
    if transport == "ipc":
        eng.dist_init_ipc(rank, world, uid, part, copy=ipc_mode == "copy", inplace=ipc_mode == "inplace")
    else:
        eng.dist_init(rank, world, uid, part)
    sizes = WL.build_engine_topics(eng, wl)
    expected = wl.expected_deliveries(sizes)
    pname = "peer" if part == PART_PEER else "subtree"
    if rank == 0:
        print(f"[bench] {wl.name} on {world} GPUs ({pname} partition), setup {time.perf_counter() - t0:.1f}s",
              file=sys.stderr, flush=True)

    def step():
        eng.publish(wl.msg_topics)
        return eng.run()

    for _ in range(args.warmup):
        st = step()
    _, warm = job_totals(dist, 0.0, st.deliveries if args.warmup else 0, tdev)
    if args.warmup and not args.no_check:
        assert warm == expected, (warm, expected)
    dist.barrier()
    t0 = time.perf_counter()
    local_deliv = 0
    if getattr(args, "sync", False):
        for _ in range(args.steps):
            st = step()
            local_deliv += st.deliveries
    else:
        # pipelined like bench.py: batch k + 1 is published and enqueued (its
        # RCCL exchanges included, stream-ordered) while batch k runs
        for i in range(args.steps):
            eng.publish(wl.msg_topics)
            eng.run_async()
            if i:
                local_deliv += eng.wait().deliveries
        if args.steps:
            local_deliv += eng.wait().deliveries
    dist.barrier()
    elapsed = time.perf_counter() - t0
    wall, total = job_totals(dist, elapsed, local_deliv, tdev)
    # roofline pass: HIP events around every hot-kernel launch (untimed above)
    eng.set_time_kernels(True)
    bytes_, exp_ms, launches = 0, 0.0, 0
    for _ in range(3):
        st = step()
        bytes_ += st.expand_bytes
        exp_ms += st.expand_ms
        launches += st.expand_launches
    eng.set_time_kernels(False)
    _, tot_bytes = job_totals(dist, 0.0, bytes_, tdev)
    slow_exp_ms, _ = job_totals(dist, exp_ms, 0, tdev)
    if not args.no_check:
        assert total == expected * args.steps, (total, expected * args.steps)
    out = None
    if rank == 0:
        value = total / wall
        # per GPU: the job's expand bytes over the slowest rank's expand time / N
        achieved = tot_bytes / max(1e-12, slow_exp_ms * 1e-3) / 1e9 / world
        out = {
            "metric": metric,
            "value": value,
            "unit": "deliveries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": f"{wl.name}: {descr[wl.name]}", "peers": wl.n_peers,
                       "topics": len(wl.topics), "subscriptions": int(sum(sizes)),
                       "messages": wl.n_msgs, "deliveries_per_step": expected,
                       "parallelism": f"{world} ranks, nodes partitioned ({pname}), " + (
                           "RCCL all-to-allv frontier exchange per round" if transport == "rccl" else
                           f"IPC transport ({ipc_mode}: "
                           + {"inplace": "owners' rows read in place", "zc": "senders' records read in place",
                              "copy": "records copied"}[ipc_mode] + "), device-flag ordered rounds")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0, "traffic": None,
                         "kernel": MODE_KERNEL.get(st.expand_mode, "k_expand"),
                         "note": "per-GPU: job expand bytes / slowest rank's expand time / N"},
            "last_step_rank0": {"rounds": st.rounds, "run_ms": st.run_ms,
                                "expand_ms": st.expand_ms, "host_ms": st.host_ms,
                                "xchg_path": {0: "none", 1: "zero-copy", 2: "copy", 3: "in-place"}.get(int(st.xchg_path)),
                                "xchg_rounds": st.xchg_rounds, "xchg_bytes_received": st.xchg_bytes,
                                "max_rounds_per_launch": st.plan_max_rounds},
            "plan_opts": eng.plan_opts(),
        }
    eng.close()
    return out


def one_rank_reference(args, dev, world: int) -> float:
    """ms per step of one engine (no partition) disseminating the weak-scaled
    workload's world x messages alone, pipelined like the partitioned run."""
    wl = workload(args, world)
    local = int(dev)
    eng = Engine(wl.n_peers, len(wl.topics), device=local, seed=wl.seed, msg_window=1 << 20)
    try:
        sizes = WL.build_engine_topics(eng, wl)
        expected = wl.expected_deliveries(sizes)
        for _ in range(max(1, args.warmup)):
            eng.publish(wl.msg_topics)
            assert args.no_check or eng.run().deliveries == expected
        t0 = time.perf_counter()
        for i in range(args.steps):
            eng.publish(wl.msg_topics)
            eng.run_async()
            if i:
                eng.wait()
        if args.steps:
            eng.wait()
        return (time.perf_counter() - t0) * 1e3 / max(1, args.steps)
    finally:
        eng.close()


def message_sharded(args, dist, dev, rank: int, world: int, descr: dict, totals_dev=None) -> dict:
    """Every rank: a one-GPU engine over the whole topology, its own batch of
    the N=1 workload's messages (weak scaling: N x the messages in all), the
    same pipelined steps; the job's deliveries over the slowest rank's time."""
    wl = WL.CONFIGS[args.workload]() if args.scale == 1.0 else WL.scaled(args.workload, args.scale)
    local = int(dev)
    eng = Engine(wl.n_peers, len(wl.topics), device=local, seed=wl.seed)
    sizes = WL.build_engine_topics(eng, wl)
    expected = wl.expected_deliveries(sizes)
    for _ in range(args.warmup):
        eng.publish(wl.msg_topics)
        st = eng.run()
        assert args.no_check or st.deliveries == expected
    dist.barrier()
    t0 = time.perf_counter()
    local_deliv = 0
    for i in range(args.steps):
        eng.publish(wl.msg_topics)
        eng.run_async()
        if i:
            local_deliv += eng.wait().deliveries
    if args.steps:
        local_deliv += eng.wait().deliveries
    dist.barrier()
    elapsed = time.perf_counter() - t0
    wall, total = job_totals(dist, elapsed, local_deliv, totals_dev)
    eng.close()
    if not args.no_check:
        assert total == expected * args.steps * world, (total, expected * args.steps * world)
    return {"value": total / wall, "unit": "deliveries/s", "ms_per_step": wall * 1e3 / max(1, args.steps),
            "workload": f"{wl.name}: each of {world} ranks disseminates {wl.n_msgs} messages over the whole "
                        "topology (replicated CSR, no exchange; SURVEY.md §8e alternative)",
            "scaling": "weak"}
