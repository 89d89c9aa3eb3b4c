#!/usr/bin/env python3
"""Benchmark of the subtree-dissemination hot path (BASELINE.json metric).

A step = one ps_run over one batch of synthetic publishes of the workload
(default cfg3: 1M peers, 64 topics with Zipf subscriptions, 100k messages),
topology already resident in HBM.  Prints ONE JSON line (rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3]

N > 1 runs one process per GPU: under torch.distributed.run (WORLD_SIZE must
equal --gpus), or, started without a launcher, bench.py starts that launcher
itself as a child process (launch_plan).  Peers are hash-partitioned
(owner(p) = splitmix64(p) mod N) and the per-round frontier exchange runs over
RCCL (see psengine/dist.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402

METRIC = "deliveries/sec (peer×msg) at 1M peers, 1/2/4/8 GPU; % of HBM roofline"
TRAFFIC_FILE = os.path.join(REPO, "profiles", "pmc_traffic.json")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PAIR_BYTES = 28.375  # SURVEY.md §8d bytes/delivery of the (peer,msg)-pair formulation
# HBM rates this pool's MI355X reaches (context for frac; peak stays the spec)
MEASURED_CEILINGS = {"copy_read_plus_write_GBs": [5400, 5700], "write_only_GBs": [5800, 6100],
                     "hipMemset_GBs": [6500, 6700],
                     "source": "tools/probe/hbm_write_probe.hip, profiles/r02/hbm_probe.txt"}

DESCR = {
    "cfg2": "100k peers, 1 topic, TreeOpts{8,20}, 10k-message burst",
    "cfg3": "1M peers, 64 topics, Zipf(1) subscriptions, W=2/MaxW=5, 100k msgs Zipf(1) over topics",
    "cfg4": "16M peers, 1 topic, W=8/MaxW=20, 1k-message burst",
    "cfg5": "1M peers, 1 topic, W=2/MaxW=5, 90% subscribed; per batch 1% leave (Part + repair) "
            "and 1% join, then a 1k-message burst; tree maintenance + CSR rebuild + propagation "
            "end to end",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads():
    """Host threads the CPU legs use: this process's CPU share (affinity mask,
    capped by OMP_NUM_THREADS where the box sets it), and what the host reports."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = max(1, min(aff, int(omp)) if omp and omp.isdigit() else aff)
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return threads, {"os_cpu_count": os.cpu_count(), "affinity": aff, "omp_num_threads": omp,
                     "cgroup_cpus": cgroup_cpus(), "model": model}


def cgroup_cpus():
    """CPUs this process's cgroup may use (cpu.max / cfs quota), or None when
    unlimited.  On the GPU box the quota is the GPU's share of the host (~16 of
    256): 256 OpenMP threads on it time-slice every level barrier (measured:
    one cfg3 pass took 124 s, 2.8e8 deliveries/s)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            per = int(fh.read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(eng, wl, sizes, budget_s: float = 10.0, deliv_expected=None):
    """The CPU restatements (oracle/, ports) timed on the host's cores, on the
    same trees and the same message mix:
      value        or_levels_run -- the algorithm the GPU runs (messages as
                   bits, rounds level-synchronous, OpenMP over each level's
                   nodes), whole passes of the workload, on every host thread
                   the process may run (the affinity mask,
                   capped by the cgroup CPU quota -- not by OMP_NUM_THREADS),
                   a third of the budget; the per-topology work (BFS numbering, rows allocated
                   and touched) is done once before, as the GPU's timed steps
                   exclude the node-space build;
      share        the same on this process's CPU share (affinity capped by
                   OMP_NUM_THREADS: 16 on the GPU box), a third of the budget;
      per_message  or_disseminate -- one BFS per message (subtree.go:319-354 +
                   client.go:100-132 literally), OpenMP over messages, on a
                   growing sample of the messages for the last third.
    Every pass's deliveries are checked against the workload's."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    share, host = host_threads()
    # every host thread the process may run (threads = nproc),
    # within the cgroup's CPU quota where there is one
    every = max(1, min(host["affinity"], host["cgroup_cpus"] or host["affinity"]))
    graphs = {}
    for t in range(len(wl.topics)):
        rp, cl = O.parents_to_csr(eng.parents(t))
        graphs[t] = (rp, cl)
    live = np.ones(wl.n_peers, dtype=np.uint8)
    counts = np.bincount(wl.msg_topics, minlength=len(wl.topics))
    plans = {t: O.Levels(*graphs[t], wl.topics[t].root, int(k)) for t, k in enumerate(counts) if k}
    for t, pl in plans.items():  # untimed: first touch of every row page
        pl.run(live, threads=share)

    def bits_leg(threads, budget):
        deliv, spent, passes = 0, 0.0, 0
        while passes == 0 or spent < budget:
            t0 = time.perf_counter()
            got = sum(pl.run(live, threads=threads) for pl in plans.values())
            spent += time.perf_counter() - t0
            passes += 1
            if deliv_expected is not None:
                assert got == deliv_expected, (got, deliv_expected)
            deliv += got
        return deliv, spent, passes

    all_d, all_s, all_p = bits_leg(every, budget_s / 3)
    sh_d, sh_s, sh_p = bits_leg(share, budget_s / 3) if share != every else (all_d, all_s, all_p)
    for pl in plans.values():
        pl.close()
    # per-message BFS: a growing sample, topic mix kept
    frac = 0.0005
    done_deliv, done_msgs, spent = 0, 0, 0.0
    while spent < budget_s / 3 and frac <= 1.0:
        per_topic = np.maximum(1, np.round(counts.astype(np.float64) * frac)).astype(int)
        per_topic[counts == 0] = 0
        t0 = time.perf_counter()
        for t, k in enumerate(per_topic):
            if k:
                tot, _, _ = O.disseminate(*graphs[t], wl.topics[t].root, live, int(k),
                                          want_hops=False, threads=share)
                done_deliv += tot
                done_msgs += int(k)
        spent += time.perf_counter() - t0
        frac *= 2
    algo = ("oracle/psoracle.c or_levels_run, the GPU's algorithm restated (64 messages per u64, "
            "level-synchronous rounds, OpenMP over each level's nodes; BFS numbering and row "
            "allocation once per topic, untimed); Go reference not buildable (no go toolchain)")
    return {"value": all_d / all_s, "unit": "deliveries/s", "cores": every, "kind": "port",
            "host": host,
            "sample": f"{all_p} whole pass(es) of the workload ({all_d} deliveries, {all_s:.1f} s on "
                      f"{every} host threads: every CPU of the affinity mask within the cgroup quota"
                      f" (os.cpu_count() {os.cpu_count()}, quota {host['cgroup_cpus']})): {algo}",
            "share": {"value": sh_d / sh_s, "unit": "deliveries/s", "cores": share, "kind": "port",
                      "sample": f"{sh_p} whole pass(es), {sh_d} deliveries, {sh_s:.1f} s on {share} threads "
                                "(this process's CPU share: affinity capped by OMP_NUM_THREADS)"},
            "per_message": {"value": done_deliv / spent, "unit": "deliveries/s", "cores": share,
                            "kind": "port",
                            "sample": f"{done_msgs} of the workload's messages (topic mix kept), {done_deliv} "
                                      f"deliveries, {spent:.1f} s: oracle/psoracle.c or_disseminate, one BFS "
                                      "per message restating subtree.go:319-354 + client.go:100-132, "
                                      "OpenMP over messages"}}


def cpu_baseline_cfg5(wl, plan, budget_s: float = 10.0):
    """cfg5 on the CPU restatement (oracle/, a port), end to end per batch:
    the restated leaves / joins (psoracle.c Tree), the attached tree as CSR,
    the batch's messages by the GPU's algorithm restated (or_levels_bits:
    messages as bits, level-synchronous rounds, OpenMP over each level) and the
    lazy prune pass -- as many batches of the plan as fit the budget."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    threads, host = host_threads()
    ot = O.Tree(wl.n_peers, 0, 2, 5, PE.Engine.topic_seed(wl.seed, 0))
    ot.join_all(wl.topics[0].join_order)
    live = np.ones(wl.n_peers, dtype=np.uint8)
    deliv, spent, batches = 0, 0.0, 0
    for leave, join in plan:
        if spent >= budget_s:
            break
        t0 = time.perf_counter()
        for p in leave:
            ot.leave(int(p))
        for p in join:
            ot.join(int(p))
        rp, cl = O.parents_to_csr(ot.parents())
        tot = O.levels_bits(rp, cl, 0, live, wl.n_msgs, threads=threads)
        ot.message()  # lazy prune / repair after the batch's first message
        spent += time.perf_counter() - t0
        deliv += tot
        batches += 1
    return {"value": deliv / spent, "unit": "deliveries/s", "cores": threads, "kind": "port", "host": host,
            "sample": f"{batches} batches of the cfg5 churn plan from the initial tree "
                      f"({deliv} deliveries, {spent:.1f} s on {threads} host threads): "
                      "oracle/psoracle.c tree restatement + or_levels_bits"}


def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE runs of this bench), or None."""
    try:
        with open(TRAFFIC_FILE) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    for x in d.get("entries", []):
        if x.get("kernel") == kernel and x.get("workload") == workload:
            return x.get("traffic_bytes_per_launch"), x.get("source")
    return None, None


def kernel_split(st):
    """{kernel: (algorithmic bytes, device ms, launches)} of one run, by the
    rocprofv3 names of the launches that ran its rounds (ps_stats.round_kernel
    where the engine reports it): k_flood (the leading rounds of a single-rank
    level window, one persistent launch, timed into round 1), k_pull (one
    launch per round), k_pull_pair (two rounds per launch, timed into the
    first) or k_expand (compaction mode)."""
    kern = PE.MODE_KERNEL.get(st.expand_mode, "k_expand")
    fr = int(getattr(st, "flood_rounds", 0))
    kinds = list(getattr(st, "round_kernel", []))
    n = min(int(st.rounds), PE.MAX_ROUNDS - 1)
    if st.windows == 1 and any(kinds[1:n + 1]) and st.expand_mode != PE.MODE_COMPACT:
        per = {}
        for q in range(1, n + 1):
            name = PE.ROUND_KERNEL.get(kinds[q])
            if name is None:
                continue
            acc = per.setdefault(name, [0, 0.0, 0])
            acc[0] += int(st.expand_bytes_per_round[q])
            acc[1] += float(st.expand_ms_per_round[q])
            first = {PE.K_FLOOD: q == 1, PE.K_PULL: int(st.expand_bytes_per_round[q]) > 0,
                     PE.K_PAIR: True, PE.K_CHAIN: True}.get(kinds[q], False)
            acc[2] += 1 if first else 0
        return {k: tuple(v) for k, v in per.items()}
    if st.expand_mode != PE.MODE_FLOOD or fr >= st.rounds or st.windows != 1:
        return {kern: (st.expand_bytes, st.expand_ms, st.expand_launches)}
    bf = sum(int(st.expand_bytes_per_round[q]) for q in range(1, fr + 1))
    tf = float(st.expand_ms_per_round[1])
    return {"k_flood": (bf, tf, 1),
            "k_pull": (st.expand_bytes - bf, st.expand_ms - tf, st.expand_launches - 1)}


def hot_kernel(st):
    """The kernel the roofline is quoted on: of kernel_split's launches, the
    one with the most device time (by bytes when untimed)."""
    sp = kernel_split(st)
    return max(sp, key=lambda k: (sp[k][1], sp[k][0]))


def instrumented(eng, step, n):
    """Roofline pass: n steps with HIP events around every hot-kernel launch
    on the engine's stream (PS_F_TIME_KERNELS); the timed steps run without.
    Returns ({kernel: [bytes, ms, launches]}, last stats)."""
    eng.set_time_kernels(True)
    per, st = {}, None
    for _ in range(n):
        st = step()
        for k, v in kernel_split(st).items():
            acc = per.setdefault(k, [0, 0.0, 0])
            for i in range(3):
                acc[i] += v[i]
    eng.set_time_kernels(False)
    return per, st


def roofline_of(per, traffic=None, traffic_src=None):
    """The roofline object for the dominant kernel of `per` (the most device
    time), with every kernel's own figures under "kernels"."""
    def fig(k):
        b, ms, n = per[k]
        gbs = b / max(1e-12, ms * 1e-3) / 1e9
        return {"achieved": gbs, "frac": gbs / HBM_PEAK_GBS, "avg_launch_us": ms * 1e3 / max(1, n),
                "bytes_per_launch": b / max(1, n), "launches": n, "device_ms": ms}
    hot = max(per, key=lambda k: (per[k][1], per[k][0]))
    f = fig(hot)
    return {"bound": "hbm", "achieved": f["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": f["frac"], "traffic": traffic, "kernel": hot, "avg_launch_us": f["avg_launch_us"],
            "measured_ceilings": MEASURED_CEILINGS,
            "bytes_per_launch": f["bytes_per_launch"],
            "timing": "HIP events around every launch on the engine stream, "
                      "separate instrumented steps after the timed region",
            "traffic_source": traffic_src,
            "kernels": {k: fig(k) for k in sorted(per)}}


def bench_cfg5(args):
    """cfg5 end to end: a step = one batch = churn (graceful leaves with the
    restated repair, joins through the restated join protocol) + node-space /
    CSR rebuild + upload + propagation of the batch's messages."""
    wl = WL.CONFIGS["cfg5"]() if args.scale == 1.0 else WL.scaled("cfg5", args.scale)
    t0 = time.perf_counter()
    eng = PE.Engine(wl.n_peers, 1, seed=wl.seed)
    WL.build_engine_topics(eng, wl)
    plan = WL.churn_plan(wl, args.warmup + args.steps + 3)
    log(f"[bench] cfg5: {wl.n_peers} peers, {wl.topics[0].join_order.size} initial members, "
        f"setup {time.perf_counter() - t0:.1f}s")

    def churn(b):
        leave, join = plan[b]
        tc = time.perf_counter()
        try:
            eng.leave(0, leave)
        except PE.EngineError:
            pass  # orphaned peers cannot Part (their client panicked, client.go:96-98)
        tl = time.perf_counter()
        eng.join(0, join, check=False)
        tj = time.perf_counter()
        eng.publish(wl.msg_topics)
        return tl - tc, tj - tl

    def step(b):
        c = churn(b)
        return eng.run(), c

    for b in range(args.warmup):
        step(b)
    # pipelined like the other workloads: batch b's churn (host: the restated
    # leaves and joins), rebuild, plan and launch; its propagation runs while
    # batch b + 1's churn runs on the host (ps_run_async / ps_wait; a batch's
    # rebuild waits for the previous batch's kernels, its lazy prune only
    # for its own node space)
    tot, leave_s, join_s, run_host, run_gpu, wait_s = 0, 0.0, 0.0, 0.0, 0.0, 0.0
    t0 = time.perf_counter()
    for k, b in enumerate(range(args.warmup, args.warmup + args.steps)):
        cl, cj = churn(b)
        tr = time.perf_counter()
        eng.run_async()
        ta = time.perf_counter()
        leave_s += cl
        join_s += cj
        run_host += (ta - tr) * 1e3
        if k:
            st = eng.wait()
            wait_s += time.perf_counter() - ta
            tot += st.deliveries
            run_gpu += st.run_ms
    tw = time.perf_counter()
    st = eng.wait()
    wait_s += time.perf_counter() - tw
    tot += st.deliveries
    run_gpu += st.run_ms
    wall = time.perf_counter() - t0
    gpu_ms = []  # device span of the blocking instrumented batches (init start .. reduce end)

    def blocking(it=iter(range(args.warmup + args.steps, args.warmup + args.steps + 3))):
        st_b = step(next(it))[0]
        gpu_ms.append(st_b.run_ms)
        return st_b

    per, st = instrumented(eng, blocking, 3)
    out = {
        "metric": METRIC + " [cfg5 end to end]",
        "value": tot / wall,
        "unit": "deliveries/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"cfg5: {DESCR['cfg5']}", "peers": wl.n_peers,
                   "messages_per_batch": wl.n_msgs, "parallelism": "1 GPU"},
        "breakdown_ms_per_step": {"leave_host": leave_s * 1e3 / args.steps,
                                  "join_host": join_s * 1e3 / args.steps,
                                  "ps_run_async_host": run_host / args.steps,
                                  "ps_wait": wait_s * 1e3 / args.steps,
                                  "ps_run_gpu": sum(gpu_ms) / len(gpu_ms),
                                  "window_span_pipelined": run_gpu / args.steps,
                                  "note": "ps_run_async_host = rebuild + plan + launch + lazy prune of the batch "
                                          "(host wall inside the call); its propagation overlaps the next "
                                          "batch's churn. ps_run_gpu = the window's device span (init start .. "
                                          "reduce end) in the blocking instrumented batches; "
                                          "window_span_pipelined = the same stamps in the timed pipelined "
                                          "batches, where a window's counter reduce rides in the next batch's "
                                          "first launch (after that batch's host churn)"},
        "roofline": roofline_of(per),
        "last_step": {"deliveries": st.deliveries, "rounds": st.rounds, "host_ms": st.host_ms,
                      "run_ms": st.run_ms},
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_cfg5(wl, plan, args.cpu_budget)
    print(json.dumps(out), flush=True)
    eng.close()


def general_path(eng, wl, deliv_expected, steps: int, warmup: int = 1, max_start: int = 7, compact_steps: int = 2):
    """The general path: the same workload published with staggered start
    rounds, uniform over 0..max_start -- paced publishing as the reference's
    tests do it (pubsub_test.go:101-131).  Level mode runs each topic's
    window as start groups (one word block per start round, k_pull per
    round); the same steps forced through the compaction path (PS_F_COMPACT:
    k_expand over a compacted frontier with the seen test-and-set,
    client.go:103-131) are timed beside it.  On a tree every message still
    reaches every subscriber: the same deliveries."""
    starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(max_start + 1)).astype(np.uint32)

    def step():
        eng.publish(wl.msg_topics, starts)
        return eng.run()

    def leg(modes, n_steps):
        for _ in range(warmup):
            st = step()
            assert st.deliveries == deliv_expected, (st.deliveries, deliv_expected)
            assert st.expand_mode in modes, (st.expand_mode, modes)
        # pipelined like the headline: batch k + 1 is published and planned
        # while batch k's kernels run; every batch completes inside the region
        t0 = time.perf_counter()
        tot = 0
        eng.publish(wl.msg_topics, starts)
        for i in range(n_steps):
            eng.run_async()
            if i + 1 < n_steps:  # (batch i + 1 published before waiting for i - 1, as steps_pipelined)
                eng.publish(wl.msg_topics, starts)
            if i:
                tot += eng.wait().deliveries
        tot += eng.wait().deliveries
        wall = time.perf_counter() - t0
        assert tot == deliv_expected * n_steps
        per, st = instrumented(eng, step, 2)
        hot = max(per, key=lambda k: (per[k][1], per[k][0]))
        roof = roofline_of(per, *pmc_traffic(hot, f"{wl.name}-staggered"))
        roof["device_ms_per_step"] = sum(v[1] for v in per.values()) / 2
        d = st.as_dict()
        return {"value": tot / wall, "unit": "deliveries/s", "steps": n_steps, "ms_per_step": wall * 1e3 / n_steps,
                "rounds": st.rounds, "level_aligned": int(st.level_aligned), "roofline": roof,
                "expand_us_per_round": [round(x * 1e3, 1) for x in d["expand_ms_per_round"]],
                "mbytes_per_round": [round(x / 1e6, 1) for x in d["expand_bytes_per_round"]]}

    flags = eng.flags
    out = leg((PE.MODE_FLOOD, PE.MODE_LEVEL_PULL), steps)
    out["workload"] = (f"{wl.name} with start rounds uniform over 0..{max_start} (paced publishing): "
                       "start groups, level-aligned (launch round q writes BFS level q of every group; "
                       "each group's deliveries counted in round start + q)")
    out["deliveries_per_step"] = deliv_expected
    eng.set_flags(flags | PE.F_COMPACT)
    try:
        comp = leg((PE.MODE_COMPACT,), compact_steps)
    finally:
        eng.set_flags(flags)
    comp["workload"] = "the same steps through the compaction path (PS_F_COMPACT): k_expand + frontier compaction"
    comp["note"] = ("k_expand moves only arrival extents (one start-group block per node and round); short "
                    "entries go through flattened (child, word) passes (round 6: ~39 SALU per entry, was 224), "
                    "and what bounds it is each batch's chain of dependent metadata loads, not HBM: SQ counters "
                    "and A/B records in profiles/r06/expand/NOTES.md")
    out["compaction"] = comp
    return out


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(args, env, argv, port=None):
    """How this invocation gets its ranks, decided before any GPU call:
      None          run here (one GPU, or a rank of a torchrun launch whose
                    WORLD_SIZE equals --gpus);
      [cmd, ...]    --gpus N > 1 without a launcher: start N ranks as a child
                    `python -m torch.distributed.run` (rendezvous on
                    127.0.0.1) with the same arguments; its rank 0 prints the line;
      "message"     refuse: a launch whose rank count differs from --gpus
                    (the line would report the wrong n_gpus), or cfg5 on N > 1.
    So no invocation can print a line whose n_gpus differs from --gpus."""
    ws = env.get("WORLD_SIZE")
    if args.gpus < 1:
        return f"--gpus {args.gpus}: need at least 1"
    if args.workload == "cfg5" and (args.gpus > 1 or (ws is not None and int(ws) > 1)):
        return "cfg5 (churn end to end) is a single-GPU workload: run it with --gpus 1"
    if ws is None:
        if args.gpus == 1:
            return None
        return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
                "--master-addr=127.0.0.1", f"--master-port={port or free_port()}",
                os.path.abspath(__file__)] + list(argv)
    if int(ws) != args.gpus:
        return f"launched with WORLD_SIZE={ws} but --gpus {args.gpus}: they must agree"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 500 on one GPU -- 0.7 s of back-to-back cfg3 batches, "
                         "long enough for a utilisation sampler to see -- and 10 for cfg5 or N > 1)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg3", choices=sorted(DESCR))
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the workload (debug)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--sustain", type=float, default=8.0,
                    help="seconds of back-to-back pipelined steps after the timed region (one GPU; "
                         "reported under 'sustained', not in value); 0 skips")
    ap.add_argument("--no-check", action="store_true", help="skip delivery assertions (experiments)")
    ap.add_argument("--no-general", action="store_true",
                    help="skip the general-path leg (staggered starts, compaction mode)")
    ap.add_argument("--general-only", action="store_true",
                    help="run only the general-path leg and print it as the JSON line (its PMC passes)")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the torch.distributed driver even with one rank (testing)")
    ap.add_argument("--partition", default="peer", choices=["peer", "subtree"],
                    help="multi-GPU node ownership: peer hash owner(p) = splitmix64(p) mod N (default, "
                         "SURVEY.md §8e) or level-L subtrees")
    ap.add_argument("--sync", action="store_true",
                    help="one blocking ps_run per step (default: pipelined ps_run_async / ps_wait, "
                         "the next batch is published and planned while the previous one's kernels run)")
    ap.add_argument("--no-message-leg", action="store_true",
                    help="N>1: skip the alternative decompositions (the other partition, and message "
                         "sharding: replicated topology, no exchange)")
    ap.add_argument("--message-only", action="store_true",
                    help="N>1: only the message-sharded leg (gloo bootstrap, no RCCL; testing)")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "ipc"],
                    help="N>1: the frontier exchange -- rccl (value's transport, a GPU per rank), ipc (one "
                         "process per rank, buffers mapped across processes; ranks may share a GPU); auto = "
                         "rccl when every rank has its own GPU, else ipc")
    ap.add_argument("--ipc-leg", action="store_true",
                    help="N>1 on separate GPUs: also time the peer partition over the IPC transport, owners' rows "
                         "read in place over xGMI peer mappings (the `ipc_in_place` leg)")
    ap.add_argument("--ipc-mode", default="inplace", choices=["inplace", "zc", "copy"],
                    help="--transport ipc: owners' rows read in place (no records), senders' records read in "
                         "place, or records copied into the receive buffer")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N>1: weak = N x the messages on the same topology (per-GPU work of "
                         "N=1), strong = the N=1 workload unchanged")
    args = ap.parse_args()

    # --gpus N: N ranks, whoever starts us (before anything touches the GPU)
    plan = launch_plan(args, os.environ, sys.argv[1:])
    if plan is not None:
        if isinstance(plan, str):
            log(f"[bench] {plan}")
            sys.exit(2)
        log(f"[bench] starting {args.gpus} ranks: {' '.join(plan)}")
        sys.exit(subprocess.run(plan).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.steps is None:
        one = args.gpus <= 1 and world <= 1 and not args.force_dist
        args.steps = 500 if one and args.workload != "cfg5" else 10
    if args.workload == "cfg5":
        return bench_cfg5(args)
    if args.gpus > 1 or world > 1 or args.force_dist:
        from psengine import dist

        return dist.bench_main(args, DESCR, METRIC)

    wl = WL.CONFIGS[args.workload]() if args.scale == 1.0 else WL.scaled(args.workload, args.scale)
    t0 = time.perf_counter()
    eng = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
    sizes = WL.build_engine_topics(eng, wl)
    deliv_expected = wl.expected_deliveries(sizes)
    log(f"[bench] {wl.name}: {wl.n_peers} peers, {len(wl.topics)} topics, {sum(sizes)} "
        f"subscriptions, {wl.n_msgs} msgs, setup {time.perf_counter() - t0:.1f}s")

    def step():
        eng.publish(wl.msg_topics)
        return eng.run()

    if args.general_only:
        g = general_path(eng, wl, deliv_expected, max(2, min(args.steps, 100)), warmup=max(1, args.warmup))
        print(json.dumps({"metric": METRIC + " [general path only]", "general_path": g}), flush=True)
        eng.close()
        return

    def steps_pipelined(n):
        """n steps, each batch published and enqueued while the previous
        batch's kernels run; every batch completes inside the call."""
        out = []
        if n:
            eng.publish(wl.msg_topics)
        for i in range(n):
            eng.run_async()
            # batch i + 1 published while batches i - 1 and i run, so the wait
            # below returns straight into its enqueue (cfg2 35.3 -> 34.9 us,
            # cfg3 0.870 -> 0.864 ms/step: profiles/r06/ab/publish_ahead.txt)
            if i + 1 < n:
                eng.publish(wl.msg_topics)
            if i:
                out.append(eng.wait())
        if n:
            out.append(eng.wait())
        return out

    def steps(n):
        return [step() for _ in range(n)] if args.sync else steps_pipelined(n)

    for st in steps(args.warmup):
        assert args.no_check or st.deliveries == deliv_expected, (st.deliveries, deliv_expected)
    t0 = time.perf_counter()
    sts = steps(args.steps)
    wall = time.perf_counter() - t0
    overlapped_timed = sum(int(st.overlapped) for st in sts)
    tot_deliv = sum(st.deliveries for st in sts)
    assert args.no_check or tot_deliv == deliv_expected * args.steps
    value = tot_deliv / wall
    per, st = instrumented(eng, step, max(3, min(args.steps, 5)))
    assert args.no_check or st.deliveries == deliv_expected
    kernel = max(per, key=lambda k: (per[k][1], per[k][0]))
    traffic, traffic_src = pmc_traffic(kernel, wl.name)
    pair_gbs = value * PAIR_BYTES / 1e9
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "deliveries/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"{wl.name}: {DESCR[wl.name]}", "peers": wl.n_peers,
                   "topics": len(wl.topics), "subscriptions": int(sum(sizes)),
                   "messages": wl.n_msgs, "deliveries_per_step": deliv_expected,
                   "parallelism": "1 GPU",
                   "steps_issue": "blocking ps_run" if args.sync else
                   "pipelined ps_run_async/ps_wait (<= 2 batches in flight)"},
        "roofline": roofline_of(per, traffic, traffic_src),
        # SURVEY.md §8d's (peer,msg)-pair formulation: the HBM rate a pair-frontier
        # engine would need for this delivery rate.  A model figure, NOT bandwidth
        # this engine moves; compare roofline.frac, not this, with the peak.
        "pair_model": {"bytes_per_delivery": PAIR_BYTES, "equiv_GBs_not_achievable": pair_gbs,
                       "note": "model-equivalent rate of the 28.375 B/delivery pair formulation; "
                               "this engine moves 64 messages per 8-B word (roofline.bytes_per_launch)"},
        # the plan the timed steps ran: the engine's plan options (ps_get_plan_opts:
        # the measured defaults; the environment cannot change them) and the
        # effective plan of the last window
        "plan": {"opts": eng.plan_opts(), "max_rounds_per_launch": st.plan_max_rounds,
                 "prefix_rounds": st.prefix_rounds, "flood_rounds": st.flood_rounds,
                 "overlapped_windows_timed": overlapped_timed},
        "last_step": {"rounds": st.rounds, "windows": st.windows, "flood_rounds": st.flood_rounds,
                      "run_ms": st.run_ms,
                      "expand_ms": st.expand_ms, "host_ms": st.host_ms,
                      "edge_words": st.edge_words,
                      "frontier_per_round": st.as_dict()["frontier_per_round"],
                      "deliveries_per_round": st.as_dict()["deliveries_per_round"],
                      "mbytes_per_round": [round(x / 1e6, 1) for x in st.as_dict()["expand_bytes_per_round"]],
                      "expand_us_per_round": [round(x * 1e3, 1) for x in
                                              st.as_dict()["expand_ms_per_round"]]},
    }
    if args.sustain > 0:
        # the same pipelined steps back to back for a few seconds after the
        # timed region: sustained throughput, and device activity long enough
        # for a utilisation sampler polling every few seconds to see
        n_sus, deliv_sus, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < args.sustain:
            for st in steps_pipelined(100):
                deliv_sus += st.deliveries
            n_sus += 100
        wall_sus = time.perf_counter() - t0
        assert args.no_check or deliv_sus == deliv_expected * n_sus
        out["sustained"] = {"value": deliv_sus / wall_sus, "unit": "deliveries/s", "steps": n_sus,
                            "seconds": wall_sus, "ms_per_step": wall_sus * 1e3 / n_sus}
    if not args.no_general and not args.no_check:
        out["general_path"] = general_path(eng, wl, deliv_expected, max(20, min(args.steps, 100)))
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(eng, wl, sizes, args.cpu_budget, deliv_expected)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
