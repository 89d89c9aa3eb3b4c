#!/usr/bin/env python3
"""A/B of launch-plan options (ps_set_plan_opts) on one engine.

    python tools/ab_opts.py --workload cfg2 --variants '[{}, {"overlap_min_bytes": 0}]' [--reps 6 --steps 200]

Variants alternate (A B A B ...) on the same engine and topology; each rep
runs `steps` pipelined steps (ps_run_async / ps_wait, as bench.py times them)
and checks the deliveries.  Prints one JSON line: per variant the ms/step of
every rep, the median, and the effective plan of its last window."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

import psengine as PE  # noqa: E402
from psengine import workloads as WL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--variants", default='[{}]')
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--sync", action="store_true")
    ap.add_argument("--staggered", type=int, default=0,
                    help="start rounds uniform over 0..N (bench.py's general path: paced publishing)")
    args = ap.parse_args()
    variants = json.loads(args.variants)
    wl = WL.CONFIGS[args.workload]()
    # a variant's "env" (engine switches read at creation, PSAMD_AB=1 set
    # for it) gets an engine of its own; the others share one
    engines = {}

    def engine_for(v):
        env = v.get("env", {})
        k = json.dumps(env, sort_keys=True)
        if k not in engines:
            old = {n: os.environ.get(n) for n in env}
            os.environ.update({n: str(x) for n, x in env.items()})
            if env:
                os.environ["PSAMD_AB"] = "1"
            e = PE.Engine(wl.n_peers, len(wl.topics), seed=wl.seed)
            for n, x in old.items():
                if x is None:
                    os.environ.pop(n, None)
                else:
                    os.environ[n] = x
            os.environ.pop("PSAMD_AB", None)
            engines[k] = (e, WL.build_engine_topics(e, wl))
        return engines[k]

    eng, sizes = engine_for({})
    expect = wl.expected_deliveries(sizes)
    starts = None
    if args.staggered:
        import numpy as np

        starts = (WL.stream(wl.seed ^ 0x57A6, np.arange(wl.n_msgs)) % np.uint64(args.staggered + 1)).astype(np.uint32)
    base = eng.plan_opts()
    res = [[] for _ in variants]
    last = [None] * len(variants)
    for rep in range(args.reps):
        for i, v in enumerate(variants):
            eng, _ = engine_for(v)
            eng.set_plan(**{**base, **{k: x for k, x in v.items() if k != "env"}})
            for _ in range(3):  # warm: plans rebuilt, uploads done
                eng.publish(wl.msg_topics, starts)
                assert eng.run().deliveries == expect
            t0 = time.perf_counter()
            tot = 0
            if args.sync:
                for _ in range(args.steps):
                    eng.publish(wl.msg_topics, starts)
                    st = eng.run()
                    tot += st.deliveries
            else:
                for k in range(args.steps):
                    eng.publish(wl.msg_topics, starts)
                    eng.run_async()
                    if k:
                        tot += eng.wait().deliveries
                st = eng.wait()
                tot += st.deliveries
            wall = time.perf_counter() - t0
            assert tot == expect * args.steps, (tot, expect)
            res[i].append(wall * 1e3 / args.steps)
            last[i] = {"plan_max_rounds": st.plan_max_rounds, "prefix_rounds": st.prefix_rounds,
                       "flood_rounds": st.flood_rounds, "rounds": st.rounds, "overlapped": st.overlapped}
        print(f"[ab] rep {rep}: " + "  ".join(f"{r[-1]:.4f}" for r in res), file=sys.stderr, flush=True)
    out = {"workload": args.workload, "steps": args.steps, "sync": args.sync,
           "variants": [{"opts": v, "ms_per_step": [round(x, 4) for x in r], "median": round(statistics.median(r), 4),
                         "last_window": l} for v, r, l in zip(variants, res, last)]}
    print(json.dumps(out))
    for e, _ in engines.values():
        e.close()


if __name__ == "__main__":
    main()
