#!/usr/bin/env python3
"""Generates the committed golden fixtures of tests/golden/ (data only).

Every expected output here comes from oracle/event_sim.py -- the independent,
asynchronous, pure-Python restatement of go-libp2p-pubsub v0 -- never from the
engine under test.  The reference itself (Go) cannot be built or run here
(SURVEY.md F8), and ships no golden vectors; the scenario fixtures restate its
four tests (pubsub_test.go:133-325) and carry their assertions ("every
non-skipped subscriber receives the exact payload") next to the expected
deliveries, so tests check both the restatement and the engine against them.

    python tests/golden/make_golden.py      # rewrites the *.json fixtures
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import event_sim as ES  # noqa: E402

NONE = ES.NONE


def hops_of(got, n, mi):
    h = [255] * n
    for peer, lst in enumerate(got):
        for m, hop in lst:
            if m == mi:
                h[peer] = hop
    return h


def hexrow(h):
    return bytes(h).hex()


# ---------------------------------------------------------------- cfg1 -----
def make_cfg1():
    """BASELINE config 1: 16 peers, topic "foobar", W=2/MaxW=5, peers 1..15
    subscribe in order (pubsub_test.go:65-83), 1000 paced publishes of
    "message number %d" (pubsub_test.go:101-131)."""
    n, seed = 16, 1
    t = ES.build_join_tree(n, 0, 2, 5, seed)
    parent = t.parents()
    payloads = [f"message number {i}".encode() for i in range(1000)]
    got = t.publish(payloads, random.Random(seed), pace=100.0)
    # per-peer delivery order must be publish order (FIFO path, client.go:103-131)
    for peer in range(1, n):
        assert [m for m, _ in got[peer]] == list(range(1000))
    hop = hops_of(got, n, 0)
    for mi in range(1, 1000, 97):
        assert hops_of(got, n, mi) == hop
    return {
        "what": "BASELINE cfg1: 16 peers, 1 topic, W=2/MaxW=5, join order 1..15, 1000 paced publishes",
        "ref": "pubsub_test.go:65-131, subtree.go:100-354, client.go:65-132",
        "n_peers": n, "root": 0, "width": 2, "max_width": 5, "seed": seed,
        "join_order": list(range(1, n)),
        "parent": parent,
        "n_msgs": 1000,
        "payload_format": "message number %d",
        "hops_per_message": hexrow(hop),
        "deliveries": sum(len(g) for g in got),
    }


# ------------------------------------------------------- multi-topic 1k ----
def make_multitopic():
    n, n_topics, seed = 1000, 4, 3
    rng = random.Random(seed)
    topics = []
    for k in range(n_topics):
        w, mw = [(2, 5), (8, 20), (3, 6), (1, 3)][k]
        order = [p for p in range(n_topics, n) if rng.random() < 1.0 / (k + 1)]
        t = ES.build_join_tree(n, k, w, mw, seed * 100 + k, order)
        got = t.publish([b"x"], random.Random(k))
        topics.append({"root": k, "width": w, "max_width": mw, "seed": seed * 100 + k,
                       "join_order": order, "parent": t.parents(),
                       "hops": hexrow(hops_of(got, n, 0))})
    return {"what": "1k peers, 4 topics with their own roots/widths, join-built trees, hop per peer",
            "ref": "pubsub.go:54-97 (one tree per topic), subtree.go:100-354",
            "n_peers": n, "topics": topics}


# ----------------------------------------------------- reference tests ----
SCENARIOS = [
    {"name": "TestBasicPubsub", "ref": "pubsub_test.go:133-155", "hosts": 4,
     "steps": [["publish", list(range(10)), []]]},
    {"name": "TestNodesDropping", "ref": "pubsub_test.go:158-202", "hosts": 4,
     "steps": [["publish", [0], []], ["drop", 1], ["publish", [1], [0, 2]],
               ["publish", list(range(100, 110)), [0]]]},
    {"name": "TestLowerNodesDropping", "ref": "pubsub_test.go:231-279", "hosts": 8,
     "steps": [["publish", [0], []], ["drop", 3], ["publish", [1], [2, 5, 6]],
               ["publish", list(range(100, 110)), [2]]]},
    {"name": "TestNodesDroppingGracefully", "ref": "pubsub_test.go:281-325", "hosts": 4,
     "steps": [["publish", [0], []], ["leave", 1], ["publish", [1], [0]],
               ["publish", list(range(100, 110)), [0]]]},
]


def run_scenario(sc, seed):
    """Restated run of one reference test; subscriber i is host i+1 (subchs)."""
    n = sc["hosts"]
    t = ES.build_join_tree(n, 0, 2, 5, seed)  # initPubsub: hosts[1..] subscribe in order
    trace = {"seed": seed, "parent": t.parents(), "publishes": []}
    for step in sc["steps"]:
        if step[0] == "publish":
            mids, skip = step[1], set(step[2])
            got = t.publish([f"message number {m}".encode() for m in mids], random.Random(seed))
            for k, mid in enumerate(mids):
                hop = hops_of(got, n, k)
                # the reference test's assertion (checkSystem, pubsub_test.go:113-127)
                for i in range(n - 1):
                    if i not in skip:
                        assert hop[i + 1] != 255, (sc["name"], seed, mid, i)
                trace["publishes"].append({"mid": mid, "hops": hexrow(hop)})
        elif step[0] == "drop":
            t.drop(step[1])
        elif step[0] == "leave":
            t.leave(step[1])
    return trace


def make_scenarios():
    out = []
    for sc in SCENARIOS:
        runs = [run_scenario(sc, seed) for seed in range(32)]
        out.append(dict(sc, runs=runs))
    return {"what": "the reference's four tests restated deterministically; for each tie-break "
                    "seed: tree after initPubsub and the hop of every publish at every host",
            "payload_format": "message number %d", "subscriber_i_is_host": "i+1",
            "width": 2, "max_width": 5, "scenarios": out}


# ------------------------------------------------------------- churn ------
def make_churn():
    n, W, MW, seed = 300, 2, 5, 17
    rng = random.Random(seed)
    t = ES.Topic(n, 0, W, MW, seed)
    ops = []
    for _ in range(400):
        x = rng.random()
        members = [p for p in range(1, n) if p in t.subs and t._receives(p)]
        if x < 0.5:
            p = rng.randrange(1, n)
            try:
                t.subscribe(p)
                ok = True
            except (ValueError, ConnectionError, RuntimeError):
                ok = False
            ops.append({"op": "join", "peer": p, "ok": ok})
        elif x < 0.62 and members:
            p = rng.choice(members)
            t.leave(p)
            ops.append({"op": "leave", "peer": p})
        elif x < 0.7 and members:
            p = rng.choice(members)
            t.drop(p)
            ops.append({"op": "drop", "peer": p})
        else:
            got = t.publish([b"m"], random.Random(len(ops)))
            ops.append({"op": "publish", "hops": hexrow(hops_of(got, n, 0))})
        if ops[-1]["op"] == "publish":
            ops[-1]["parent"] = hexrow_u32(t.parents())
    return {"what": "random join/leave/drop/publish sequence: hops per publish, attached "
                    "parents at every publish", "ref": "subtree.go:46-375, client.go:30-132",
            "n_peers": n, "root": 0, "width": W, "max_width": MW, "seed": seed, "ops": ops}


def hexrow_u32(a):
    return b"".join(int(x).to_bytes(4, "little") for x in a).hex()


def main():
    for name, fn in [("cfg1", make_cfg1), ("multitopic_1k", make_multitopic),
                     ("scenarios", make_scenarios), ("churn_300", make_churn)]:
        path = os.path.join(HERE, f"{name}.json")
        with open(path, "w") as f:
            json.dump(fn(), f, separators=(",", ":"))
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
