"""ctypes binding of the host-only planner probe (include/psengine_plan.h):
one rank's node space and one window's launch plans, built by the engine's
own C++ planners without touching a device, for CPU tests."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import DistConfig, EngineError, PART_PEER, PlanOpts, _P, _p, _u32arr, load

INFO, NODES, PARENT, GHOST_REF, TOPIC, LAYOUT, ROUND_KIND, PULL, PAIR, XCHG, SEGS, SHIP, PACK, CHAIN = range(14)
CHAIN_FIELDS = ("node_begin", "node_end", "topic", "W", "row0", "w0", "S", "levels", "r0", "group")
CHAIN_LEVELS = 6  # kChainLevels
CHUNK_FIELDS = ("node_begin", "node_end", "topic", "W", "row0", "e_lo", "e_hi", "gin", "gout", "group",
                "p_lo", "p_hi", "c_lo")
PROTOTYPES = [
    ("ps_plan_create", C.c_int, [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                 C.POINTER(DistConfig), C.POINTER(_P)]),
    ("ps_plan_destroy", None, [_P]),
    ("ps_plan_set_msg_window", C.c_int, [_P, C.c_uint32]),
    ("ps_plan_window", C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_size_t, C.c_uint32]),
    ("ps_plan_get", C.c_int, [_P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.c_size_t,
                              C.POINTER(C.c_size_t)]),
]
_bound = False


def lib():
    global _bound
    L = load()
    if not _bound:
        for name, res, args in PROTOTYPES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _bound = True
    return L


class Plan:
    """One rank's plans for trees `parents` (n_topics x n_peers, NONE =
    absent) rooted at `roots`."""

    def __init__(self, parents, roots, world: int = 1, rank: int = 0, partition: int = PART_PEER,
                 split_depth: int = 0, plan: dict | None = None):
        par = np.ascontiguousarray(np.asarray(parents, dtype=np.uint32).reshape(len(roots), -1))
        self.n_topics, self.n_peers = par.shape
        rt = _u32arr(roots)
        dc = DistConfig(rank, world, partition, split_depth)
        h = _P()
        rc = lib().ps_plan_create(self.n_peers, self.n_topics, _p(rt, C.c_uint32), _p(par, C.c_uint32),
                                  C.byref(dc), C.byref(h))
        if rc != 0:
            raise EngineError(rc, "ps_plan_create")
        self._h = h
        self.world, self.rank = world, rank
        if plan:
            self.set_plan(**plan)

    def close(self):
        if getattr(self, "_h", None):
            lib().ps_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_plan(self, **kw) -> dict:
        """Launch-plan options by name (ps_set_plan_opts on the probe)."""
        L = lib()
        o = PlanOpts()
        L.ps_get_plan_opts(self._h, C.byref(o))
        for k, v in kw.items():
            if k not in dict(PlanOpts._fields_):
                raise KeyError(f"no plan option {k!r}")
            setattr(o, k, int(v))
        rc = L.ps_set_plan_opts(self._h, C.byref(o))
        if rc != 0:
            raise EngineError(rc, "ps_set_plan_opts")
        L.ps_get_plan_opts(self._h, C.byref(o))
        return o.as_dict()

    def set_msg_window(self, n: int):
        rc = lib().ps_plan_set_msg_window(self._h, n)
        if rc != 0:
            raise EngineError(rc, "ps_plan_set_msg_window")

    def window(self, topics, starts=None, flags: int = 0):
        t = _u32arr(topics)
        s = None if starts is None else _u32arr(starts)
        rc = lib().ps_plan_window(self._h, _p(t, C.c_uint32), None if s is None else _p(s, C.c_uint32),
                                  t.shape[0], flags)
        if rc != 0:
            raise EngineError(rc, "ps_plan_window")

    def get(self, what: int, index: int = 0) -> np.ndarray:
        n = C.c_size_t()
        lib().ps_plan_get(self._h, what, index, None, 0, C.byref(n))
        out = np.zeros(max(1, n.value), dtype=np.uint64)
        rc = lib().ps_plan_get(self._h, what, index, out.ctypes.data_as(C.POINTER(C.c_uint64)), out.shape[0],
                               C.byref(n))
        if rc != 0:
            raise EngineError(rc, f"ps_plan_get({what}, {index})")
        return out[:n.value]

    def info(self) -> dict:
        v = self.get(INFO)
        keys = ("rounds", "nodes", "pull_chunks", "pair_chunks", "world", "rank", "send_half", "recv_words",
                "segs", "level", "ship", "aligned")
        return {k: int(x) for k, x in zip(keys, v)}

    def chunks(self, what: int, q: int):
        """(first, split, end, [chunk dicts]) of round q's pull (or pair) launch."""
        v = self.get(what, q)
        lo, split, hi = (int(x) for x in v[:3])
        body = v[3:].reshape(-1, len(CHUNK_FIELDS))
        return lo, split, hi, [dict(zip(CHUNK_FIELDS, (int(x) for x in row))) for row in body]

    def topic(self, t: int) -> dict:
        v = self.get(TOPIC, t)
        depth = int(v[2])
        return {"nbase": int(v[0]), "n_nodes": int(v[1]), "depth": depth, "root_local": bool(v[3]),
                "level_off": v[4:4 + depth + 2].astype(np.int64),
                "level_local": v[4 + depth + 2:4 + 2 * depth + 3].astype(np.int64)}

    def layout(self, t: int) -> dict:
        v = self.get(LAYOUT, t)
        ng = int(v[3])
        na = int(v[4 + 3 * ng])
        a0 = 5 + 3 * ng
        return {"W": int(v[0]), "wbase": int(v[1]), "flags": int(v[2]),
                "groups": [tuple(int(x) for x in v[4 + 3 * i:7 + 3 * i]) for i in range(ng)],
                "aligned_groups": [tuple(int(x) for x in v[a0 + 3 * i:a0 + 3 + 3 * i]) for i in range(na)]}

    def xchg(self, q: int) -> dict:
        v = self.get(XCHG, q)
        if v.shape[0] <= 1:
            return {"any": bool(v[0]) if v.shape[0] else False}
        r = v[1:].reshape(-1, 4).astype(np.int64)
        return {"any": bool(v[0]), "s_off": r[:, 0], "s_len": r[:, 1], "r_off": r[:, 2], "r_len": r[:, 3]}

    def segs(self):
        w = self.world
        v = self.get(SEGS).reshape(-1, 2 + 2 * w).astype(np.int64)
        return [{"topic": int(x[0]), "rw": int(x[1]), "rbase": x[2:2 + w], "sbase": x[2 + w:]} for x in v]

    def ship(self) -> np.ndarray:
        return self.get(SHIP).reshape(-1, 2).astype(np.int64)

    def pack(self, q: int):
        v = self.get(PACK, q).reshape(-1, 6).astype(np.int64)
        return [dict(zip(("e0", "e1", "gseg", "W", "row", "unit0"), (int(x) for x in r))) for r in v]

    def chain(self, q: int):
        """(rounds, [chunk dicts]) of the chain launch starting at round q (rounds 0: none)."""
        v = self.get(CHAIN, q)
        n = int(v[0])
        if n == 0:
            return 0, []
        body = v[1:].reshape(-1, len(CHAIN_FIELDS) + CHAIN_LEVELS + 1)
        out = []
        for row in body:
            c = dict(zip(CHAIN_FIELDS, (int(x) for x in row[:len(CHAIN_FIELDS)])))
            c["first"] = [int(x) for x in row[len(CHAIN_FIELDS):]]
            out.append(c)
        return n, out
