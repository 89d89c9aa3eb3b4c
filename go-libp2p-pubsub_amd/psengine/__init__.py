"""ctypes binding of libpsengine.so (include/psengine.h).

This is plumbing for tests and bench.py: every call goes straight into the
C ABI, whose hot path runs only as HIP kernels on the GPU.  There is no CPU
fallback: if the library or a GPU is missing, construction fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _build

NONE = 0xFFFFFFFF
HOP_NONE = 0xFF
MAX_ROUNDS = 256

PS_OK = 0
ERRORS = {
    -1: "PS_E_INVAL", -2: "PS_E_NOMEM", -3: "PS_E_STATE", -4: "PS_E_NOPARENT",
    -5: "PS_E_UNREACHABLE", -6: "PS_E_DEVICE", -7: "PS_E_RANGE", -8: "PS_E_NOTREADY",
}
PART_PEER = 0
PART_SUBTREE = 1
F_RECORD_HOPS = 0x1
F_TIME_KERNELS = 0x2
F_NO_LAZY_SEEN = 0x4
F_COMPACT = 0x8
MODE_COMPACT, MODE_LEVEL_PULL, MODE_FLOOD = 0, 2, 3
# ps_stats.expand_mode -> the kernel that ran the window's rounds
# ps_stats.round_kernel: the launch kind that wrote each round
K_NONE, K_FLOOD, K_PULL, K_PAIR, K_PAIR2, K_EXPAND, K_CHAIN, K_CHAIN2 = 0, 1, 2, 3, 4, 5, 6, 7
ROUND_KERNEL = {K_FLOOD: "k_flood", K_PULL: "k_pull", K_PAIR: "k_pull_pair", K_PAIR2: "k_pull_pair",
                K_EXPAND: "k_expand", K_CHAIN: "k_pull_chain", K_CHAIN2: "k_pull_chain"}
MODE_KERNEL = {MODE_COMPACT: "k_expand", MODE_LEVEL_PULL: "k_pull", MODE_FLOOD: "k_flood"}

# C prototypes exported by libpsengine.so: (name, restype, argtypes)
_P = C.c_void_p
_u32 = C.c_uint32
_u32p = C.POINTER(C.c_uint32)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)


class Config(C.Structure):
    _fields_ = [("n_peers", C.c_uint32), ("n_topics", C.c_uint32), ("tree_width", C.c_uint32),
                ("tree_max_width", C.c_uint32), ("msg_window", C.c_uint32), ("device", C.c_int32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32), ("seed", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [("deliveries", C.c_uint64), ("duplicates", C.c_uint64),
                ("frontier_entries", C.c_uint64), ("child_visits", C.c_uint64),
                ("edge_words", C.c_uint64), ("expand_bytes", C.c_uint64),
                ("windows", C.c_uint64), ("rounds", C.c_uint64), ("expand_launches", C.c_uint64),
                ("run_ms", C.c_double), ("expand_ms", C.c_double), ("host_ms", C.c_double),
                ("expand_mode", C.c_uint32), ("flood_rounds", C.c_uint32),
                ("deliveries_per_round", C.c_uint64 * MAX_ROUNDS),
                ("expand_ms_per_round", C.c_float * MAX_ROUNDS),
                ("frontier_per_round", C.c_uint32 * MAX_ROUNDS),
                ("expand_bytes_per_round", C.c_uint64 * MAX_ROUNDS),
                ("round_kernel", C.c_uint8 * MAX_ROUNDS),
                ("plan_max_rounds", C.c_uint32), ("prefix_rounds", C.c_uint32),
                ("overlapped", C.c_uint32), ("xchg_path", C.c_uint32),
                ("xchg_rounds", C.c_uint64), ("xchg_bytes", C.c_uint64),
                ("level_aligned", C.c_uint32), ("reserved2", C.c_uint32)]

    PER_ROUND = ("deliveries_per_round", "expand_ms_per_round", "frontier_per_round", "expand_bytes_per_round",
                 "round_kernel")

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in self.PER_ROUND}
        n = int(self.rounds) + 1 if self.windows == 1 else MAX_ROUNDS
        for k in self.PER_ROUND:
            per = list(getattr(self, k))[:min(n, MAX_ROUNDS)]
            while per and per[-1] == 0:
                per.pop()
            d[k] = per
        return d


class DistConfig(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("partition", C.c_uint32),
                ("split_depth", C.c_uint32), ("flags", C.c_uint32), ("reserved", C.c_uint32)]


DIST_F_COPY = 0x1  # loopback: copy the records into the receive buffer (the RCCL data path)
DIST_F_INPLACE = 0x2  # loopback: ghost-fed nodes read the owner's rows in place (no records)
XCHG_NONE, XCHG_ZERO_COPY, XCHG_COPY, XCHG_IN_PLACE = 0, 1, 2, 3  # ps_stats.xchg_path


class PlanOpts(C.Structure):
    """ps_plan_opts (include/psengine.h): the launch-plan knobs."""
    _fields_ = [("flood_top_bytes", C.c_uint64), ("overlap_min_bytes", C.c_uint64),
                ("launch_bytes", C.c_uint64), ("flood", C.c_uint32), ("chain_max", C.c_uint32),
                ("chain_max_groups", C.c_uint32), ("chain_tail", C.c_uint32), ("chain_words", C.c_uint32),
                ("flood_words", C.c_uint32), ("pad_words", C.c_uint32), ("overlap", C.c_uint32),
                ("overlap_min_rounds", C.c_uint32), ("xchg_overlap", C.c_int32), ("gpu_build", C.c_uint32),
                ("flood_spin_ticks", C.c_uint32), ("chain_nt", C.c_uint32), ("chain_waves", C.c_uint32),
                ("flood_min_rounds", C.c_uint32), ("align_groups", C.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class MessageC(C.Structure):
    """ps_message (include/psengine.h): pubsub.go:146-153 Message."""
    _fields_ = [("type", C.c_int32), ("data", _u8p), ("data_len", C.c_size_t),
                ("peers", C.POINTER(C.c_char_p)), ("n_peers", C.c_size_t),
                ("tree_width", C.c_int64), ("tree_max_width", C.c_int64), ("num_peers", C.c_int64)]


class MessageBuf(C.Structure):
    """ps_message_buf: caller-owned decode target."""
    _fields_ = [("type", C.c_int32), ("reserved", C.c_int32), ("data", _u8p),
                ("data_cap", C.c_size_t), ("data_len", C.c_size_t), ("peers", C.c_char_p),
                ("peers_cap", C.c_size_t), ("peers_len", C.c_size_t), ("n_peers", C.c_size_t),
                ("tree_width", C.c_int64), ("tree_max_width", C.c_int64), ("num_peers", C.c_int64)]


ABI_VERSION = 5  # PS_ABI_VERSION of include/psengine.h this binding mirrors

PROTOTYPES = [
    ("ps_version", C.c_char_p, []),
    ("ps_abi_version", C.c_uint32, []),
    ("ps_abi_check", C.c_int, [C.c_uint32, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t]),
    ("ps_create", C.c_int, [C.POINTER(Config), C.POINTER(_P)]),
    ("ps_destroy", None, [_P]),
    ("ps_last_error", C.c_char_p, [_P]),
    ("ps_topic_create", C.c_int, [_P, _u32, _u32, _u32, _u32]),
    ("ps_topic_close", C.c_int, [_P, _u32]),
    ("ps_topic_join", C.c_int, [_P, _u32, _u32p, C.c_size_t, _i32p]),
    ("ps_topic_leave", C.c_int, [_P, _u32, _u32p, C.c_size_t]),
    ("ps_topic_drop", C.c_int, [_P, _u32, _u32p, C.c_size_t]),
    ("ps_topic_set_tree", C.c_int, [_P, _u32, _u32, _u32p]),
    ("ps_topic_set_children", C.c_int, [_P, _u32, _u32, _u32p, _u32p]),
    ("ps_topic_get_parents", C.c_int, [_P, _u32, _u32p]),
    ("ps_topic_depth", C.c_int, [_P, _u32, _u32p, _u32p]),
    ("ps_set_live", C.c_int, [_P, _u8p]),
    ("ps_set_flags", C.c_int, [_P, _u32]),
    ("ps_plan_opts_default", C.c_int, [C.POINTER(PlanOpts)]),
    ("ps_get_plan_opts", C.c_int, [_P, C.POINTER(PlanOpts)]),
    ("ps_set_plan_opts", C.c_int, [_P, C.POINTER(PlanOpts)]),
    ("ps_publish", C.c_int, [_P, _u32p, C.c_size_t, _u32p]),
    ("ps_publish_at", C.c_int, [_P, _u32p, _u32p, C.c_size_t, _u32p]),
    ("ps_run", C.c_int, [_P, C.POINTER(Stats)]),
    ("ps_run_async", C.c_int, [_P]),
    ("ps_wait", C.c_int, [_P, C.POINTER(Stats)]),
    ("ps_read_hops", C.c_int, [_P, _u32, _u8p]),
    ("ps_read_delivered", C.c_int, [_P, _u32, _u8p]),
    ("ps_read_peer_messages", C.c_int, [_P, _u32, _u32, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("ps_seen_digest", C.c_int, [_P, _u64p]),
    ("ps_overlapped_windows", C.c_int, [_P, _u64p]),
    ("ps_msg_encode", C.c_int, [C.POINTER(MessageC), C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("ps_msg_decode", C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(MessageBuf), C.POINTER(C.c_size_t)]),
    ("ps_dist_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("ps_dist_init", C.c_int, [_P, C.POINTER(DistConfig), C.POINTER(C.c_uint8)]),
    ("ps_device_count", C.c_int, [_i32p]),
    ("ps_dist_ipc_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("ps_dist_init_ipc", C.c_int, [_P, C.POINTER(DistConfig), C.POINTER(C.c_uint8)]),
    ("ps_loopback_create", C.c_int, [C.c_int32, C.POINTER(_P)]),
    ("ps_loopback_destroy", None, [_P]),
    ("ps_dist_init_loopback", C.c_int, [_P, C.POINTER(DistConfig), _P]),
    ("ps_partition_owner", C.c_int, [_u32, _u32, _u32p, _u32, C.POINTER(DistConfig), _i32p]),
]

_lib = None


def lib_path() -> str:
    return _build.LIB


def load(build_if_missing: bool = False):
    """Loads libpsengine.so and binds every prototype (raises if absent)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_build.LIB):
            if not build_if_missing:
                raise FileNotFoundError(
                    f"{_build.LIB} missing: run __graft_entry__.build() (no CPU fallback exists)")
            _build.build()
        # (A/B tools: another build of the library, only under PSAMD_AB=1)
        ab = os.environ.get("PSENGINE_LIB_AB") if os.environ.get("PSAMD_AB") == "1" else None
        L = C.CDLL(ab or _build.LIB)
        for name, res, args in PROTOTYPES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        # the structs this module declares must match the library's layouts
        rc = L.ps_abi_check(ABI_VERSION, C.sizeof(Config), C.sizeof(Stats), C.sizeof(PlanOpts),
                            C.sizeof(DistConfig))
        if rc != 0:
            raise RuntimeError(f"libpsengine ABI mismatch: {L.ps_last_error(None).decode()}")
        _lib = L
    return _lib


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def _u32arr(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class Engine:
    """One engine = one GPU's worth of topics (NewTopicManager, pubsub.go:26-31)."""

    _pub_arr = None  # the last uint32 array published and its ctypes pointer
    _pub_ptr = None

    def __init__(self, n_peers: int, n_topics: int = 1, tree_width: int = 2,
                 tree_max_width: int = 5, msg_window: int = 65536, device: int = 0,
                 record_hops: bool = False, time_kernels: bool = False, seed: int = 1,
                 flags: int = 0, plan: dict | None = None):
        """plan: launch-plan options to set right away (ps_set_plan_opts)."""
        L = load()
        self.n_peers = n_peers
        self.n_topics = n_topics
        self.seed = seed
        f = flags | (F_RECORD_HOPS if record_hops else 0) | (F_TIME_KERNELS if time_kernels else 0)
        cfg = Config(n_peers, n_topics, tree_width, tree_max_width, msg_window, device, f, 0, seed)
        self.flags = f
        h = _P()
        rc = L.ps_create(C.byref(cfg), C.byref(h))
        if rc != PS_OK:
            raise EngineError(rc, "ps_create failed (is a GPU visible?)")
        self._h = h
        self._L = L
        if plan:
            self.set_plan(**plan)

    def close(self):
        if getattr(self, "_h", None):
            self._L.ps_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int) -> int:
        if rc < 0:
            raise EngineError(rc, self._L.ps_last_error(self._h).decode())
        return rc

    @staticmethod
    def topic_seed(seed: int, topic: int) -> int:
        """Redirect tie-break seed of a topic created with ps_topic_create."""
        return (seed ^ (0xA5A5A5A5 * (topic + 1))) & ((1 << 64) - 1)

    # topics
    def topic_create(self, topic: int, root: int, tree_width: int = 0, tree_max_width: int = 0):
        self._check(self._L.ps_topic_create(self._h, topic, root, tree_width, tree_max_width))

    def topic_close(self, topic: int):
        self._check(self._L.ps_topic_close(self._h, topic))

    def join(self, topic: int, peers, check: bool = True) -> np.ndarray:
        p = _u32arr(peers)
        st = np.zeros(p.shape[0], dtype=np.int32)
        rc = self._L.ps_topic_join(self._h, topic, _p(p, C.c_uint32), p.shape[0],
                                   _p(st, C.c_int32))
        if check:
            self._check(rc)
        return st

    def leave(self, topic: int, peers):
        p = _u32arr(peers)
        self._check(self._L.ps_topic_leave(self._h, topic, _p(p, C.c_uint32), p.shape[0]))

    def drop(self, topic: int, peers):
        p = _u32arr(peers)
        self._check(self._L.ps_topic_drop(self._h, topic, _p(p, C.c_uint32), p.shape[0]))

    def set_tree(self, topic: int, root: int, parent):
        par = _u32arr(parent)
        assert par.shape[0] == self.n_peers
        self._check(self._L.ps_topic_set_tree(self._h, topic, root, _p(par, C.c_uint32)))

    def set_children(self, topic: int, root: int, row_ptr, col):
        rp, cl = _u32arr(row_ptr), _u32arr(col)
        assert rp.shape[0] == self.n_peers + 1
        if cl.shape[0] == 0:
            cl = np.zeros(1, dtype=np.uint32)
        self._check(self._L.ps_topic_set_children(self._h, topic, root, _p(rp, C.c_uint32),
                                                  _p(cl, C.c_uint32)))

    def parents(self, topic: int) -> np.ndarray:
        out = np.empty(self.n_peers, dtype=np.uint32)
        self._check(self._L.ps_topic_get_parents(self._h, topic, _p(out, C.c_uint32)))
        return out

    def depth(self, topic: int) -> tuple[int, int]:
        d, n = C.c_uint32(), C.c_uint32()
        self._check(self._L.ps_topic_depth(self._h, topic, C.byref(d), C.byref(n)))
        return d.value, n.value

    def set_flags(self, flags: int):
        """Replaces the PS_F_* flags for the next runs (ps_set_flags)."""
        self._check(self._L.ps_set_flags(self._h, flags))
        self.flags = flags

    def plan_opts(self) -> dict:
        """The effective launch-plan options (ps_get_plan_opts)."""
        o = PlanOpts()
        self._check(self._L.ps_get_plan_opts(self._h, C.byref(o)))
        return o.as_dict()

    def set_plan(self, **kw) -> dict:
        """Changes launch-plan options by name (ps_set_plan_opts), e.g.
        set_plan(flood=0, chain_max=2); returns the effective options."""
        o = PlanOpts()
        self._check(self._L.ps_get_plan_opts(self._h, C.byref(o)))
        for k, v in kw.items():
            if k not in dict(PlanOpts._fields_):
                raise KeyError(f"no plan option {k!r}")
            setattr(o, k, int(v))
        self._check(self._L.ps_set_plan_opts(self._h, C.byref(o)))
        return self.plan_opts()

    def set_time_kernels(self, on: bool):
        self.set_flags((self.flags & ~F_TIME_KERNELS) | (F_TIME_KERNELS if on else 0))

    def set_live(self, live):
        lv = np.ascontiguousarray(live, dtype=np.uint8)
        assert lv.shape[0] == self.n_peers
        self._check(self._L.ps_set_live(self._h, _p(lv, C.c_uint8)))

    # hot path
    def publish(self, topics, start_rounds=None) -> int:
        # (the same uint32 array again, the usual batch loop: its pointer is
        # reused -- ndarray.ctypes costs microseconds per call)
        if topics is self._pub_arr:
            t, tp = topics, self._pub_ptr
        else:
            t = _u32arr(topics)
            tp = _p(t, C.c_uint32)
            if t is topics:
                self._pub_arr, self._pub_ptr = t, tp
        first = C.c_uint32()
        if start_rounds is None:
            self._check(self._L.ps_publish(self._h, tp, t.shape[0], C.byref(first)))
        else:
            s = _u32arr(start_rounds)
            assert s.shape == t.shape
            self._check(self._L.ps_publish_at(self._h, tp, _p(s, C.c_uint32),
                                              t.shape[0], C.byref(first)))
        return first.value

    def run(self) -> Stats:
        st = Stats()
        self._check(self._L.ps_run(self._h, C.byref(st)))
        return st

    def run_async(self):
        """Enqueues the run (ps_run_async); ps_wait / wait() completes it."""
        self._check(self._L.ps_run_async(self._h))

    def wait(self) -> Stats:
        st = Stats()
        self._check(self._L.ps_wait(self._h, C.byref(st)))
        return st

    def hops(self, msg: int) -> np.ndarray:
        out = np.empty(self.n_peers, dtype=np.uint8)
        self._check(self._L.ps_read_hops(self._h, msg, _p(out, C.c_uint8)))
        return out

    def delivered(self, msg: int) -> np.ndarray:
        out = np.empty(self.n_peers, dtype=np.uint8)
        self._check(self._L.ps_read_delivered(self._h, msg, _p(out, C.c_uint8)))
        return out

    def peer_messages(self, topic: int, peer: int) -> np.ndarray:
        """Message ids `peer`'s client.Messages() yields for `topic` from the
        last window, in arrival order (ps_read_peer_messages)."""
        n = C.c_size_t()
        cap = 1024
        while True:
            out = np.empty(cap, dtype=np.uint32)
            rc = self._L.ps_read_peer_messages(self._h, topic, peer, _p(out, C.c_uint32), cap, C.byref(n))
            if rc == -7 and n.value > cap:
                cap = n.value
                continue
            self._check(rc)
            return out[:n.value].copy()

    def seen_digest(self) -> int:
        d = C.c_uint64()
        self._check(self._L.ps_seen_digest(self._h, C.byref(d)))
        return d.value

    def overlapped_windows(self) -> int:
        """Pipelined windows whose prefix ran beside the previous window."""
        d = C.c_uint64()
        self._check(self._L.ps_overlapped_windows(self._h, C.byref(d)))
        return d.value

    # multi-GPU
    def dist_init(self, rank: int, world: int, unique_id: bytes, partition: int = PART_PEER,
                  split_depth: int = 0):
        """RCCL-backed sharding: this engine owns a hash partition of every topic."""
        dc = DistConfig(rank, world, partition, split_depth)
        uid = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._check(self._L.ps_dist_init(self._h, C.byref(dc), uid))

    def dist_init_ipc(self, rank: int, world: int, group_id: bytes, partition: int = PART_PEER,
                      split_depth: int = 0, copy: bool = False, inplace: bool = False):
        """Process-shared sharding (ps_dist_init_ipc): one process per rank on
        one node, device memory mapped across processes (several ranks may
        share a GPU); group_id from ipc_group_id() on one rank.  copy / inplace
        as for dist_init_loopback."""
        flags = (DIST_F_COPY if copy else 0) | (DIST_F_INPLACE if inplace else 0)
        dc = DistConfig(rank, world, partition, split_depth, flags, 0)
        gid = (C.c_uint8 * 128).from_buffer_copy(group_id)
        self._check(self._L.ps_dist_init_ipc(self._h, C.byref(dc), gid))

    def dist_init_loopback(self, group: "Loopback", rank: int, partition: int = PART_PEER,
                           split_depth: int = 0, copy: bool = False, inplace: bool = False):
        """copy: the records go through the receive buffer (PS_DIST_F_COPY), the
        RCCL transport's data path, instead of being read in place.  inplace:
        no records below the roots -- ghost-fed nodes read their parents' rows
        in the owner's row set (PS_DIST_F_INPLACE)."""
        flags = (DIST_F_COPY if copy else 0) | (DIST_F_INPLACE if inplace else 0)
        dc = DistConfig(rank, group.world, partition, split_depth, flags, 0)
        self._check(self._L.ps_dist_init_loopback(self._h, C.byref(dc), group._h))


def unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    rc = load().ps_dist_unique_id(buf)
    if rc != PS_OK:
        raise EngineError(rc, "ps_dist_unique_id")
    return bytes(buf)


def device_count() -> int:
    """GPUs visible to this process, through the engine's own HIP runtime."""
    n = C.c_int32()
    load().ps_device_count(C.byref(n))
    return int(n.value)


def ipc_group_id() -> bytes:
    """A fresh group id for ps_dist_init_ipc (host only; ship it to every rank)."""
    buf = (C.c_uint8 * 128)()
    rc = load().ps_dist_ipc_id(buf)
    if rc != PS_OK:
        raise EngineError(rc, "ps_dist_ipc_id")
    return bytes(buf)


class Loopback:
    """In-process transport: `world` engines (one thread each) exchange
    frontier regions through device copies -- the multi-GPU path on one GPU."""

    def __init__(self, world: int):
        self.world = world
        h = _P()
        rc = load().ps_loopback_create(world, C.byref(h))
        if rc != PS_OK:
            raise EngineError(rc, "ps_loopback_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            load().ps_loopback_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def partition_owner(parent, root: int, topic: int, world: int, partition: int = PART_PEER,
                    split_depth: int = 0) -> np.ndarray:
    """Host-only: owner rank of every peer of a tree (-1 outside the tree)."""
    par = _u32arr(parent)
    out = np.empty(par.shape[0], dtype=np.int32)
    dc = DistConfig(0, world, partition, split_depth)
    rc = load().ps_partition_owner(par.shape[0], root, _p(par, C.c_uint32), topic, C.byref(dc),
                                   _p(out, C.c_int32))
    if rc != PS_OK:
        raise EngineError(rc, "ps_partition_owner")
    return out


def default_plan_opts() -> dict:
    """ps_plan_opts_default: the options every engine starts from."""
    o = PlanOpts()
    rc = load().ps_plan_opts_default(C.byref(o))
    if rc != PS_OK:
        raise EngineError(rc, "ps_plan_opts_default")
    return o.as_dict()


def version() -> str:
    return load().ps_version().decode()
