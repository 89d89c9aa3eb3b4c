"""ctypes binding of oracle/psoracle.c (TEST INFRASTRUCTURE ONLY).

Loaded by tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg.
The engine under go-libp2p-pubsub_amd/ never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libpsoracle.so")
NONE = 0xFFFFFFFF
OUT, IN, DEAD, FAILED, ORPHAN = range(5)

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        u32p = C.POINTER(C.c_uint32)
        u8p = C.POINTER(C.c_uint8)
        L.or_tree_new.restype = P
        L.or_tree_new.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64]
        L.or_tree_free.argtypes = [P]
        for f in ("or_tree_join", "or_tree_leave", "or_tree_drop"):
            getattr(L, f).argtypes = [P, C.c_uint32]
            getattr(L, f).restype = C.c_int
        L.or_tree_message.argtypes = [P, u8p]
        L.or_tree_message.restype = C.c_int
        L.or_tree_parents.argtypes = [P, u32p]
        L.or_tree_state.argtypes = [P, C.c_uint32]
        L.or_tree_state.restype = C.c_uint32
        L.or_disseminate.restype = C.c_int64
        L.or_disseminate.argtypes = [C.c_uint32, u32p, u32p, C.c_uint32, u8p, C.c_uint32,
                                     u32p, u8p, C.POINTER(C.c_uint64), C.c_uint32, C.c_int]
        L.or_levels_bits.restype = C.c_int64
        L.or_levels_bits.argtypes = [C.c_uint32, u32p, u32p, C.c_uint32, u8p, C.c_uint32, C.c_int]
        L.or_levels_new.restype = P
        L.or_levels_new.argtypes = [C.c_uint32, u32p, u32p, C.c_uint32, C.c_uint32]
        L.or_levels_run.restype = C.c_int64
        L.or_levels_run.argtypes = [P, u8p, C.c_int]
        L.or_levels_free.argtypes = [P]
        L.or_splitmix64.argtypes = [C.POINTER(C.c_uint64)]
        L.or_splitmix64.restype = C.c_uint64
        _lib = L
    return _lib


def _ptr(a, t):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


class Tree:
    """Restated subtree join / leave / drop for one topic."""

    def __init__(self, n_peers: int, root: int = 0, width: int = 2, max_width: int = 5,
                 seed: int = 1):
        self.n = n_peers
        self.root = root
        self._t = lib().or_tree_new(n_peers, root, width, max_width, seed)
        if not self._t:
            raise MemoryError("or_tree_new")

    def __del__(self):
        if getattr(self, "_t", None):
            lib().or_tree_free(self._t)
            self._t = None

    def join(self, peer: int) -> int:
        return lib().or_tree_join(self._t, peer)

    def join_all(self, peers) -> None:
        for p in peers:
            rc = self.join(int(p))
            if rc:
                raise RuntimeError(f"join({p}) -> {rc}")

    def leave(self, peer: int) -> int:
        return lib().or_tree_leave(self._t, peer)

    def drop(self, peer: int) -> int:
        return lib().or_tree_drop(self._t, peer)

    def message(self) -> np.ndarray:
        hop = np.empty(self.n, dtype=np.uint8)
        rc = lib().or_tree_message(self._t, _ptr(hop, C.c_uint8))
        if rc:
            raise RuntimeError(rc)
        return hop

    def parents(self) -> np.ndarray:
        out = np.empty(self.n, dtype=np.uint32)
        lib().or_tree_parents(self._t, _ptr(out, C.c_uint32))
        return out

    def state(self, peer: int) -> int:
        return lib().or_tree_state(self._t, peer)


def parents_to_csr(parent: np.ndarray):
    """Child lists (row_ptr, col) in peer space from a parent array; children in
    ascending peer order."""
    parent = np.asarray(parent, dtype=np.uint32)
    n = parent.shape[0]
    kids = np.nonzero(parent != NONE)[0].astype(np.uint32)
    par = parent[kids]
    order = np.lexsort((kids, par))
    kids, par = kids[order], par[order]
    counts = np.bincount(par, minlength=n).astype(np.uint32)
    row_ptr = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(counts, out=row_ptr[1:])
    return row_ptr, kids.astype(np.uint32)


def disseminate(row_ptr, col, root: int, live, n_msgs: int, want_hops: bool = True,
                hist_len: int = 256, threads: int = 1):
    """Round-synchronous per-message BFS (the hot path restated).  Returns
    (total deliveries, hop table [n_msgs, n] or None, hop histogram)."""
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint32)
    col = np.ascontiguousarray(col, dtype=np.uint32)
    n = row_ptr.shape[0] - 1
    live = np.ascontiguousarray(live, dtype=np.uint8)
    hops = np.full((n_msgs, n), 0xFF, dtype=np.uint8) if want_hops else None
    hist = np.zeros(hist_len, dtype=np.uint64)
    tot = lib().or_disseminate(n, _ptr(row_ptr, C.c_uint32), _ptr(col, C.c_uint32), root,
                               _ptr(live, C.c_uint8), n_msgs, None, _ptr(hops, C.c_uint8),
                               _ptr(hist, C.c_uint64), hist_len, threads)
    if tot < 0:
        raise RuntimeError(f"or_disseminate -> {tot}")
    return int(tot), hops, hist


def levels_bits(row_ptr, col, root: int, live, n_msgs: int, threads: int = 1) -> int:
    """The hot path as the GPU engine computes it (messages as bits, rounds
    level-synchronous, OpenMP over each level's nodes): total deliveries."""
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint32)
    col = np.ascontiguousarray(col, dtype=np.uint32)
    live = np.ascontiguousarray(live, dtype=np.uint8)
    tot = lib().or_levels_bits(row_ptr.shape[0] - 1, _ptr(row_ptr, C.c_uint32), _ptr(col, C.c_uint32), root,
                               _ptr(live, C.c_uint8), n_msgs, threads)
    if tot < 0:
        raise RuntimeError(f"or_levels_bits -> {tot}")
    return int(tot)


class Levels:
    """or_levels_new / or_levels_run: the bit-sliced restatement with the
    per-topology work (BFS numbering, rows allocated and touched) done once,
    so a timed pass is the level loop alone (bench.py cpu_baseline)."""

    def __init__(self, row_ptr, col, root: int, n_msgs: int):
        self._rp = np.ascontiguousarray(row_ptr, dtype=np.uint32)
        self._cl = np.ascontiguousarray(col, dtype=np.uint32)
        self._h = lib().or_levels_new(self._rp.shape[0] - 1, _ptr(self._rp, C.c_uint32),
                                      _ptr(self._cl, C.c_uint32), root, n_msgs)
        if not self._h:
            raise RuntimeError("or_levels_new failed")

    def run(self, live, threads: int = 1) -> int:
        lv = np.ascontiguousarray(live, dtype=np.uint8)
        tot = lib().or_levels_run(self._h, _ptr(lv, C.c_uint8), threads)
        if tot < 0:
            raise RuntimeError(f"or_levels_run -> {tot}")
        return int(tot)

    def close(self):
        if getattr(self, "_h", None):
            lib().or_levels_free(self._h)
            self._h = None

    def __del__(self):
        self.close()
