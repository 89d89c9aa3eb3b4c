"""The reference's wire codec through the C ABI (ps_msg_encode /
ps_msg_decode): writeMessage / readMessage, pubsub.go:122-134, over the
Message struct of pubsub.go:136-153.  Host-only; needs no GPU."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

from . import EngineError, MessageBuf, MessageC, load

DATA, JOIN, PART, UPDATE, STATE = range(5)  # MessageType, pubsub.go:138-144


@dataclass
class Message:
    type: int = DATA
    data: bytes = b""
    peers: list[str] = field(default_factory=list)
    tree_width: int = 0
    tree_max_width: int = 0
    num_peers: int = 0


def encode(m: Message) -> bytes:
    """json.NewEncoder(s).Encode(m): one '\\n'-terminated JSON line."""
    L = load()
    data = (C.c_uint8 * max(1, len(m.data))).from_buffer_copy(m.data or b"\0")
    pids = [p.encode() for p in m.peers]
    arr = (C.c_char_p * max(1, len(pids)))(*pids) if pids else (C.c_char_p * 1)()
    cm = MessageC(m.type, C.cast(data, C.POINTER(C.c_uint8)), len(m.data),
                  C.cast(arr, C.POINTER(C.c_char_p)), len(pids), m.tree_width, m.tree_max_width,
                  m.num_peers)
    n = C.c_size_t()
    L.ps_msg_encode(C.byref(cm), None, 0, C.byref(n))
    buf = C.create_string_buffer(n.value)
    rc = L.ps_msg_encode(C.byref(cm), buf, n.value, C.byref(n))
    if rc != 0:
        raise EngineError(rc, "ps_msg_encode")
    return buf.raw[:n.value]


def decode(line: bytes) -> tuple[Message, int]:
    """json.NewDecoder(r).Decode(m) of the first value; returns (message,
    bytes consumed)."""
    L = load()
    cap_d, cap_p = max(16, len(line)), max(16, len(line))
    dbuf = (C.c_uint8 * cap_d)()
    pbuf = C.create_string_buffer(cap_p)
    mb = MessageBuf()
    mb.data, mb.data_cap = C.cast(dbuf, C.POINTER(C.c_uint8)), cap_d
    mb.peers, mb.peers_cap = C.cast(pbuf, C.c_char_p), cap_p
    used = C.c_size_t()
    rc = L.ps_msg_decode(line, len(line), C.byref(mb), C.byref(used))
    if rc != 0:
        raise EngineError(rc, "ps_msg_decode")
    raw = pbuf.raw[:mb.peers_len]
    peers = [x.decode() for x in raw.split(b"\0")[:-1]] if mb.n_peers else []
    return Message(mb.type, bytes(dbuf[:mb.data_len]), peers, mb.tree_width, mb.tree_max_width,
                   mb.num_peers), used.value
