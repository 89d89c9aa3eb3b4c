"""The wire codec through the C ABI (ps_msg_encode / ps_msg_decode), host
only: writeMessage / readMessage of pubsub.go:122-134 over the Message struct
of pubsub.go:136-153.

Pinned by tests/golden/wire_vectors.json (make_wire_vectors.py restates
encoding/json's rules independently of the C code; no Go toolchain here).
"""
import json
import os

import pytest

import psengine as PE
from psengine import wire as W

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "wire_vectors.json")


def vectors():
    with open(GOLDEN) as f:
        return json.load(f)


def to_msg(d: dict) -> W.Message:
    # peers in the fixtures are hex: a Go string may hold any bytes
    return W.Message(d["type"], bytes.fromhex(d.get("data", "")),
                     [bytes.fromhex(p).decode("utf-8", "surrogateescape") for p in d.get("peers", [])],
                     d.get("tree_width", 0), d.get("tree_max_width", 0), d.get("num_peers", 0))


def encode_raw(m: dict) -> bytes:
    """Encode with peers passed as raw bytes (invalid UTF-8 included)."""
    import ctypes as C
    L = PE.load()
    data = bytes.fromhex(m.get("data", ""))
    dbuf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    peers = [bytes.fromhex(p) for p in m.get("peers", [])]
    arr = (C.c_char_p * max(1, len(peers)))(*peers)
    cm = PE.MessageC(m["type"], C.cast(dbuf, C.POINTER(C.c_uint8)), len(data),
                     C.cast(arr, C.POINTER(C.c_char_p)), len(peers), m.get("tree_width", 0),
                     m.get("tree_max_width", 0), m.get("num_peers", 0))
    n = C.c_size_t()
    assert L.ps_msg_encode(C.byref(cm), None, 0, C.byref(n)) == -7  # PS_E_RANGE: sizing call
    buf = C.create_string_buffer(n.value)
    assert L.ps_msg_encode(C.byref(cm), buf, n.value, C.byref(n)) == 0
    return buf.raw[:n.value]


@pytest.mark.parametrize("i", range(len(vectors())))
def test_encode_matches_golden(i):
    v = vectors()[i]
    assert encode_raw(v["msg"]) == bytes.fromhex(v["line"])


def test_reference_payload_lines():
    """pubsub_test.go:106's payloads, as a Go peer reads them off the stream."""
    assert W.encode(W.Message(W.DATA, b"message number 0")) == b'{"Type":0,"data":"bWVzc2FnZSBudW1iZXIgMA=="}\n'
    assert W.encode(W.Message(W.JOIN)) == b'{"Type":1}\n'
    assert W.encode(W.Message(W.PART)) == b'{"Type":2}\n'


@pytest.mark.parametrize("i", range(len(vectors())))
def test_decode_golden_round_trip(i):
    v = vectors()[i]
    line = bytes.fromhex(v["line"])
    m, used = W.decode(line)
    assert used == len(line)  # the trailing newline is consumed as whitespace
    exp = to_msg(v["msg"])
    assert (m.type, m.data, m.tree_width, m.tree_max_width, m.num_peers) == \
        (exp.type, exp.data, exp.tree_width, exp.tree_max_width, exp.num_peers)
    # strings come back as encoding/json decodes them: invalid UTF-8 became U+FFFD
    assert m.peers == [p.encode("utf-8", "surrogateescape").decode("utf-8", "replace") for p in exp.peers]
    assert W.encode(m) == line or any("�" in p for p in m.peers)


def test_decode_go_decoder_rules():
    """json.Decoder semantics readMessage relies on: case-insensitive field
    names, unknown fields skipped, null leaves a field unset, a repeated key
    replaces the value, whitespace anywhere, surrogate pairs."""
    m, _ = W.decode(b' {"type": 3 , "PARENTS": ["a","b"], "x": {"y": [1, 2.5e3, true, null, "z"]},'
                    b' "TreeWidth": 2, "data": null, "numPeers": -4, "parents": ["\\u00e9\\ud83d\\ude00"]}')
    assert (m.type, m.peers, m.tree_width, m.data, m.num_peers) == (3, ["é\U0001F600"], 2, b"", -4)
    m, _ = W.decode(b'{"data":"AAE=","data":"AgM="}')
    assert m.data == b"\x02\x03"
    m, used = W.decode(b'{}\n{"Type":1}\n')
    assert (m.type, used) == (0, 3)


def test_decode_stream_of_values():
    """A stream carries back-to-back Encode outputs; each Decode takes one."""
    msgs = [W.Message(W.DATA, b"message number %d" % i) for i in range(5)] + \
        [W.Message(W.UPDATE, peers=["QmA"], tree_width=2, tree_max_width=5)]
    stream = b"".join(W.encode(m) for m in msgs)
    out = []
    while stream:
        m, used = W.decode(stream)
        out.append(m)
        stream = stream[used:]
    assert out == msgs


@pytest.mark.parametrize("bad", [
    b"", b"{", b'{"Type":}', b'{"Type":1.5}', b'{"Type":"1"}', b'{"data":"AAE"}',
    b'{"data":"A=AA"}', b'{"data":"@@@@"}', b'{"parents":"x"}', b'{"parents":[1]}',
    b'{"Type":1,}', b'["Type"]', b'{"a":"\x01"}', b'{"a":tru}', b'{"a":"\\q"}',
])
def test_decode_rejects_malformed(bad):
    with pytest.raises(PE.EngineError):
        W.decode(bad)


def test_encode_sizing_and_empty_fields():
    import ctypes as C
    L = PE.load()
    cm = PE.MessageC(0, None, 0, None, 0, 0, 0, 0)
    n = C.c_size_t()
    assert L.ps_msg_encode(C.byref(cm), None, 0, C.byref(n)) == -7
    assert n.value == len(b'{"Type":0}\n')
    buf = C.create_string_buffer(n.value - 1)
    assert L.ps_msg_encode(C.byref(cm), buf, n.value - 1, C.byref(n)) == -7  # short: nothing written
    assert L.ps_msg_encode(None, None, 0, C.byref(n)) == -1


def test_cpp_api_mirror_codec():
    """writeMessage / readMessage of the C++ API mirror (include/pubsub.hpp),
    host only: the native test binary's codec case."""
    import subprocess
    from psengine import _build
    exe = _build.build_cpp_tests()
    p = subprocess.run([exe, "TestWireCodec"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and "--- PASS: TestWireCodec" in p.stdout, p.stdout + p.stderr
