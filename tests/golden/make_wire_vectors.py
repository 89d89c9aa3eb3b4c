"""Generates wire_vectors.json: the lines writeMessage (pubsub.go:122-124,
json.NewEncoder(s).Encode(m) over the Message struct of pubsub.go:146-153)
puts on a stream, restated from encoding/json's documented rules with the
Python standard library (independently of the C codec under test):

  * fields in struct order; `Type` always, the rest `omitempty`
    (data, parents, treewidth, treemaxwidth, numpeers);
  * []byte as standard base64 with padding;
  * strings: \\" \\\\ \\n \\r \\t, other control bytes as \\u00XX, HTML-safe
    <, >, & as \\u003c \\u003e \\u0026, U+2028/2029 escaped, invalid UTF-8 as
    \\ufffd (Go of the reference's era -- gx go-libp2p 3.3.7, 2016 -- predates
    Go 1.22, which writes \\b and \\f instead of \\u0008 / \\u000c);
  * Encode appends '\\n'.

The payloads are the reference test's (pubsub_test.go:106 "message number
%d") plus the control messages subtree.go builds (Join, Part, Update with
parents/treewidth/treemaxwidth, State with numpeers) and escaping edge cases.
No Go toolchain exists in this image, so the vectors are pinned to this
restatement of the published encoding rules, not to a Go run.

    python tests/golden/make_wire_vectors.py
"""
import base64
import json
import os

LS, PS = "\u2028", "\u2029"


def go_string(s: bytes) -> str:
    out = ['"']
    i = 0
    while i < len(s):
        c = s[i]
        if c < 0x80:
            ch = chr(c)
            if ch in '"\\':
                out.append("\\" + ch)
            elif ch == "\n":
                out.append("\\n")
            elif ch == "\r":
                out.append("\\r")
            elif ch == "\t":
                out.append("\\t")
            elif c < 0x20 or ch in "<>&":
                out.append("\\u%04x" % c)
            else:
                out.append(ch)
            i += 1
            continue
        cp = None
        for n in (2, 3, 4):  # the one valid UTF-8 sequence starting at i
            try:
                t = s[i:i + n].decode("utf-8")
            except UnicodeDecodeError:
                continue
            if len(t) == 1:
                cp = t
                break
        if cp is None:
            out.append("\\ufffd")
            i += 1
            continue
        out.append({LS: "\\u2028", PS: "\\u2029"}.get(cp, cp))
        i += len(cp.encode("utf-8"))
    out.append('"')
    return "".join(out)


def go_encode(m: dict) -> bytes:
    parts = ['"Type":%d' % m["type"]]
    if m.get("data"):
        parts.append('"data":"%s"' % base64.b64encode(bytes.fromhex(m["data"])).decode())
    if m.get("peers"):
        parts.append('"parents":[%s]' % ",".join(go_string(bytes.fromhex(p)) for p in m["peers"]))
    for k, name in (("tree_width", "treewidth"), ("tree_max_width", "treemaxwidth"),
                    ("num_peers", "numpeers")):
        if m.get(k):
            parts.append('"%s":%d' % (name, m[k]))
    return ("{" + ",".join(parts) + "}\n").encode("utf-8")


PID = b"QmYyQSo1c1Ym7orWxLYvCrM2EmxFTANf8wXmmE7DWjhx5N"  # a base58 multihash peer id


def messages():
    """Peers and data are hex so that invalid UTF-8 survives the JSON file."""
    ms = [{"type": 0, "data": ("message number %d" % i).encode().hex()} for i in (0, 1, 9, 42, 1000)]
    odd = [b"<a>&b", b'q"u\\o', b"t\tn\nr\r", b"\x01\x08\x0c\x1f\x7f", (LS + PS).encode(),
           "é\U0001F600".encode(), b"bad\xff\xc3(", b"\xed\xa0\x80", b""]
    ms += [
        {"type": 1},                                                           # Join
        {"type": 2},                                                           # Part
        {"type": 3, "peers": [PID.hex()], "tree_width": 2, "tree_max_width": 5},  # Update
        {"type": 4, "peers": [PID.hex(), PID[::-1].hex()], "num_peers": 3},    # State
        {"type": 0, "data": bytes(range(256)).hex()},                          # every byte
        {"type": 0, "data": "00"}, {"type": 0, "data": "0001"}, {"type": 0, "data": "000102"},
        {"type": 4, "peers": [p.hex() for p in odd], "tree_width": -1},
        {"type": 7, "num_peers": 1 << 40},
    ]
    return ms


def main():
    vec = [{"msg": m, "line": go_encode(m).hex()} for m in messages()]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wire_vectors.json")
    with open(path, "w") as f:
        json.dump(vec, f, indent=1)
    print(path, len(vec))


if __name__ == "__main__":
    main()
