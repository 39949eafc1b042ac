"""bitcoin -- mirror of the reference package src/github.com/cmu440/bitcoin.

hash.go (Hash) and message.go (Message, MsgType, NewRequest, NewResult, NewJoin) come
from the gpuhash mirror; this package adds the Go-compatible JSON framing used inside
LSP payloads (p1.pdf p.13: "each message must first be marshalled ... using Go's json
package") and the three programs of p1.pdf pp.13-15: server (job chunking + scheduler),
miner (the GPU hot path), client.
"""
from __future__ import annotations

import os

import lsp
from gojson import LONE_SURROGATE as _LONE_SURROGATE
from gojson import IntLit as _IntLit
from gojson import field as _field
from gojson import go_object, go_utf8  # noqa: F401 (re-exported for the tests)
from gojson import loads as _go_loads
from gojson import u64 as _u64
from gpuhash import Hash, Message, MsgType, NewJoin, NewRequest, NewResult

__all__ = ["Hash", "Message", "MsgType", "NewJoin", "NewRequest", "NewResult", "marshal",
           "unmarshal", "params_from_env", "SEND_COPIES", "ParseUint", "UINT64_MAX", "EMPTY_RESULT"]

UINT64_MAX = (1 << 64) - 1
# (Hash, Nonce) of an empty range: the top of the lexicographic key order, so folding it
# into any merge changes nothing (the identity of the (hash, nonce) min)
EMPTY_RESULT = (UINT64_MAX, UINT64_MAX)


def ParseUint(s: str) -> int:
    """strconv.ParseUint(s, 10, 64) as Go's client would parse maxNonce: ASCII decimal
    digits only (no sign, no spaces, no '_'), value <= 2^64-1; ValueError otherwise.
    (Python's int() also accepts '+5', ' 5', '1_000' and negatives.)"""
    if not s or not s.isascii() or not s.isdigit():
        raise ValueError(f'strconv.ParseUint: parsing "{s}": invalid syntax')
    v = int(s)
    if v > UINT64_MAX:
        raise ValueError(f'strconv.ParseUint: parsing "{s}": value out of range')
    return v


def go_json_string(s: str) -> str:
    """A string as Go's encoding/json writes it (encodeState.string): \\" and \\\\, \\n \\r
    \\t, other control characters as \\u00XX, <, > and & as \\u003c.. (HTML-safe), U+2028
    and U+2029 as \\u2028/\\u2029, any other character as raw UTF-8, and what is not valid
    UTF-8 (here: a lone surrogate) as U+FFFD."""
    out = ['"']
    for c in s:
        o = ord(c)
        if c == '"':
            out.append('\\"')
        elif c == "\\":
            out.append("\\\\")
        elif c == "\n":
            out.append("\\n")
        elif c == "\r":
            out.append("\\r")
        elif c == "\t":
            out.append("\\t")
        elif o < 0x20 or c in "<>&" or o in (0x2028, 0x2029):
            out.append(f"\\u{o:04x}")
        elif 0xD800 <= o < 0xE000:
            out.append("\ufffd")
        else:
            out.append(c)
    out.append('"')
    return "".join(out)


def marshal(m: Message) -> bytes:
    """json.Marshal(bitcoin.Message) byte for byte as Go writes it: fields in the order
    of message.go:16-21, no spaces, Data escaped as go_json_string."""
    d = m.to_json()
    return ("{" + ",".join(f'"{k}":' + (go_json_string(v) if k == "Data" else str(int(v)))
                           for k, v in d.items()) + "}").encode()


def unmarshal(raw: bytes) -> Message:
    """json.Unmarshal into bitcoin.Message (message.go:16-21); raises ValueError where Go
    would return an error, so callers drop the message as the reference would."""
    # invalid UTF-8 becomes U+FFFD (Go does not fail the message); NaN / Infinity are refused
    d = _go_loads(raw)
    if not isinstance(d, dict):
        raise ValueError("json: cannot unmarshal non-object into Go value of type bitcoin.Message")
    t = int(_field(d, "Type", lambda v: isinstance(v, _IntLit) and -(1 << 63) <= v < 1 << 63, 0))
    data = _field(d, "Data", lambda v: isinstance(v, str), "")
    # a "\ud800" escape without its pair: Go decodes it to U+FFFD (json.loads keeps the lone
    # surrogate, which has no UTF-8 bytes to hash); valid pairs are already combined
    data = _LONE_SURROGATE.sub("\ufffd", data)
    return Message(MsgType(t), Data=data, Lower=_u64(d, "Lower"), Upper=_u64(d, "Upper"),
                   Hash=_u64(d, "Hash"), Nonce=_u64(d, "Nonce"))


# Datagram copies the server, miner and client send (lsp.Params.SendCopies; 1 is the
# protocol exactly as p1.pdf specifies it).  At config 5's 10% read and write drops a lone
# datagram is lost with p = 0.19 and waits for the next 2-s epoch; three copies make that
# p^3 = 0.007.
SEND_COPIES = 3


def params_from_env() -> lsp.Params:
    """The programs' LSP parameters: lsp.NewParams() with SendCopies = SEND_COPIES, and
    LSP_EPOCH_LIMIT / LSP_EPOCH_MILLIS / LSP_WINDOW_SIZE / LSP_SEND_COPIES overrides."""
    p = lsp.NewParams()
    p.EpochLimit = int(os.environ.get("LSP_EPOCH_LIMIT", p.EpochLimit))
    p.EpochMillis = int(os.environ.get("LSP_EPOCH_MILLIS", p.EpochMillis))
    p.WindowSize = int(os.environ.get("LSP_WINDOW_SIZE", p.WindowSize))
    p.SendCopies = max(1, int(os.environ.get("LSP_SEND_COPIES", SEND_COPIES)))
    return p
