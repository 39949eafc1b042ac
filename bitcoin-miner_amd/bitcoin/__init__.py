"""bitcoin -- mirror of the reference package src/github.com/cmu440/bitcoin.

hash.go (Hash) and message.go (Message, MsgType, NewRequest, NewResult, NewJoin) come
from the gpuhash mirror; this package adds the Go-compatible JSON framing used inside
LSP payloads (p1.pdf p.13: "each message must first be marshalled ... using Go's json
package") and the three programs of p1.pdf pp.13-15: server (job chunking + scheduler),
miner (the GPU hot path), client.
"""
from __future__ import annotations

import json
import os
import re

import lsp
from gpuhash import Hash, Message, MsgType, NewJoin, NewRequest, NewResult

__all__ = ["Hash", "Message", "MsgType", "NewJoin", "NewRequest", "NewResult", "marshal",
           "unmarshal", "params_from_env", "ParseUint", "UINT64_MAX", "EMPTY_RESULT"]

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


_FOLD = str.maketrans("ABCDEFGHIJKLMNOPQRSTUVWXYZ", "abcdefghijklmnopqrstuvwxyz")


class _Members(list):
    """Every value one struct field received, in document order (go_object)."""


def go_object(pairs) -> dict:
    """json.loads object hook with encoding/json's field matching: a key selects the
    struct field whose name equals it ignoring (ASCII) case.  Go decodes EVERY such member
    in order into the field, so all of them are kept (case-folded key -> _Members): a later
    null leaves the field as an earlier member set it, and a member of the wrong type fails
    the message even when a later one is fine (csrc/lsp_native.h jfields)."""
    out: dict = {}
    for k, v in pairs:
        out.setdefault(k.translate(_FOLD), _Members()).append(v)
    return out


def _field(d: dict, key: str, ok, default):
    """The value json.Unmarshal leaves in field `key`: each matching member in order,
    null skipped, the last accepted one wins; `ok(v)` False for any member -> ValueError
    (Go keeps the first UnmarshalTypeError and returns it)."""
    val = default
    for v in d.get(key.translate(_FOLD), ()):
        if v is None:
            continue
        if not ok(v):
            raise ValueError(f"json: cannot unmarshal {v!r} into Go struct field Message.{key}")
        val = v
    return val


class _IntLit(int):
    """A JSON integer literal that keeps its text: Go's strconv.ParseUint refuses "-0",
    which int() reads as 0."""

    def __new__(cls, text: str):
        o = int.__new__(cls, int(text))
        o.text = text
        return o


def _u64(d: dict, key: str) -> int:
    """A uint64 field as Go's json.Unmarshal accepts it: an integer literal in
    [0, 2^64-1] (no fraction, exponent or sign); anything else fails the whole message."""
    return int(_field(d, key, lambda v: isinstance(v, _IntLit) and not v.text.startswith("-")
                      and v <= UINT64_MAX, 0))


_LONE_SURROGATE = re.compile("[\ud800-\udfff]")


def _go_replace(err: UnicodeDecodeError):
    """utf-8 decode error handler with Go's utf8.DecodeRune rule: ONE U+FFFD per invalid
    byte, decoding resumes at the next byte (Python's 'replace' emits one U+FFFD for a
    whole truncated sequence: b'\xe2\x82A' -> '\ufffdA' where Go gives '\ufffd\ufffdA')."""
    return "\ufffd", err.start + 1


import codecs  # noqa: E402

codecs.register_error("go-utf8", _go_replace)


def go_utf8(raw: bytes) -> str:
    """bytes -> str as Go's JSON decoder reads string contents: invalid UTF-8 (truncated or
    overlong sequences, encoded surrogates, stray continuation bytes) as U+FFFD per byte."""
    return bytes(raw).decode("utf-8", "go-utf8")


def _not_json(name: str):
    raise ValueError(f"invalid character in JSON: {name}")


def unmarshal(raw: bytes) -> Message:
    """json.Unmarshal into bitcoin.Message (message.go:16-21); raises ValueError where Go
    would return an error, so callers drop the message as the reference would."""
    if isinstance(raw, (bytes, bytearray)):
        # Go's decoder turns invalid UTF-8 into U+FFFD instead of failing the message
        raw = go_utf8(raw)
    d = json.loads(raw, object_pairs_hook=go_object, parse_int=_IntLit,
                   parse_constant=_not_json)  # NaN / Infinity: not JSON, Go refuses them
    if not isinstance(d, dict):
        raise ValueError("json: cannot unmarshal non-object into Go value of type bitcoin.Message")
    t = int(_field(d, "Type", lambda v: isinstance(v, _IntLit) and -(1 << 63) <= v < 1 << 63, 0))
    data = _field(d, "Data", lambda v: isinstance(v, str), "")
    # a "\ud800" escape without its pair: Go decodes it to U+FFFD (json.loads keeps the lone
    # surrogate, which has no UTF-8 bytes to hash); valid pairs are already combined
    data = _LONE_SURROGATE.sub("\ufffd", data)
    return Message(MsgType(t), Data=data, Lower=_u64(d, "Lower"), Upper=_u64(d, "Upper"),
                   Hash=_u64(d, "Hash"), Nonce=_u64(d, "Nonce"))


def params_from_env() -> lsp.Params:
    """lsp.NewParams() with LSP_EPOCH_LIMIT / LSP_EPOCH_MILLIS / LSP_WINDOW_SIZE overrides."""
    p = lsp.NewParams()
    p.EpochLimit = int(os.environ.get("LSP_EPOCH_LIMIT", p.EpochLimit))
    p.EpochMillis = int(os.environ.get("LSP_EPOCH_MILLIS", p.EpochMillis))
    p.WindowSize = int(os.environ.get("LSP_WINDOW_SIZE", p.WindowSize))
    return p
