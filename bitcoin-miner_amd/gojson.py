"""gojson -- the rules of Go's encoding/json that the reference's message readers rely on,
shared by bitcoin.unmarshal (bitcoin.Message, bitcoin/message.go:16-21) and
lsp.Message.unmarshal (lsp/message.go:17-22), and restated in C++ by csrc/lsp_native.h:

  go_object   json.loads object hook: keys select struct fields ignoring case (ASCII, and
              the long s / Kelvin sign that fold to s / k), and
              EVERY matching member is kept in document order (Go decodes each of them)
  field       the value Unmarshal leaves in a scalar field: members in order, null
              skipped, a wrong-typed member fails the message
  IntLit      an integer literal that keeps its text (ParseUint refuses "-0")
  go_utf8     invalid UTF-8 as one U+FFFD per byte (utf8.DecodeRune)
  loads       json.loads with these hooks; NaN / Infinity refused
"""
from __future__ import annotations

import codecs
import json
import re

UINT64_MAX = (1 << 64) - 1
INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1

# key folding as encoding/json matches a key to a field name: ASCII case, plus the two
# non-ASCII runes whose simple case folding reaches an ASCII letter, the long s U+017F (~ s)
# and the Kelvin sign U+212A (~ k) (fold.go equalFoldRight)
_FOLD = str.maketrans({**{chr(c): chr(c + 32) for c in range(ord("A"), ord("Z") + 1)},
                       "\u017f": "s", "\u212a": "k"})


class Members(list):
    """Every value one struct field received, in document order (go_object)."""


def go_object(pairs) -> dict:
    """json.loads object hook with encoding/json's field matching: a key selects the
    struct field whose name equals it ignoring (ASCII) case.  Go decodes EVERY such member
    in order into the field, so all of them are kept (case-folded key -> Members): a later
    null leaves the field as an earlier member set it, and a member of the wrong type fails
    the message even when a later one is fine (csrc/lsp_native.h jfields)."""
    out: dict = {}
    for k, v in pairs:
        out.setdefault(k.translate(_FOLD), Members()).append(v)
    return out


def field(d: dict, key: str, ok, default):
    """The value json.Unmarshal leaves in a scalar field `key` (int, uint64, string): each
    matching member in order, null skipped (a no-op for these kinds; a []byte field, where
    null resets to nil, is read by lsp.message), the last accepted one wins; `ok(v)` False
    for any member -> ValueError (Go keeps the first UnmarshalTypeError and returns it)."""
    val = default
    for v in d.get(key.translate(_FOLD), ()):
        if v is None:
            continue
        if not ok(v):
            raise ValueError(f"json: cannot unmarshal {v!r} into Go struct field Message.{key}")
        val = v
    return val


class IntLit(int):
    """A JSON integer literal that keeps its text: Go's strconv.ParseUint refuses "-0",
    which int() reads as 0."""

    def __new__(cls, text: str):
        o = int.__new__(cls, int(text))
        o.text = text
        return o


def u64(d: dict, key: str) -> int:
    """A uint64 field as Go's json.Unmarshal accepts it: an integer literal in
    [0, 2^64-1] (no fraction, exponent or sign); anything else fails the whole message."""
    return int(field(d, key, lambda v: isinstance(v, IntLit) and not v.text.startswith("-")
                     and v <= UINT64_MAX, 0))


def i64(d: dict, key: str) -> int:
    """An int (64-bit) field: an integer literal in [-2^63, 2^63-1] (strconv.ParseInt)."""
    return int(field(d, key, lambda v: isinstance(v, IntLit) and INT64_MIN <= v <= INT64_MAX, 0))


LONE_SURROGATE = re.compile("[\ud800-\udfff]")


def _go_replace(err: UnicodeDecodeError):
    """utf-8 decode error handler with Go's utf8.DecodeRune rule: ONE U+FFFD per invalid
    byte, decoding resumes at the next byte (Python's 'replace' emits one U+FFFD for a
    whole truncated sequence: b'\xe2\x82A' -> '\ufffdA' where Go gives '\ufffd\ufffdA')."""
    return "\ufffd", err.start + 1


codecs.register_error("go-utf8", _go_replace)


def go_utf8(raw: bytes) -> str:
    """bytes -> str as Go's JSON decoder reads string contents: invalid UTF-8 (truncated or
    overlong sequences, encoded surrogates, stray continuation bytes) as U+FFFD per byte."""
    return bytes(raw).decode("utf-8", "go-utf8")


def not_json(name: str):
    raise ValueError(f"invalid character in JSON: {name}")



def loads(raw):
    """json.loads with Go's field matching (go_object), integer literals kept as IntLit, and
    NaN / Infinity refused; bytes are decoded as Go's decoder reads them (go_utf8)."""
    if isinstance(raw, (bytes, bytearray)):
        raw = go_utf8(raw)
    return json.loads(raw, object_pairs_hook=go_object, parse_int=IntLit, parse_constant=not_json)
