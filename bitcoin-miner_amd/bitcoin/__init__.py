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

import lsp
from gpuhash import Hash, Message, MsgType, NewJoin, NewRequest, NewResult

__all__ = ["Hash", "Message", "MsgType", "NewJoin", "NewRequest", "NewResult", "marshal",
           "unmarshal", "params_from_env"]


def marshal(m: Message) -> bytes:
    """json.Marshal(bitcoin.Message) as Go writes it (field order of message.go:16-21)."""
    return json.dumps(m.to_json(), separators=(",", ":")).encode()


def unmarshal(raw: bytes) -> Message:
    d = json.loads(raw)
    return Message(MsgType(int(d.get("Type", 0))), Data=d.get("Data", "") or "",
                   Lower=int(d.get("Lower", 0)), Upper=int(d.get("Upper", 0)),
                   Hash=int(d.get("Hash", 0)), Nonce=int(d.get("Nonce", 0)))


def params_from_env() -> lsp.Params:
    """lsp.NewParams() with LSP_EPOCH_LIMIT / LSP_EPOCH_MILLIS / LSP_WINDOW_SIZE overrides."""
    p = lsp.NewParams()
    p.EpochLimit = int(os.environ.get("LSP_EPOCH_LIMIT", p.EpochLimit))
    p.EpochMillis = int(os.environ.get("LSP_EPOCH_MILLIS", p.EpochMillis))
    p.WindowSize = int(os.environ.get("LSP_WINDOW_SIZE", p.WindowSize))
    return p
