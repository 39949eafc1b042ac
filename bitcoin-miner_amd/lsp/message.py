"""LSP wire messages -- mirror of src/github.com/cmu440/lsp/message.go.

MsgConnect / MsgData / MsgAck (message.go:8-12) and Message{Type, ConnID, SeqNum,
Payload} (message.go:17-22), marshalled exactly as Go's encoding/json does it: field
names as-is, []byte Payload as base64 (null when nil), so the frames are interoperable
with the reference's Go programs.
"""
from __future__ import annotations

import base64
import enum
import json
from dataclasses import dataclass


class MsgType(enum.IntEnum):
    MsgConnect = 0  # connection request from a client
    MsgData = 1     # data from a client or the server
    MsgAck = 2      # acknowledgement of a connect or data message


@dataclass
class Message:
    Type: MsgType
    ConnID: int = 0
    SeqNum: int = 0
    Payload: bytes | None = None

    def marshal(self) -> bytes:
        p = None if self.Payload is None else base64.b64encode(self.Payload).decode()
        return json.dumps({"Type": int(self.Type), "ConnID": self.ConnID, "SeqNum": self.SeqNum,
                           "Payload": p}, separators=(",", ":")).encode()

    @staticmethod
    def unmarshal(raw: bytes) -> "Message":
        # encoding/json field matching: keys ignore (ASCII) case, the last one wins, unknown
        # keys of any shape are skipped (as csrc/lsp_native.h)
        d = json.loads(raw, object_pairs_hook=lambda pairs: {k.lower(): v for k, v in pairs
                                                             if k.isascii()})
        p = d.get("payload")
        return Message(MsgType(int(d["type"])), int(d.get("connid", 0)), int(d.get("seqnum", 0)),
                       None if p is None else base64.b64decode(p))

    def __str__(self) -> str:  # message.go String()
        name = {MsgType.MsgConnect: "Connect", MsgType.MsgData: "Data", MsgType.MsgAck: "Ack"}[self.Type]
        payload = " " + (self.Payload or b"").decode(errors="replace") if self.Type == MsgType.MsgData else ""
        return f"[{name} {self.ConnID} {self.SeqNum}{payload}]"


def NewConnect() -> Message:
    return Message(MsgType.MsgConnect)


def NewData(conn_id: int, seq: int, payload: bytes) -> Message:
    return Message(MsgType.MsgData, conn_id, seq, payload)


def NewAck(conn_id: int, seq: int) -> Message:
    return Message(MsgType.MsgAck, conn_id, seq)
