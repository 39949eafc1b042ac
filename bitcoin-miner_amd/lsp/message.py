"""LSP wire messages -- mirror of src/github.com/cmu440/lsp/message.go.

MsgConnect / MsgData / MsgAck (message.go:8-12) and Message{Type, ConnID, SeqNum,
Payload} (message.go:17-22), marshalled exactly as Go's encoding/json does it: field
names as-is, []byte Payload as base64 (null when nil), so the frames are interoperable
with the reference's Go programs.
"""
from __future__ import annotations

import base64
import binascii
import enum
import json
from dataclasses import dataclass

import gojson


def b64decode_go(s: str) -> bytes:
    """base64.StdEncoding.DecodeString as encoding/json applies it to a []byte: padded
    standard alphabet, '\\r' and '\\n' ignored, anything else malformed -> ValueError."""
    t = s.replace("\r", "").replace("\n", "")
    if len(t) % 4:
        raise ValueError("illegal base64 data: length")
    try:
        return base64.b64decode(t.encode("ascii"), validate=True)
    except (binascii.Error, UnicodeEncodeError) as e:
        raise ValueError(f"illegal base64 data: {e}") from None


def byte_array(v: list) -> bytes:
    """A JSON array into a []byte, as encoding/json decodes one (any slice accepts an
    array; only Marshal insists on base64): each element a uint8, i.e. an integer literal
    in [0, 255] (strconv.ParseUint: no sign, fraction or exponent); null leaves its element
    0; anything else fails the message."""
    out = bytearray()
    for x in v:
        if x is None:
            out.append(0)
        elif isinstance(x, gojson.IntLit) and not x.text.startswith("-") and x <= 255:
            out.append(int(x))
        else:
            raise ValueError(f"json: cannot unmarshal {x!r} into Go struct field Message.Payload of type uint8")
    return bytes(out)


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
        """json.Unmarshal into lsp.Message, with the same Go rules as bitcoin.unmarshal and
        csrc/lsp_native.h lsp_unmarshal (gojson): keys match ignoring (ASCII) case, every
        matching member decodes in order, a wrong-typed member fails the message (ValueError),
        an absent field keeps its zero value (Type 0 = MsgConnect).  Type / ConnID / SeqNum
        are ints (integer literals only); Payload is a []byte: a string member is base64
        (StdEncoding, padded, CR / LF ignored), an array is its bytes (byte_array), and null
        resets it to nil.  A Type outside
        the three kinds is kept as a plain int (the endpoints then ignore the message)."""
        d = gojson.loads(raw)
        if not isinstance(d, dict):
            raise ValueError("json: cannot unmarshal non-object into Go value of type lsp.Message")
        t, conn, seq = gojson.i64(d, "Type"), gojson.i64(d, "ConnID"), gojson.i64(d, "SeqNum")
        payload = None
        for v in d.get("payload", ()):
            if v is None:
                payload = None
            elif isinstance(v, str):
                payload = b64decode_go(v)
            elif isinstance(v, list):
                payload = byte_array(v)
            else:
                raise ValueError(f"json: cannot unmarshal {v!r} into Go struct field Message.Payload")
        return Message(MsgType(t) if t in MsgType._value2member_map_ else t, conn, seq, payload)

    def __str__(self) -> str:  # message.go String()
        name = {MsgType.MsgConnect: "Connect", MsgType.MsgData: "Data", MsgType.MsgAck: "Ack"}.get(self.Type, "Unknown")
        payload = " " + (self.Payload or b"").decode(errors="replace") if self.Type == MsgType.MsgData else ""
        return f"[{name} {self.ConnID} {self.SeqNum}{payload}]"


def NewConnect() -> Message:
    return Message(MsgType.MsgConnect)


def NewData(conn_id: int, seq: int, payload: bytes) -> Message:
    return Message(MsgType.MsgData, conn_id, seq, payload)


def NewAck(conn_id: int, seq: int) -> Message:
    return Message(MsgType.MsgAck, conn_id, seq)
