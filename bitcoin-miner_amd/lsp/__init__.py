"""lsp -- the Live Sequence Protocol of the reference (src/github.com/cmu440/lsp), a
reliable, in-order, windowed message protocol over UDP with epoch-based failure
detection (p1.pdf pp.2-11).  Plumbing for SURVEY.md 8(f) rows 3-4: it carries the
miner's Request/Result messages around the GPU hot path; it is not on that path."""
from .client import Client, LSPError, NewClient
from .message import Message, MsgType, NewAck, NewConnect, NewData
from .params import (DefaultEpochLimit, DefaultEpochMillis, DefaultWindowSize, NewParams,
                     Params)
from .server import NewServer, Server

__all__ = ["Client", "LSPError", "NewClient", "Message", "MsgType", "NewAck", "NewConnect",
           "NewData", "DefaultEpochLimit", "DefaultEpochMillis", "DefaultWindowSize",
           "NewParams", "Params", "NewServer", "Server"]
