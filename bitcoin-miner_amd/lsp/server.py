"""LSP server -- the API of src/github.com/cmu440/lsp/server_api.go:6-39 (NewServer,
Read, Write, CloseConn, Close), implemented over lspnet UDP with one loop thread.

Connection IDs are assigned sequentially from 1 (p1.pdf p.3); a repeated Connect from a
host:port that already has a connection is answered with its existing ID instead of
opening a second one (p1.pdf p.6)."""
from __future__ import annotations

import queue
import threading
import time

import lspnet

from .client import LSPError
from .endpoint import ConnState, CopyFilter, Loop
from .message import Message, MsgType, NewAck
from .params import Params, NewParams


class Server:
    def __init__(self, port: int, params: Params | None = None):
        self._p = params or NewParams()
        self._conn = lspnet.ListenUDP(port)
        self.port = self._conn.local_addr()[1]
        self._reads: queue.Queue = queue.Queue()
        self._conns: dict[int, ConnState] = {}
        self._addr_of: dict[int, tuple] = {}
        self._id_of: dict[tuple, int] = {}
        self._next_id = 1
        self._closing_all = False
        self._copies = CopyFilter(self._p.EpochMillis / 1000.0)
        self._done = threading.Event()
        self._closed = False
        self._lost_during_close = False
        self._loop = Loop(self._conn, self._p.EpochMillis, self._on_datagram, self._on_command,
                          self._on_epoch, role="lsp-server")
        self._loop.start()

    # ---- API -----------------------------------------------------------------
    def Read(self) -> tuple[int, bytes]:
        """Blocks for (connID, payload) from any client.  Raises LSPError(conn_id) when a
        client's connection is lost or closed (conn_id 0 once the server is closed)."""
        return self.read_until(None)

    def read_until(self, deadline: float | None):
        """Read(), but returns None once time.monotonic() passes `deadline` with nothing
        to return (None: block like Read).  Not in server_api.go: the bitcoin server uses
        it to wake for its own timers (speculative job copies) between messages."""
        try:
            if deadline is None:
                item = self._reads.get()
            else:
                item = self._reads.get(timeout=max(0.0, deadline - time.monotonic()))
        except queue.Empty:
            return None
        if item[0] == "data":
            return item[1], item[2]
        if item[0] == "closed":
            self._reads.put(item)
            raise LSPError("server closed", 0)
        raise LSPError(item[2], item[1])

    def Write(self, conn_id: int, payload: bytes) -> None:
        st = self._conns.get(conn_id)
        if self._closed or st is None or st.lost or st.closing:
            raise LSPError(f"connection {conn_id} is lost or closed", conn_id)
        self._loop.post("write", conn_id, bytes(payload))

    def CloseConn(self, conn_id: int) -> None:
        """Non-blocking: pending messages to the client are still flushed."""
        if conn_id not in self._conns:
            raise LSPError(f"no connection {conn_id}", conn_id)
        self._loop.post("closeconn", conn_id)

    def Close(self) -> None:
        """Blocks until every connection has flushed (or been lost); raises if any client
        was lost meanwhile."""
        if self._closed:
            return
        self._closed = True
        self._loop.post("close")
        self._done.wait()
        self._loop.stop()
        self._loop.post("noop")
        self._loop.stopped.wait(5)
        self._conn.close()
        self._reads.put(("closed",))
        if self._lost_during_close:
            raise LSPError("a client was lost while closing", 0)

    # ---- loop thread ------------------------------------------------------------
    def _sender(self, addr):
        return lambda m: self._conn.write_to(m.marshal(), addr)

    def _on_datagram(self, data: bytes, addr) -> None:
        again = self._copies.copy_of(addr, data, time.monotonic())
        if again is not None:  # a copy: repeat the first one's reply
            if again:
                self._conn.write_to(again, addr)
            return
        try:
            m = Message.unmarshal(data)
        except (ValueError, KeyError):
            return
        if m.Type == MsgType.MsgConnect:
            cid = self._id_of.get(addr)
            if cid is None:
                if self._closing_all:
                    return
                cid = self._next_id
                self._next_id += 1
                self._id_of[addr] = cid
                self._addr_of[cid] = addr
                self._conns[cid] = ConnState(cid, self._p.WindowSize, self._p.EpochLimit, self._sender(addr),
                                             self._p.SendCopies)
            st = self._conns.get(cid)
            if st is not None:
                st.mark_heard()
                for _ in range(max(1, self._p.SendCopies)):
                    self._conn.write_to(NewAck(cid, 0).marshal(), addr)
            return
        st = self._conns.get(m.ConnID)
        if st is None or self._addr_of.get(m.ConnID) != addr:
            return
        for payload in st.on_message(m):
            self._reads.put(("data", m.ConnID, payload))
        if m.Type == MsgType.MsgData:
            self._copies.reply(addr, data, NewAck(m.ConnID, m.SeqNum).marshal())
        self._reap()

    def _on_command(self, cmd) -> None:
        if cmd[0] == "write":
            st = self._conns.get(cmd[1])
            if st is not None and not st.lost:
                st.write(cmd[2])
        elif cmd[0] == "closeconn":
            st = self._conns.get(cmd[1])
            if st is not None:
                st.closing = True
        elif cmd[0] == "close":
            self._closing_all = True
            for st in self._conns.values():
                st.closing = True
        self._reap()

    def _on_epoch(self) -> None:
        for st in list(self._conns.values()):
            st.on_epoch()
        self._reap()

    def _reap(self) -> None:
        """Drops lost connections and closed ones whose messages are all acknowledged."""
        for cid, st in list(self._conns.items()):
            if st.lost:
                if self._closing_all:
                    self._lost_during_close = True
                self._drop(cid)
                self._reads.put(("err", cid, f"connection {cid} lost ({st.lost_reason}; this loop's "
                                             f"latest epoch {1000 * self._loop.max_late:.0f} ms late)"))
            elif st.closing and st.flushed():
                self._drop(cid)
                if not self._closing_all:
                    self._reads.put(("err", cid, f"connection {cid} closed"))
        if self._closing_all and not self._conns:
            self._done.set()

    def _drop(self, cid: int) -> None:
        self._conns.pop(cid, None)
        addr = self._addr_of.pop(cid, None)
        if addr is not None:
            self._id_of.pop(addr, None)
            self._copies.forget(addr)


def NewServer(port: int, params: Params | None = None) -> Server:
    return Server(port, params)
