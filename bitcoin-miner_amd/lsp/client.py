"""LSP client -- the API of src/github.com/cmu440/lsp/client_api.go:6-30 (NewClient,
ConnID, Read, Write, Close), implemented over lspnet UDP with one loop thread."""
from __future__ import annotations

import queue
import threading
import time

import lspnet

from .endpoint import ConnState, CopyFilter, Loop
from .message import Message, MsgType, NewAck, NewConnect
from .params import Params, NewParams


class LSPError(Exception):
    def __init__(self, msg: str, conn_id: int = 0):
        super().__init__(msg)
        self.conn_id = conn_id


class Client:
    def __init__(self, hostport: str, params: Params | None = None):
        self._p = params or NewParams()
        self._conn = lspnet.DialUDP(hostport)
        self._reads: queue.Queue = queue.Queue()
        self._st: ConnState | None = None
        self._conn_id = 0
        self._connected = threading.Event()
        self._done = threading.Event()   # Close() may return
        self._failed = False
        self._closed = False
        self._connect_silent = 0
        self._copies = CopyFilter(self._p.EpochMillis / 1000.0)
        self.lost_reason = ""
        self._loop = Loop(self._conn, self._p.EpochMillis, self._on_datagram, self._on_command,
                          self._on_epoch, role="lsp-client")
        self._loop.start()
        self._send_connect()
        self._connected.wait()
        if self._failed:
            self._shutdown()
            raise LSPError(f"could not connect to {hostport} ({self.lost_reason})")

    # ---- API -----------------------------------------------------------------
    def ConnID(self) -> int:
        return self._conn_id

    def Read(self) -> bytes:
        """Blocks for the next in-order payload; raises once the connection is closed or
        lost and nothing is left to return."""
        item = self._reads.get()
        if item[0] == "err":
            self._reads.put(item)  # every later Read fails too
            raise LSPError(item[1], self._conn_id)
        return item[1]

    def Write(self, payload: bytes) -> None:
        """Non-blocking; raises if the connection has been lost."""
        if self._closed or self._st is None or self._st.lost:
            raise LSPError("connection lost", self._conn_id)
        self._loop.post("write", bytes(payload))

    def Close(self) -> None:
        """Blocks until every pending message is sent and acknowledged (or the
        connection is lost), then stops the loop thread."""
        if self._closed:
            return
        self._closed = True
        self._loop.post("close")
        self._done.wait()
        self._shutdown()

    # ---- loop thread ------------------------------------------------------------
    def _send(self, m: Message) -> None:
        self._conn.write_to(m.marshal())

    def _send_connect(self) -> None:
        for _ in range(max(1, self._p.SendCopies)):
            self._send(NewConnect())

    def _on_datagram(self, data: bytes, addr) -> None:
        # only the server's datagrams: the reference's lspnet.DialUDP is a connected UDP
        # socket, which the kernel filters by source (csrc/lsp_native.h does the same)
        if addr != self._conn.peer:
            return
        again = self._copies.copy_of(addr, data, time.monotonic())
        if again is not None:  # a copy: repeat the first one's reply
            if again:
                self._conn.write_to(again)
            return
        try:
            m = Message.unmarshal(data)
        except (ValueError, KeyError):
            return
        if self._st is None:
            if m.Type == MsgType.MsgAck and m.SeqNum == 0 and m.ConnID > 0:
                self._conn_id = m.ConnID
                self._st = ConnState(m.ConnID, self._p.WindowSize, self._p.EpochLimit, self._send,
                                     self._p.SendCopies)
                self._connected.set()
            return
        if m.ConnID != self._conn_id:
            return
        for payload in self._st.on_message(m):
            self._reads.put(("data", payload))
        if m.Type == MsgType.MsgData:
            self._copies.reply(addr, data, NewAck(m.ConnID, m.SeqNum).marshal())
        self._check_close()

    def _on_command(self, cmd) -> None:
        if cmd[0] == "write" and self._st is not None and not self._st.lost:
            self._st.write(cmd[1])
        elif cmd[0] == "close":
            if self._st is not None:
                self._st.closing = True
            self._check_close()

    def _on_epoch(self) -> None:
        if self._st is None:
            self._connect_silent += 1
            if self._connect_silent >= self._p.EpochLimit:
                self._failed = True
                self.lost_reason = f"no connect ack in {self._connect_silent} epochs"
                self._connected.set()
            else:
                self._send_connect()
            return
        was_lost = self._st.lost
        self._st.on_epoch()
        if self._st.lost and not was_lost:
            self.lost_reason = (f"{self._st.lost_reason}; this loop's latest epoch "
                                f"{1000 * self._loop.max_late:.0f} ms late")
            self._reads.put(("err", f"connection lost ({self.lost_reason})"))
        self._check_close()

    def _check_close(self) -> None:
        st = self._st
        if st is None or (st.closing and (st.flushed() or st.lost)):
            if self._closed:
                self._reads.put(("err", "connection closed"))
                self._done.set()

    def _shutdown(self) -> None:
        self._loop.stop()
        self._loop.post("noop")
        self._loop.stopped.wait(5)
        self._conn.close()


def NewClient(hostport: str, params: Params | None = None) -> Client:
    return Client(hostport, params)
