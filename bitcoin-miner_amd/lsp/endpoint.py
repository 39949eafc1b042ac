"""Per-connection LSP state machine + the single-threaded event loop both sides use.

Protocol (p1.pdf pp.2-7; the reference's attempt is lsp/client_impl.go and
lsp/server_impl.go, which cannot carry data as written -- SURVEY.md 2 rows 8-9):
  * data messages carry per-direction sequence numbers from 1 and are each acked;
  * sliding window: with n the oldest unacknowledged seq, only n..n+w-1 may be sent;
  * the receiver delivers in order, acks duplicates again, and remembers the last w
    distinct data messages it received;
  * every epoch: resend unacked data, re-ack the last w received messages, send Ack 0
    if no data has been received yet (heartbeat / connect ack), and count the epoch as
    silent unless something arrived; K silent epochs => connection lost.

Send copies (Params.SendCopies, an extension; 1 = the protocol exactly as p1.pdf
specifies it): a Connect and its ack, a Data message when it enters the window, the ack
of a Data message seen for the first time, and each epoch's resends, heartbeat and
re-acks go out that many times back to back; a duplicate is acked once (lspnet asks for
a 4 MiB socket receive buffer, so a window of copies from many connections at once is
not a burst the kernel drops).  Every endpoint recognises a copy
before parsing it (CopyFilter) and only repeats the reply its first instance got, so a
copy costs the receiver a bytes comparison.  The wire protocol is unchanged: a copy is
a duplicate, handled as the protocol's receive rules handle one, and endpoints that send
once interoperate.  On a link that drops each datagram with probability p, a message
then holds up its window until the next epoch with probability about 2 p^copies (its
copies, or all the acks, lost) instead of 1 - (1 - p)^2.

Like the reference's design (one handleMessages goroutine per endpoint), one loop
thread owns all protocol state; API calls post commands to it through a queue.

Diagnostics: a lost connection carries its reason -- the silent
epochs and how long ago the peer was last heard -- and the loop records how late its
epochs fire (`max_late`: a loop thread that is not scheduled, or waits for the GIL, stops
heartbeating its peers).  LSP_DIAG=1 prints every epoch that fires more than one epoch
late to stderr as it happens, and every 5 s the latest lateness of that window.
"""
from __future__ import annotations

import collections
import os
import queue
import selectors
import socket
import sys
import threading
import time

from .message import Message, MsgType, NewAck, NewData


class ConnState:
    """One side of one connection."""

    def __init__(self, conn_id: int, window: int, epoch_limit: int, send, copies: int = 1):
        self.conn_id = conn_id
        self.w = max(1, window)
        self.k = max(1, epoch_limit)
        self.send = send                     # send(Message)
        self.copies = max(1, copies)         # times each originated message is sent
        self.next_seq = 1                    # next data seq to assign
        self.pending = collections.deque()   # (seq, payload) not yet inside the window
        self.unacked = {}                    # seq -> payload, sent and not acked
        self.expected = 1                    # next seq to deliver
        self.rbuf = {}                       # received out of order
        self.recent = collections.deque(maxlen=self.w)  # last w distinct received seqs
        self.got_data = False
        self.silent = 0                      # whole epochs since the peer was last heard
        self.heard = True                    # heard from the peer since the last epoch
        self.lost = False
        self.lost_reason = ""
        self.last_heard = time.monotonic()
        self.closing = False

    # -- sending ---------------------------------------------------------------
    def window_base(self) -> int:
        if self.unacked:
            return min(self.unacked)
        if self.pending:
            return self.pending[0][0]
        return self.next_seq

    def pump(self) -> None:
        base = self.window_base()
        while self.pending and self.pending[0][0] < base + self.w:
            seq, payload = self.pending.popleft()
            self.unacked[seq] = payload
            self._send_copies(NewData(self.conn_id, seq, payload))

    def _send_copies(self, m: Message) -> None:
        for _ in range(self.copies):
            self.send(m)

    def write(self, payload: bytes) -> None:
        self.pending.append((self.next_seq, payload))
        self.next_seq += 1
        self.pump()

    def flushed(self) -> bool:
        return not self.pending and not self.unacked

    # -- receiving -------------------------------------------------------------
    def on_message(self, m: Message) -> list:
        """Handles one message from the peer; returns payloads now deliverable in order."""
        self.mark_heard()
        if m.Type == MsgType.MsgAck:
            if m.SeqNum in self.unacked:
                del self.unacked[m.SeqNum]
                self.pump()
            return []
        if m.Type != MsgType.MsgData:
            return []
        new = m.SeqNum >= self.expected and m.SeqNum not in self.rbuf and m.SeqNum < self.expected + self.w
        if new:
            self._send_copies(NewAck(self.conn_id, m.SeqNum))
        else:
            self.send(NewAck(self.conn_id, m.SeqNum))  # a duplicate: acked again, once
        out = []
        if new:
            self.rbuf[m.SeqNum] = m.Payload or b""
            self.recent.append(m.SeqNum)
            self.got_data = True
            while self.expected in self.rbuf:
                out.append(self.rbuf.pop(self.expected))
                self.expected += 1
        return out

    def mark_heard(self) -> None:
        self.heard = True
        self.last_heard = time.monotonic()

    # -- epochs ----------------------------------------------------------------
    def on_epoch(self) -> None:
        """Epoch actions (p1.pdf p.6).  Marks the connection lost once K whole epochs
        have passed without hearing from the peer -- an epoch in which something arrived
        is not silent (the reference's counter: reset on receipt, lost when it exceeds
        EpochLimit, lsp/client_impl.go:236-277, server_impl.go:229-261).  Counting that
        epoch too would declare a loss after K-1 silent epochs, which at 10% read and
        write drops (one heartbeat per epoch lost with p = 0.19) loses an idle
        connection five times as often."""
        if self.lost:
            return
        if self.heard:
            self.silent = 0
            self.heard = False
        else:
            self.silent += 1
        if self.silent >= self.k:
            self.lost = True
            self.lost_reason = (f"{self.silent} silent epochs, peer last heard "
                                f"{1000 * (time.monotonic() - self.last_heard):.0f} ms ago")
            return
        if not self.got_data:
            self._send_copies(NewAck(self.conn_id, 0))
        for seq in sorted(self.unacked):
            self._send_copies(NewData(self.conn_id, seq, self.unacked[seq]))
        for seq in self.recent:
            self._send_copies(NewAck(self.conn_id, seq))


class CopyFilter:
    """Recognises the copies of a datagram before they are parsed.  A peer that sends
    copies (SendCopies) sends them back to back, so a datagram whose bytes equal one of
    the last few from the same address that arrived within `window` seconds is a copy: its
    first instance has been handled, and the receiver only repeats the reply it gave that
    one (the ack of a Data message; nothing for anything else), as the protocol's rule for
    a duplicate says, without parsing it again.  An epoch resend arrives an epoch later
    and is handled in full."""

    def __init__(self, epoch_s: float, depth: int = 8):
        self.window = min(0.01, epoch_s / 20)
        self.depth = depth
        self.seen: dict = {}  # addr -> deque of [raw bytes, arrival time, reply bytes]

    def copy_of(self, addr, raw: bytes, now: float):
        """None for a datagram to handle; for a copy, the reply to repeat (b"": none)."""
        q = self.seen.get(addr)
        if q is None:
            q = self.seen[addr] = collections.deque(maxlen=self.depth)
        for e in q:
            if e[0] == raw and now - e[1] < self.window:
                return e[2]
        q.append([raw, now, b""])
        return None

    def reply(self, addr, raw: bytes, reply: bytes) -> None:
        """Records the reply given to the datagram `raw` just handled."""
        q = self.seen.get(addr)
        if q and q[-1][0] == raw:
            q[-1][2] = reply

    def forget(self, addr) -> None:
        self.seen.pop(addr, None)


class Loop:
    """Event loop thread: UDP readiness, a command queue with a wakeup socket, epochs."""

    def __init__(self, conn, epoch_ms: int, on_datagram, on_command, on_epoch, role: str = "lsp"):
        self.conn = conn
        self.epoch = epoch_ms / 1000.0
        self.role = role
        self.max_late = 0.0   # seconds: the latest any epoch fired after it was due
        self.late_epochs = 0  # epochs that fired more than one epoch late
        self._diag = os.environ.get("LSP_DIAG", "") not in ("", "0")
        self._win_late = 0.0                  # LSP_DIAG: latest epoch of the current 5-s window
        self._win_start = time.monotonic()
        self.on_datagram, self.on_command, self.on_epoch = on_datagram, on_command, on_epoch
        self.cmds = queue.Queue()
        self._r, self._w = socket.socketpair()
        self._r.setblocking(False)
        self.stopped = threading.Event()
        self._stop = False
        self.thread = threading.Thread(target=self._run, daemon=True)

    def start(self) -> None:
        self.thread.start()

    def post(self, *cmd) -> None:
        self.cmds.put(cmd)
        try:
            self._w.send(b"x")
        except OSError:
            pass

    def stop(self) -> None:
        self._stop = True

    def _run(self) -> None:
        sel = selectors.DefaultSelector()
        sel.register(self.conn.sock, selectors.EVENT_READ, "udp")
        sel.register(self._r, selectors.EVENT_READ, "wake")
        next_epoch = time.monotonic() + self.epoch
        try:
            while not self._stop:
                timeout = max(0.0, next_epoch - time.monotonic())
                for key, _ in sel.select(timeout):
                    if key.data == "udp":
                        while True:
                            try:
                                got = self.conn.read_from()
                            except (BlockingIOError, InterruptedError):
                                break
                            except OSError:
                                break
                            if got is not None:
                                self.on_datagram(*got)
                    else:
                        try:
                            while self._r.recv(4096):
                                pass
                        except (BlockingIOError, InterruptedError):
                            pass
                while True:
                    try:
                        cmd = self.cmds.get_nowait()
                    except queue.Empty:
                        break
                    self.on_command(cmd)
                now = time.monotonic()
                if now >= next_epoch:
                    late = now - next_epoch
                    if late > self.max_late:
                        self.max_late = late
                    if late > self.epoch:
                        self.late_epochs += 1
                        if self._diag:
                            print(f"{self.role}[{os.getpid()}]: epoch fired {1000 * late:.0f} ms late "
                                  f"(epoch {1000 * self.epoch:.0f} ms)", file=sys.stderr, flush=True)
                    if self._diag:
                        self._win_late = max(self._win_late, late)
                        if now - self._win_start >= 5.0:
                            print(f"{self.role}[{os.getpid()}]: window max lateness {1000 * self._win_late:.1f} ms, "
                                  f"run max {1000 * self.max_late:.1f} ms, {self.late_epochs} epochs >1 late",
                                  file=sys.stderr, flush=True)
                            self._win_late, self._win_start = 0.0, now
                    next_epoch = now + self.epoch
                    self.on_epoch()
        finally:
            sel.close()
            self._r.close()
            self._w.close()
            self.stopped.set()
