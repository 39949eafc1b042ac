"""lspnet -- UDP wrapper with per-role drop injection (plumbing for the §8(f) rows).

Mirrors src/github.com/cmu440/lspnet of the reference:
  * net.go:37-76   ListenUDP (server role) / DialUDP (client role) register the role of a
                   connection so drops can be injected per role
  * conn.go:34-113 Read / ReadFromUDP / Write / WriteToUDP, each applying the role's
                   read or write drop percentage (dropIt, conn.go:115-117)
  * staff.go:14-48 Set{Client,Server}{Read,Write}DropPercent, ResetDropPercent,
                   EnableDebugLogs
Separate processes (BASELINE config 5) take the same knobs from the environment:
LSPNET_CLIENT_READ_DROP, LSPNET_CLIENT_WRITE_DROP, LSPNET_SERVER_READ_DROP,
LSPNET_SERVER_WRITE_DROP (percent, 0-100).
"""
from __future__ import annotations

import os
import random
import socket
import sys

_drop = {
    ("client", "read"): int(os.environ.get("LSPNET_CLIENT_READ_DROP", "0")),
    ("client", "write"): int(os.environ.get("LSPNET_CLIENT_WRITE_DROP", "0")),
    ("server", "read"): int(os.environ.get("LSPNET_SERVER_READ_DROP", "0")),
    ("server", "write"): int(os.environ.get("LSPNET_SERVER_WRITE_DROP", "0")),
}
_debug = False
_rng = random.Random()
MAX_DATAGRAM = 2000  # the reference reads into 2000-byte buffers (conn.go:35)


def SetClientReadDropPercent(p: int) -> None:
    _drop[("client", "read")] = int(p)


def SetClientWriteDropPercent(p: int) -> None:
    _drop[("client", "write")] = int(p)


def SetServerReadDropPercent(p: int) -> None:
    _drop[("server", "read")] = int(p)


def SetServerWriteDropPercent(p: int) -> None:
    _drop[("server", "write")] = int(p)


def SetReadDropPercent(p: int) -> None:
    SetClientReadDropPercent(p)
    SetServerReadDropPercent(p)


def SetWriteDropPercent(p: int) -> None:
    SetClientWriteDropPercent(p)
    SetServerWriteDropPercent(p)


def ResetDropPercent() -> None:
    """staff.go:44-48: all four drop percentages back to 0."""
    SetReadDropPercent(0)
    SetWriteDropPercent(0)


def EnableDebugLogs(on: bool) -> None:
    global _debug
    _debug = bool(on)


def _drop_it(role: str, op: str) -> bool:
    p = _drop[(role, op)]
    return p > 0 and _rng.randrange(100) < p


class UDPConn:
    """A UDP socket tagged with its role ("client" or "server")."""

    def __init__(self, sock: socket.socket, role: str, peer=None):
        self.sock = sock
        self.role = role
        self.peer = peer

    def fileno(self) -> int:
        return self.sock.fileno()

    def local_addr(self):
        return self.sock.getsockname()

    def read_from(self):
        """One datagram (payload, addr), or None when the drop injector ate it."""
        data, addr = self.sock.recvfrom(MAX_DATAGRAM)
        if _drop_it(self.role, "read"):
            if _debug:
                print(f"lspnet: {self.role} DROPPED read {data[:60]!r}", file=sys.stderr)
            return None
        return data, addr

    def write_to(self, data: bytes, addr=None) -> None:
        if _drop_it(self.role, "write"):
            if _debug:
                print(f"lspnet: {self.role} DROPPED write {data[:60]!r}", file=sys.stderr)
            return
        try:
            self.sock.sendto(data, addr or self.peer)
        except OSError:
            pass  # UDP: a failed send is a lost datagram

    def close(self) -> None:
        self.sock.close()


def resolve(hostport: str):
    host, port = hostport.rsplit(":", 1)
    return (socket.gethostbyname(host or "127.0.0.1"), int(port))


# Receive buffer asked of the kernel (it grants at most net.core.rmem_max): a server's
# socket takes bursts from every connection at once -- each epoch's resends and re-acks,
# and a window of Data messages in send copies -- and the default ~200 KB holds only a
# couple of hundred small datagrams.
RCVBUF = 4 << 20


def _udp_socket() -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, RCVBUF)
    except OSError:
        pass
    return s


def ListenUDP(port: int, host: str = "0.0.0.0") -> UDPConn:
    s = _udp_socket()
    s.bind((host, int(port)))
    s.setblocking(False)
    return UDPConn(s, "server")


def DialUDP(hostport: str) -> UDPConn:
    peer = resolve(hostport)
    s = _udp_socket()
    s.bind(("0.0.0.0", 0))
    s.setblocking(False)
    return UDPConn(s, "client", peer)
