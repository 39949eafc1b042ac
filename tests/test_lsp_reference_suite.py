"""CPU: the reference's LSP test suite, scenario for scenario.

The reference's `lsp{1,2,3,4}_test.go` (src/github.com/cmu440/lsp) hold 44 Go tests. No Go
toolchain exists here or on the GPU box, so each test is restated below under its Go name.
The restatement keeps the Go test's client count, message count, window size, EpochLimit,
drop pattern and assertions, and drives `bitcoin-miner_amd/lsp` through the same API
(NewServer/NewClient/Read/Write/CloseConn/Close and the lspnet drop knobs of staff.go).

Time is scaled. Tests that need epochs to pass run with EpochMillis / EPOCH_DIV (the
500-message lsp4 tests: / EPOCH_DIV_BULK), floored at MIN_EPOCH_MS, and their time limits
(maxEpochs x EpochMillis) scale with it. Tests that
must finish WITHOUT any epoch (TestBasic*, TestSendReceive*) keep their full epochs and
time limits, so a message that needed a resend would still fail them.

  lsp1_test.go:201-335  TestBasic1-9, TestSendReceive1-3, TestRobust1-6  (echo system)
  lsp2_test.go:476-516  TestWindow1-6         (max capacity / scattered, windowTestSystem)
  lsp3_test.go:322-390  TestServerSlowStart1-2, TestServerClose1-2,
                        TestServerCloseConns1-2, TestClientClose1-2     (closeTestSystem)
  lsp4_test.go:444-526  TestServerFastClose1-3, TestServerToClient1-3,
                        TestClientToServer1-3, TestRoundTrip1-3        (syncTestSystem)
"""
from __future__ import annotations

import os
import json
import queue
import random
import socket
import threading
import time

import pytest

import lsp
import lspnet

EPOCH_DIV = 5
MIN_EPOCH_MS = 100


# The 500-message lsp4 tests must move 5 x 500 window-1 round trips while the network is
# on for 2 epochs.  A Python endpoint needs ~2 s for that, so at half the Go test's epoch
# (a 2 s window) they failed about half the time; they keep the Go test's full epochs
# (the 4 s window).  The window tests use the same epochs (lsp2_test: 5 epochs of 0.5 s).
EPOCH_DIV_BULK = 1


# Every scenario runs twice: with each datagram sent once (the protocol exactly as
# specified) and with the programs' three send copies (lsp/endpoint.py, bitcoin.SEND_COPIES).
SEND_COPIES = 1


@pytest.fixture(autouse=True, params=[1, 3], ids=["single_sends", "send_copies3"])
def send_copies(request):
    global SEND_COPIES
    SEND_COPIES = request.param
    yield request.param
    SEND_COPIES = 1


def scaled(epoch_ms: int, div: int = EPOCH_DIV) -> int:
    return max(MIN_EPOCH_MS, epoch_ms // div) if epoch_ms > MIN_EPOCH_MS else epoch_ms


def P(limit: int, millis: int, window: int, scale: bool = True, div: int = EPOCH_DIV) -> lsp.Params:
    return lsp.Params(EpochLimit=limit, EpochMillis=scaled(millis, div) if scale else millis,
                      WindowSize=window, SendCopies=SEND_COPIES)


@pytest.fixture(autouse=True)
def reset_drops():
    lspnet.ResetDropPercent()
    yield
    lspnet.ResetDropPercent()


def free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class Failed(Exception):
    pass


def get(q: queue.Queue, deadline: float, what: str):
    left = deadline - time.monotonic()
    if left <= 0:
        raise Failed(f"timed out waiting for {what}")
    try:
        v = q.get(timeout=left)
    except queue.Empty:
        raise Failed(f"timed out waiting for {what}") from None
    if v is False or isinstance(v, Exception):
        raise Failed(f"{what} failed: {v}")
    return v


def spawn(fn, *args):
    t = threading.Thread(target=fn, args=args, daemon=True)
    t.start()
    return t


# --------------------------------------------------------------------------------------
# lsp1_test.go: echo server, clients write i+rand and expect it echoed (runClient :118-160)
# --------------------------------------------------------------------------------------
def echo_system(num_clients, params, num_msgs, timeout_ms, max_sleep_ms=0, drop=0):
    srv = lsp.NewServer(0, params)
    clients = [lsp.NewClient(f"127.0.0.1:{srv.port}", params) for _ in range(num_clients)]
    lspnet.SetWriteDropPercent(drop)
    exit_ev = threading.Event()
    done: queue.Queue = queue.Queue()

    def rand_sleep():
        if max_sleep_ms > 0:
            time.sleep(random.randrange(max_sleep_ms) / 1000)

    def run_server():
        while not exit_ev.is_set():
            try:
                cid, data = srv.Read()
            except lsp.LSPError:
                return
            rand_sleep()
            try:
                srv.Write(cid, data)
            except lsp.LSPError:
                pass

    def run_client(cli):
        for i in range(num_msgs):
            if exit_ev.is_set():
                return
            wt = random.randrange(100)
            try:
                cli.Write(json.dumps(i + wt).encode())
                got = json.loads(cli.Read())
            except lsp.LSPError as e:
                done.put(e)
                return
            if got != i + wt:
                done.put(Failed(f"client {cli.ConnID()} got {got}, expected {i + wt}"))
                return
            rand_sleep()
        done.put(True)

    spawn(run_server)
    for c in clients:
        spawn(run_client, c)
    deadline = time.monotonic() + timeout_ms / 1000
    try:
        for _ in clients:
            get(done, deadline, "echo client")
    finally:
        exit_ev.set()
        lspnet.ResetDropPercent()
        for c in clients:
            c._closed = True
            c._shutdown()
        srv._closed = True
        srv._loop.stop()
        srv._loop.post("noop")
        srv._conn.close()


# TestBasic*: epochs (2000 ms) longer than the whole test -> no resend may be needed
@pytest.mark.parametrize("name,nc,params,nmsgs,timeout,sleep", [
    ("TestBasic1", 1, (5, 2000, 1), 3, 2000, 0),
    ("TestBasic2", 1, (5, 2000, 1), 50, 2000, 0),
    ("TestBasic3", 2, (5, 2000, 1), 50, 2000, 0),
    ("TestBasic4", 10, (5, 2000, 2), 50, 2000, 0),
    ("TestBasic5", 2, (5, 2000, 2), 500, 2000, 0),
    ("TestBasic6", 10, (5, 2000, 20), 500, 15000, 0),
    ("TestBasic7", 4, (5, 2000, 2), 10, 15000, 100),
    ("TestBasic8", 5, (5, 2000, 10), 10, 15000, 100),
    ("TestBasic9", 2, (5, 2000, 10), 50, 15000, 100),
])
def test_lsp1_basic(name, nc, params, nmsgs, timeout, sleep):
    if nmsgs >= 500 and timeout <= 2000 and SEND_COPIES > 1:
        # TestBasic5's 2 x 500 echoes must fit 2 s of a Python endpoint; three copies are ~4x
        # the datagrams per message, so this variant gets twice the time and twice the epoch
        # (still no resend needed within the test)
        params, timeout = (params[0], 2 * params[1], params[2]), 2 * timeout
    echo_system(nc, P(*params, scale=False), nmsgs, timeout, max_sleep_ms=sleep)


@pytest.mark.parametrize("name,nc,params,nmsgs,timeout,sleep", [
    ("TestSendReceive1", 1, (3, 5000, 1), 6, 5000, 0),
    ("TestSendReceive2", 4, (3, 5000, 1), 6, 5000, 0),
    ("TestSendReceive3", 4, (3, 10000, 1), 6, 10000, 100),
])
def test_lsp1_send_receive_without_epochs(name, nc, params, nmsgs, timeout, sleep):
    echo_system(nc, P(*params, scale=False), nmsgs, timeout, max_sleep_ms=sleep)


# TestRobust*: 20% write drops on both sides, 50 ms epochs as in the reference
@pytest.mark.parametrize("name,nc,params,nmsgs", [
    ("TestRobust1", 1, (20, 50, 1), 10),
    ("TestRobust2", 3, (20, 50, 1), 15),
    ("TestRobust3", 5, (20, 50, 1), 10),
    ("TestRobust4", 1, (20, 50, 2), 10),
    ("TestRobust5", 3, (20, 50, 5), 15),
    ("TestRobust6", 5, (20, 50, 10), 10),
])
def test_lsp1_robust(name, nc, params, nmsgs):
    echo_system(nc, P(*params, scale=False), nmsgs, 15000, drop=20)


# --------------------------------------------------------------------------------------
# lsp2_test.go: sliding window -- at most W unacked messages out (max capacity); in-order
# delivery when the first half of a burst is lost (scattered)
# --------------------------------------------------------------------------------------
class WindowSystem:
    def __init__(self, num_clients, num_msgs, params, max_epochs):
        self.p = params
        self.num_clients = num_clients
        self.num_msgs = num_msgs
        self.timeout = max_epochs * params.EpochMillis / 1000
        self.server = lsp.NewServer(0, params)
        self.clients = {}
        for _ in range(num_clients):
            c = lsp.NewClient(f"127.0.0.1:{self.server.port}", params)
            self.clients[c.ConnID()] = c
        self.server_read = {cid: [] for cid in self.clients}
        self.client_read = {cid: [] for cid in self.clients}
        self.lock = threading.Lock()
        self.server_msgs = [str(random.getrandbits(62)) for _ in range(num_msgs)]
        self.client_msgs = [str(random.getrandbits(62)) for _ in range(num_msgs)]
        self.server_done: queue.Queue = queue.Queue()
        self.client_done: queue.Queue = queue.Queue()
        self.deadline = time.monotonic() + self.timeout

    def stream_to_server(self, cli, msgs):
        try:
            for m in msgs:
                cli.Write(m.encode())
        except lsp.LSPError as e:
            self.client_done.put(e)
            return
        self.client_done.put(True)

    def stream_to_client(self, cid, msgs):
        try:
            for m in msgs:
                self.server.Write(cid, m.encode())
        except lsp.LSPError as e:
            self.server_done.put(e)
            return
        self.server_done.put(True)

    def read_from_server(self, cid, cli, total, *checkpoints):
        cps = list(checkpoints)
        for i in range(total):
            if cps and i == cps[0]:
                self.client_done.put(True)
                cps.pop(0)
            try:
                b = cli.Read()
            except lsp.LSPError as e:
                self.client_done.put(e)
                return
            with self.lock:
                self.client_read[cid].append(b.decode())
        self.client_done.put(True)

    def read_from_all_clients(self, total, *checkpoints):
        cps = list(checkpoints)
        for i in range(total):
            if cps and i == cps[0]:
                self.server_done.put(True)
                cps.pop(0)
            try:
                cid, b = self.server.Read()
            except lsp.LSPError as e:
                self.server_done.put(e)
                return
            with self.lock:
                if cid not in self.server_read:
                    self.server_done.put(Failed(f"unknown client {cid}"))
                    return
                self.server_read[cid].append(b.decode())
        self.server_done.put(True)

    def wait_server(self):
        get(self.server_done, self.deadline, "server")

    def wait_clients(self):
        for _ in range(self.num_clients):
            get(self.client_done, self.deadline, "clients")

    def check_server_read(self, sent):
        with self.lock:
            for cid, got in self.server_read.items():
                assert got == sent, f"server read {got} from client {cid}, expected {sent}"

    def check_client_read(self, sent):
        with self.lock:
            for cid, got in self.client_read.items():
                assert got == sent, f"client {cid} read {got}, expected {sent}"

    def run_max_capacity(self):  # lsp2_test.go:316-383
        w, n = self.p.WindowSize, self.num_msgs
        assert n > w
        lspnet.SetServerWriteDropPercent(100)  # no acks from the server
        spawn(self.read_from_all_clients, self.num_clients * n, w * self.num_clients)
        for cid, cli in self.clients.items():
            spawn(self.stream_to_server, cli, self.client_msgs)
        self.wait_clients()
        self.wait_server()
        time.sleep(0.05)
        self.check_server_read(self.client_msgs[:w])
        lspnet.SetServerWriteDropPercent(0)
        self.wait_server()
        time.sleep(0.05)
        self.check_server_read(self.client_msgs)

        lspnet.SetClientWriteDropPercent(100)  # no acks from the clients
        for cid, cli in self.clients.items():
            spawn(self.read_from_server, cid, cli, n, w)
            spawn(self.stream_to_client, cid, self.server_msgs)
        for _ in range(self.num_clients):
            self.wait_server()
        self.wait_clients()
        time.sleep(0.05)
        self.check_client_read(self.server_msgs[:w])
        lspnet.SetClientWriteDropPercent(0)
        self.wait_clients()
        time.sleep(0.05)
        self.check_client_read(self.server_msgs)

    def run_scattered(self):  # lsp2_test.go:385-474
        w, n = self.p.WindowSize, self.num_msgs
        assert w > n
        lspnet.SetClientWriteDropPercent(100)  # first half of every client's burst is lost
        for cli in self.clients.values():
            spawn(self.stream_to_server, cli, self.client_msgs[: n // 2])
        self.wait_clients()
        lspnet.SetClientWriteDropPercent(0)
        for cli in self.clients.values():
            spawn(self.stream_to_server, cli, self.client_msgs[n // 2:])
        self.wait_clients()
        spawn(self.read_from_all_clients, n * self.num_clients, 0)
        self.wait_server()
        time.sleep(0.05)
        self.wait_server()
        time.sleep(0.05)
        self.check_server_read(self.client_msgs)

        lspnet.SetServerWriteDropPercent(100)
        for cid in self.clients:
            spawn(self.stream_to_client, cid, self.server_msgs[: n // 2])
        for _ in self.clients:
            self.wait_server()
        lspnet.SetServerWriteDropPercent(0)
        for cid in self.clients:
            spawn(self.stream_to_client, cid, self.server_msgs[n // 2:])
        for _ in self.clients:
            self.wait_server()
        for cid, cli in self.clients.items():
            spawn(self.read_from_server, cid, cli, n, 0)
        self.wait_clients()
        time.sleep(0.05)
        self.wait_clients()
        time.sleep(0.05)
        self.check_client_read(self.server_msgs)

    def teardown(self):
        lspnet.ResetDropPercent()
        for c in self.clients.values():
            c._closed = True
            c._shutdown()
        self.server._closed = True
        self.server._loop.stop()
        self.server._loop.post("noop")
        self.server._conn.close()


@pytest.mark.parametrize("name,mode,nc,nmsgs,params", [
    ("TestWindow1", "max", 1, 10, (3, 500, 5)),
    ("TestWindow2", "max", 5, 25, (3, 500, 10)),
    ("TestWindow3", "max", 10, 25, (3, 500, 10)),
    ("TestWindow4", "scattered", 1, 10, (3, 1000, 20)),
    ("TestWindow5", "scattered", 5, 10, (3, 1000, 20)),
    ("TestWindow6", "scattered", 10, 10, (3, 1000, 20)),
])
def test_lsp2_window(name, mode, nc, nmsgs, params):
    # the "max" runs wait out two resend epochs inside a 5-epoch limit with up to 10
    # clients' threads; at EPOCH_DIV's 100 ms epochs a scheduling hiccup of the Python
    # threads under a loaded suite is a whole epoch, so these run at the Go test's epochs
    ts = WindowSystem(nc, nmsgs, P(*params, div=EPOCH_DIV_BULK), max_epochs=5)
    try:
        ts.run_max_capacity() if mode == "max" else ts.run_scattered()
    finally:
        ts.teardown()


# --------------------------------------------------------------------------------------
# lsp3_test.go: Close/CloseConn semantics and a server that starts after its clients
# --------------------------------------------------------------------------------------
def close_system(mode, num_clients, max_epochs, params, num_msgs=10, delay_epochs=3):
    port = free_port()
    clients: list = [None] * num_clients
    server_box: list = [None]
    server_done: queue.Queue = queue.Queue()
    client_done: queue.Queue = queue.Queue()
    exit_ev = threading.Event()

    def build_server():  # lsp3_test.go:183-253
        if mode == "slowstart":
            time.sleep(delay_epochs * params.EpochMillis / 1000)
        try:
            srv = lsp.NewServer(port, params)
        except OSError as e:
            server_done.put(e)
            return
        server_box[0] = srv
        num_dead = num_echo = 0
        while not exit_ev.is_set():
            try:
                cid, data = srv.Read()
            except lsp.LSPError:
                num_dead += 1
                if mode == "clientclose" and num_dead == num_clients:
                    server_done.put(True)
                    try:
                        srv.Close()
                    except lsp.LSPError:
                        pass
                    return
                continue
            try:
                srv.Write(cid, data)
            except lsp.LSPError as e:
                server_done.put(e)
                return
            num_echo += 1
            if num_echo == num_clients * num_msgs:
                if mode == "serverclose":
                    try:
                        srv.Close()
                    except lsp.LSPError:
                        pass
                    server_done.put(True)
                    return
                if mode == "closeconns":
                    for c in clients:
                        srv.CloseConn(c.ConnID())
                    server_done.put(True)
                    return
                if mode != "clientclose":
                    server_done.put(True)
                    srv.CloseConn(cid)
                    return

    def build_client(i):  # lsp3_test.go:256-320
        try:
            cli = lsp.NewClient(f"127.0.0.1:{port}", params)
        except lsp.LSPError as e:
            client_done.put(e)
            return
        clients[i] = cli
        for m in range(num_msgs):
            if exit_ev.is_set():
                return
            tv = m * 100 + random.randrange(100)
            try:
                cli.Write(json.dumps(tv).encode())
                got = json.loads(cli.Read())
            except lsp.LSPError as e:
                client_done.put(Failed(f"client {i} lost the server after {m} messages: {e}"))
                cli.Close()
                return
            if got != tv:
                client_done.put(Failed(f"client {i} got {got}, expected {tv}"))
                cli.Close()
                return
        if mode == "clientclose":
            cli.Close()
            client_done.put(True)
        elif mode in ("closeconns", "serverclose"):
            try:
                cli.Read()
            except lsp.LSPError:
                client_done.put(True)  # server termination detected
                cli.Close()
                return
            client_done.put(Failed(f"client {i} received unexpected data"))
            cli.Close()
        else:
            cli.Close()
            client_done.put(True)

    spawn(build_server)
    for i in range(num_clients):
        spawn(build_client, i)
    deadline = time.monotonic() + max_epochs * params.EpochMillis / 1000
    try:
        if mode == "clientclose":
            get(server_done, deadline, "server")
            for _ in range(num_clients):
                get(client_done, deadline, "client")
        else:
            for _ in range(num_clients):
                get(client_done, deadline, "client")
            get(server_done, deadline, "server")
    finally:
        exit_ev.set()
        srv = server_box[0]
        if srv is not None and not srv._closed:
            srv._closed = True
            srv._loop.stop()
            srv._loop.post("noop")
            srv._conn.close()


@pytest.mark.parametrize("name,mode,nc,max_epochs,params", [
    ("TestServerSlowStart1", "slowstart", 1, 5, (5, 500, 1)),
    ("TestServerSlowStart2", "slowstart", 3, 5, (5, 500, 1)),
    ("TestServerClose1", "serverclose", 1, 10, (5, 500, 1)),
    ("TestServerClose2", "serverclose", 3, 5, (2, 500, 1)),
    ("TestServerCloseConns1", "closeconns", 1, 10, (5, 500, 1)),
    ("TestServerCloseConns2", "closeconns", 3, 5, (2, 500, 1)),
    ("TestClientClose1", "clientclose", 2, 10, (5, 500, 1)),
    ("TestClientClose2", "clientclose", 3, 15, (5, 500, 1)),
])
def test_lsp3_close(name, mode, nc, max_epochs, params):
    close_system(mode, nc, max_epochs, P(*params))


# --------------------------------------------------------------------------------------
# lsp4_test.go: messages buffered while the network is off (100% write drops on every
# role), fast Close calls that can only finish once the network comes back
# --------------------------------------------------------------------------------------
class SyncSystem:
    def __init__(self, num_clients, num_msgs, mode, params, max_epochs):
        self.nc, self.n, self.mode, self.p = num_clients, num_msgs, mode, params
        self.data = [[random.getrandbits(62) for _ in range(num_msgs)] for _ in range(num_clients)]
        self.port = free_port()
        self.clients: list = [None] * num_clients
        self.client_of: dict = {}
        self.lock = threading.Lock()
        self.server = None
        self.c2m: queue.Queue = queue.Queue()
        self.s2m: queue.Queue = queue.Queue()
        self.n2m: queue.Queue = queue.Queue()
        # one command queue per client: Go's unbuffered masterToClientChan hands each
        # client exactly one token per signal (a client cannot take two)
        self.m2c = [queue.Queue() for _ in range(num_clients)]
        self.m2s: queue.Queue = queue.Queue()
        self.m2n: queue.Queue = queue.Queue()
        self.errs: queue.Queue = queue.Queue()
        self.exit = threading.Event()
        self.deadline = time.monotonic() + max_epochs * params.EpochMillis / 1000

    def _wait_cmd(self, q):
        while not self.exit.is_set():
            try:
                return q.get(timeout=0.05)
            except queue.Empty:
                pass
        raise SystemExit

    def run_network(self):  # lsp4_test.go:110-135
        lspnet.SetWriteDropPercent(0)
        try:
            while True:
                self._wait_cmd(self.m2n)
                lspnet.SetWriteDropPercent(100)
                self.n2m.put(True)
                self._wait_cmd(self.m2n)
                lspnet.SetWriteDropPercent(0)
                self.n2m.put(True)
                time.sleep(2 * self.p.EpochMillis / 1000)
        except SystemExit:
            return

    def run_server(self):  # lsp4_test.go:137-225
        try:
            self.server = srv = lsp.NewServer(self.port, self.p)
            self.s2m.put(True)
            if self.mode != "s2c":
                self._wait_cmd(self.m2s)
                rcvd = [0] * self.nc
                for _ in range(self.n * self.nc):
                    cid, b = srv.Read()
                    v = json.loads(b)
                    with self.lock:
                        ci = self.client_of.get(cid)
                    if ci is None:
                        raise Failed(f"server read from unknown client {cid}")
                    if rcvd[ci] >= self.n:
                        raise Failed(f"too many messages from client {cid}")
                    if v != self.data[ci][rcvd[ci]]:
                        raise Failed(f"server got {v} as #{rcvd[ci]} of client {ci}")
                    rcvd[ci] += 1
                self.s2m.put(True)
            if self.mode != "c2s":
                self._wait_cmd(self.m2s)
                sent = [0] * self.nc
                nsent = 0
                while nsent < self.n * self.nc:
                    ci = random.randrange(self.nc)
                    if sent[ci] >= self.n:
                        continue
                    srv.Write(self.clients[ci].ConnID(), json.dumps(self.data[ci][sent[ci]]).encode())
                    sent[ci] += 1
                    nsent += 1
                self.s2m.put(True)
            self._wait_cmd(self.m2s)
            try:
                srv.Close()
            except lsp.LSPError:
                pass
            self.s2m.put(True)
        except SystemExit:
            return
        except Exception as e:  # noqa: BLE001 -- reported to the master like errChan
            self.errs.put(e)

    def run_client(self, i):  # lsp4_test.go:227-300
        try:
            cli = lsp.NewClient(f"127.0.0.1:{self.port}", self.p)
            self.clients[i] = cli
            with self.lock:
                self.client_of[cli.ConnID()] = i
            self.c2m.put(True)
            if self.mode != "s2c":
                self._wait_cmd(self.m2c[i])
                for v in self.data[i]:
                    cli.Write(json.dumps(v).encode())
                self.c2m.put(True)
            if self.mode != "c2s":
                self._wait_cmd(self.m2c[i])
                for k in range(self.n):
                    v = json.loads(cli.Read())
                    if v != self.data[i][k]:
                        raise Failed(f"client {i} got {v} as #{k}, expected {self.data[i][k]}")
                self.c2m.put(True)
            self._wait_cmd(self.m2c[i])
            cli.Close()
            self.c2m.put(True)
        except SystemExit:
            return
        except Exception as e:  # noqa: BLE001
            self.errs.put(e)

    def _wait(self, q, what):
        while True:
            if not self.errs.empty():
                raise Failed(f"{what}: {self.errs.get()}")
            if time.monotonic() > self.deadline:
                raise Failed(f"timed out waiting for {what}")
            try:
                q.get(timeout=0.02)
                return
            except queue.Empty:
                pass

    def wait_server(self):
        self._wait(self.s2m, "server")

    def wait_clients(self):
        for _ in range(self.nc):
            self._wait(self.c2m, "clients")

    def signal_server(self):
        self.m2s.put(True)

    def signal_clients(self):
        for q in self.m2c:
            q.put(True)

    def toggle(self):
        self.m2n.put(True)
        self._wait(self.n2m, "network")

    def master(self):  # lsp4_test.go:355-425
        spawn(self.run_network)
        spawn(self.run_server)
        self.wait_server()  # server first: clients dial a fixed port
        for i in range(self.nc):
            spawn(self.run_client, i)
        self.wait_clients()
        self.toggle()  # network off
        if self.mode != "s2c":
            self.signal_clients()  # clients write into the dead network
            self.wait_clients()
        if self.mode == "c2s":
            self.signal_clients()  # fast close of the clients: cannot finish yet
        if self.mode != "s2c":
            self.toggle()  # network on
            if self.mode == "c2s":
                self.wait_clients()  # the clients' Close calls completed
            self.toggle()  # off
            self.signal_server()  # server reads what was buffered
            self.wait_server()
        if self.mode != "c2s":
            self.signal_server()  # server writes into the dead network
            self.wait_server()
        if self.mode != "roundtrip":
            self.signal_server()  # fast close of the server
        if self.mode != "c2s":
            self.toggle()  # on
            if self.mode != "roundtrip":
                self.wait_server()  # its Close completed
            self.toggle()  # off
            self.signal_clients()  # clients read what was buffered
            self.wait_clients()
            self.signal_clients()  # clients close
            self.wait_clients()
        if self.mode == "roundtrip":
            self.signal_server()
            self.wait_server()

    def teardown(self):
        self.exit.set()
        lspnet.ResetDropPercent()
        for c in self.clients:
            if c is not None and not c._closed:
                c._closed = True
                c._shutdown()
        srv = self.server
        if srv is not None and not srv._closed:
            srv._closed = True
            srv._loop.stop()
            srv._loop.post("noop")
            srv._conn.close()


@pytest.mark.parametrize("name,nc,nmsgs,mode,params,max_epochs", [
    ("TestServerFastClose1", 1, 10, "fastclose", (5, 500, 1), 12),
    ("TestServerFastClose2", 3, 10, "fastclose", (5, 500, 1), 12),
    ("TestServerFastClose3", 5, 500, "fastclose", (5, 2000, 1), 20),
    ("TestServerToClient1", 1, 10, "s2c", (5, 500, 1), 12),
    ("TestServerToClient2", 3, 10, "s2c", (5, 500, 1), 12),
    ("TestServerToClient3", 5, 500, "s2c", (5, 2000, 1), 20),
    ("TestClientToServer1", 1, 10, "c2s", (5, 500, 1), 12),
    ("TestClientToServer2", 3, 10, "c2s", (5, 500, 1), 12),
    ("TestClientToServer3", 5, 500, "c2s", (5, 2000, 1), 20),
    ("TestRoundTrip1", 1, 10, "roundtrip", (5, 500, 1), 12),
    ("TestRoundTrip2", 3, 10, "roundtrip", (5, 500, 1), 12),
    ("TestRoundTrip3", 5, 500, "roundtrip", (5, 2000, 1), 20),
])
def test_lsp4_sync(name, nc, nmsgs, mode, params, max_epochs):
    # "fastclose" moves data both ways like RoundTrip, but issues the server's Close while
    # the network is still off (lsp4_test.go:395-397)
    div = EPOCH_DIV_BULK if nmsgs >= 500 else EPOCH_DIV
    if nmsgs >= 500 and SEND_COPIES > 1:
        # 5 x 500 window-1 round trips must fit the 2 epochs the network is on; with three
        # copies a Python endpoint sends and reads ~4x the datagrams per message, so under a
        # loaded suite these runs get twice the Go test's epochs (the scenario is the same)
        params = (params[0], 2 * params[1], params[2])
    ts = SyncSystem(nc, nmsgs, mode, P(*params, div=div), max_epochs)
    try:
        ts.master()
    finally:
        ts.teardown()
