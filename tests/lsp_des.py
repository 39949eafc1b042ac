"""Discrete-event model of the whole system -- server, miners, clients -- over the real LSP
state machine, for sizing the server's jobs on lossy links.

Test infrastructure (tests/test_scheduler_sim.py, tools/des_sweep.py), not product code.
What is real and what is modelled:
  * REAL: each connection end is lsp.endpoint.ConnState (window, in-order delivery, acks,
    epoch resends and re-acks, loss after EpochLimit silent epochs, send copies) behind
    lsp.endpoint.CopyFilter, the connect
    handshake follows lsp/client.py and lsp/server.py, and the server is
    bitcoin.server.ServerCore over its Scheduler -- the code the server program runs;
  * MODELLED: the network (each datagram is dropped at the sender with the role's write
    probability and at the receiver with its read probability, as lspnet does, and
    otherwise arrives after `latency`); each endpoint's epoch timer (every epoch from its
    start, like lsp.endpoint.Loop); the GPU (a miner's job takes work/rate plus a fixed
    per-call overhead; miners that share a GPU share it equally, work-conserving); a
    killed miner (its endpoint goes silent at once).
Clocks are simulated seconds; a run of config 5 takes well under a second of CPU.
"""
from __future__ import annotations

import heapq
import itertools
import random

import lsp
from bitcoin import MsgType as BMsg
from bitcoin import NewJoin, NewRequest, NewResult, marshal, unmarshal
from bitcoin import server as bserver
from lsp.endpoint import ConnState, CopyFilter
from lsp.message import MsgType, NewAck, NewConnect


class Sim:
    def __init__(self, seed: int = 1):
        self.t = 0.0
        self.q: list = []
        self._seq = itertools.count()
        self.rng = random.Random(seed)

    def at(self, t: float, fn, *args) -> None:
        heapq.heappush(self.q, (t, next(self._seq), fn, args))

    def run(self, until: float = 1e9, stop=lambda: False) -> None:
        while self.q and not stop():
            t, _, fn, args = heapq.heappop(self.q)
            if t > until:
                heapq.heappush(self.q, (t, 0, fn, args))
                return
            self.t = t
            fn(*args)


class Net:
    """Datagrams between endpoints: lspnet's per-role write (sender) and read (receiver)
    drop percentages, then a fixed latency."""

    def __init__(self, sim: Sim, latency: float = 0.0002):
        self.sim = sim
        self.latency = latency
        self.datagrams = 0

    def send(self, src, dst, msg) -> None:
        if src.dead:
            return
        self.datagrams += 1
        if self.sim.rng.random() < src.wdrop:
            return
        self.sim.at(self.sim.t + self.latency, self._arrive, src, dst, msg)

    def _arrive(self, src, dst, msg) -> None:
        if dst.dead or self.sim.rng.random() < dst.rdrop:
            return
        # lsp.endpoint.CopyFilter: a copy only repeats its first instance's reply
        raw = (msg.Type, msg.ConnID, msg.SeqNum, msg.Payload)
        again = dst.copies.copy_of(id(src), raw, self.sim.t)
        if again is not None:
            if again:
                self.send(dst, src, again)
            return
        dst.on_datagram(src, msg)
        if msg.Type == MsgType.MsgData:
            dst.copies.reply(id(src), raw, NewAck(msg.ConnID, msg.SeqNum))


class Endpoint:
    def __init__(self, sim: Sim, net: Net, params, rdrop: float, wdrop: float):
        self.sim, self.net, self.p = sim, net, params
        self.rdrop, self.wdrop = rdrop, wdrop
        self.dead = False
        self.epoch = params.EpochMillis / 1000.0
        self.copies = CopyFilter(self.epoch)
        sim.at(sim.t + self.epoch, self._epoch)

    def _epoch(self) -> None:
        if self.dead:
            return
        self.on_epoch()
        self.sim.at(self.sim.t + self.epoch, self._epoch)


class ServerEP(Endpoint):
    """lsp/server.py's connection table and loop actions; `app` gets on_payload(conn, p)
    and on_lost(conn, reason)."""

    def __init__(self, sim, net, params, rdrop, wdrop):
        super().__init__(sim, net, params, rdrop, wdrop)
        self.conns: dict[int, ConnState] = {}
        self.peer: dict[int, Endpoint] = {}
        self.id_of: dict[int, int] = {}
        self.next_id = 1
        self.app = None

    def on_datagram(self, src, m) -> None:
        if m.Type == MsgType.MsgConnect:
            cid = self.id_of.get(id(src))
            if cid is None:
                cid = self.next_id
                self.next_id += 1
                self.id_of[id(src)] = cid
                self.peer[cid] = src
                self.conns[cid] = ConnState(cid, self.p.WindowSize, self.p.EpochLimit,
                                            lambda x, d=src: self.net.send(self, d, x), self.p.SendCopies)
            st = self.conns.get(cid)
            if st is not None:
                st.mark_heard()
                for _ in range(max(1, self.p.SendCopies)):
                    self.net.send(self, src, NewAck(cid, 0))
            return
        st = self.conns.get(m.ConnID)
        if st is None or self.peer.get(m.ConnID) is not src:
            return
        for payload in st.on_message(m):
            self.app.on_payload(m.ConnID, payload)
        self._reap()

    def on_epoch(self) -> None:
        for st in list(self.conns.values()):
            st.on_epoch()
        self._reap()

    def _reap(self) -> None:
        for cid, st in list(self.conns.items()):
            if st.lost or (st.closing and st.flushed()):
                why = st.lost_reason if st.lost else "closed"
                del self.conns[cid]
                self.id_of.pop(id(self.peer.pop(cid)), None)
                self.app.on_lost(cid, f"connection {cid} {'lost (' + why + ')' if st.lost else why}")

    def write(self, cid: int, payload: bytes) -> None:
        st = self.conns.get(cid)
        if st is None or st.lost or st.closing:
            raise lsp.LSPError(f"connection {cid} is lost or closed", cid)
        st.write(payload)

    def close_conn(self, cid: int) -> None:
        st = self.conns.get(cid)
        if st is None:
            raise lsp.LSPError(f"no connection {cid}", cid)
        st.closing = True
        self.sim.at(self.sim.t, self._reap)


class ClientEP(Endpoint):
    """lsp/client.py: Connect (resent every epoch, EpochLimit tries), then one ConnState;
    `app` gets on_connected(), on_payload(p), on_lost()."""

    def __init__(self, sim, net, params, rdrop, wdrop, server: ServerEP, app):
        super().__init__(sim, net, params, rdrop, wdrop)
        self.server, self.app = server, app
        self.st: ConnState | None = None
        self.connect_silent = 0
        self.closing = False
        self._connect()

    def _connect(self) -> None:
        for _ in range(max(1, self.p.SendCopies)):
            self.net.send(self, self.server, NewConnect())

    def on_datagram(self, src, m) -> None:
        if src is not self.server:
            return
        if self.st is None:
            if m.Type == MsgType.MsgAck and m.SeqNum == 0 and m.ConnID > 0:
                self.st = ConnState(m.ConnID, self.p.WindowSize, self.p.EpochLimit,
                                    lambda x: self.net.send(self, self.server, x), self.p.SendCopies)
                self.app.on_connected()
            return
        if m.ConnID != self.st.conn_id:
            return
        for payload in self.st.on_message(m):
            self.app.on_payload(payload)
        self._check_close()

    def on_epoch(self) -> None:
        if self.st is None:
            self.connect_silent += 1
            if self.connect_silent >= self.p.EpochLimit:
                self.dead = True
                self.app.on_lost()
            else:
                self._connect()
            return
        was = self.st.lost
        self.st.on_epoch()
        if self.st.lost and not was:
            self.dead = True
            self.app.on_lost()
        self._check_close()

    def write(self, payload: bytes) -> None:
        if self.st is not None and not self.st.lost:
            self.st.write(payload)

    def close(self) -> None:
        self.closing = True
        if self.st is not None:
            self.st.closing = True
        self._check_close()

    def _check_close(self) -> None:
        if self.closing and (self.st is None or self.st.flushed() or self.st.lost):
            self.dead = True  # the program exits


class GPU:
    """Processor sharing among the miners' running jobs (one job per miner at a time)."""

    def __init__(self, sim: Sim, rate: float):
        self.sim, self.rate = sim, rate
        self.active: dict = {}  # miner -> [remaining work, on_done]
        self.t = 0.0
        self.version = 0
        self.busy = 0.0  # seconds with at least one job running

    def _advance(self) -> None:
        dt = self.sim.t - self.t
        if self.active and dt > 0:
            share = self.rate / len(self.active)
            for v in self.active.values():
                v[0] -= share * dt
            self.busy += dt
        self.t = self.sim.t

    def _arm(self) -> None:
        self.version += 1
        if not self.active:
            return
        share = self.rate / len(self.active)
        m, v = min(self.active.items(), key=lambda kv: kv[1][0])
        self.sim.at(self.sim.t + max(0.0, v[0]) / share, self._finish, self.version)

    def run(self, miner, work: float, on_done) -> None:
        self._advance()
        self.active[miner] = [work, on_done]
        self._arm()

    def cancel(self, miner) -> None:
        self._advance()
        self.active.pop(miner, None)
        self._arm()

    def _finish(self, version: int) -> None:
        if version != self.version:
            return
        self._advance()
        # finished: less than a nanosecond of work left (relative, so any rate converges)
        eps = 1e-9 * self.rate / max(1, len(self.active))
        done = [m for m, v in self.active.items() if v[0] <= eps]
        for m in done:
            cb = self.active.pop(m)[1]
            cb()
        self._arm()


class Miner:
    """bitcoin/miner.py: Join, then Read Request -> compute -> Write Result, in order."""

    def __init__(self, sim: Sim, gpu: GPU, overhead: float, log: list, name: int):
        self.sim, self.gpu, self.overhead, self.log, self.name = sim, gpu, overhead, log, name
        self.ep: ClientEP | None = None
        self.queue: list = []
        self.running = None

    def on_connected(self) -> None:
        self.ep.write(marshal(NewJoin()))

    def on_payload(self, p: bytes) -> None:
        m = unmarshal(p)
        if m.Type == BMsg.Request:
            self.queue.append(m)
            self._next()

    def on_lost(self) -> None:
        self.kill()

    def _next(self) -> None:
        if self.running is not None or not self.queue or self.ep.dead:
            return
        m = self.running = self.queue.pop(0)
        start = self.sim.t
        n = m.Upper - m.Lower + 1
        self.gpu.run(self, n + self.overhead * self.gpu.rate,
                     lambda: self._done(m, start, n))

    def _done(self, m, start: float, n: int) -> None:
        self.running = None
        self.log.append((self.name, m.Data, m.Lower, m.Upper, start, self.sim.t))
        self.ep.write(marshal(NewResult((m.Lower * 2654435761) % (1 << 64), m.Lower)))
        self._next()

    def kill(self) -> None:
        self.ep.dead = True
        self.gpu.cancel(self)
        self.running = None
        self.queue.clear()


class Client:
    def __init__(self, sim: Sim, data: str, lower: int, upper: int):
        self.sim, self.data, self.lower, self.upper = sim, data, lower, upper
        self.ep: ClientEP | None = None
        self.done_at = None
        self.result = None
        self.disconnected = False

    def on_connected(self) -> None:
        self.ep.write(marshal(NewRequest(self.data, self.lower, self.upper)))

    def on_payload(self, p: bytes) -> None:
        m = unmarshal(p)
        if m.Type == BMsg.Result and self.done_at is None:
            self.done_at = self.sim.t
            self.result = (m.Hash, m.Nonce)
            self.ep.close()

    def on_lost(self) -> None:
        if self.done_at is None:
            self.done_at = self.sim.t
            self.disconnected = True


class ServerApp:
    """ServerCore plus its wake-up timer (serve()'s read_until)."""

    def __init__(self, sim: Sim, ep: ServerEP, sched):
        self.sim = sim
        sched.clock = lambda: sim.t
        self.core = bserver.ServerCore(sched, ep.write, ep.close_conn)
        self._armed = None
        self.arrivals: dict = {}  # Data -> when the server read its Request


    def _rearm(self) -> None:
        w = self.core.sched.next_wakeup()
        if w is not None and (self._armed is None or w < self._armed or self._armed < self.sim.t):
            self._armed = max(w, self.sim.t)
            self.sim.at(self._armed, self._timer, self._armed)

    def _timer(self, when: float) -> None:
        if when != self._armed:
            return
        self._armed = None
        self.core.on_timer()
        self._rearm()

    def on_payload(self, conn: int, p: bytes) -> None:
        m = unmarshal(p)
        if m.Type == BMsg.Request:
            self.arrivals.setdefault(m.Data, self.sim.t)
        self.core.on_payload(conn, p)
        self._rearm()

    def on_lost(self, conn: int, reason: str) -> None:
        self.core.on_lost(conn, reason)
        self._rearm()


def run_system(sched, gpus: list[float], miners_per_gpu: int = 1, requests=(), params=None,
               drop: float = 0.10, latency: float = 0.0002, overhead: float = 0.002,
               kill: tuple | None = None, client_start: float = 5.0, seed: int = 1,
               horizon: float = 3600.0, kills: list | None = None) -> dict:
    """Runs one system to completion.  gpus: rate of each GPU (nonces/s); requests:
    (data, lower, upper) per client, all started at `client_start` (the miners start at 0
    and join first, as tools/system_bench.py starts them); kill: (time after client_start,
    miner index) or None, kills: a list of them.  Returns timings and the GPU work log."""
    kills = list(kills or []) + ([kill] if kill is not None else [])
    params = params or lsp.NewParams()
    sim = Sim(seed)
    net = Net(sim, latency)
    srv = ServerEP(sim, net, params, drop, drop)
    app = ServerApp(sim, srv, sched)
    srv.app = app
    log: list = []
    dev = [GPU(sim, r) for r in gpus]
    miners = []
    for g in dev:
        for _ in range(miners_per_gpu):
            mi = Miner(sim, g, overhead, log, len(miners))
            sim.at(sim.rng.uniform(0, 0.05), _start_client, sim, net, params, drop, srv, mi)
            miners.append(mi)
    clients = []
    for data, lo, hi in requests:
        c = Client(sim, data, lo, hi)
        sim.at(client_start + sim.rng.uniform(0, 0.05), _start_client, sim, net, params, drop, srv, c)
        clients.append(c)
    for t, i in kills:
        sim.at(client_start + t, miners[i].kill)
    sim.run(until=horizon, stop=lambda: clients and all(c.done_at is not None for c in clients))
    out = _summary(sim, clients, log, dev, gpus, client_start, kills, net, miners_per_gpu)
    out["busy_avail"] = busy_while_available(app.arrivals, log, gpus, miners_per_gpu,
                                             [(client_start + t, i) for t, i in kills])
    out["speculated"] = sched.speculated
    return out


def busy_while_available(arrivals: dict, log: list, gpus: list, miners_per_gpu: int = 1, kills=()) -> float:
    """Useful GPU time over the GPU time during which work was available: from a request's
    arrival at the server until its last nonce was computed on some GPU (not until its
    Result reached anyone -- a Result stuck in the network idles no GPU that has work).
    Idle GPU time inside those spans is what the scheduler and the LSP's stalls cost.
    The same measure as tools/system_bench.py's `busy_frac_avail`."""
    spans = []
    first = {}
    for _, data, lo, hi, s, e in log:
        key = (data, lo, hi)
        if key not in first or e < first[key][1]:
            first[key] = (s, e)
    done = {}
    for (data, lo, hi), (s, e) in first.items():
        done[data] = max(done.get(data, 0.0), e)
    for data, t in arrivals.items():
        if data in done:
            spans.append((t, done[data]))
    spans.sort()
    merged = []
    for a, b in spans:
        if merged and a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    ngpus = len(gpus)
    cap = 0.0
    for a, b in merged:
        cap += ngpus * (b - a)
        if miners_per_gpu == 1:  # a killed miner's GPU leaves the node
            for t, _ in kills:
                cap -= max(0.0, b - max(a, t))
    # GPU-seconds of distinct work (a job's wall span overstates it on a shared GPU)
    useful = sum(hi - lo + 1 for data, lo, hi in first) / (sum(gpus) / ngpus)
    return useful / cap if cap > 0 else 0.0


def _start_client(sim, net, params, drop, srv, app) -> None:
    app.ep = ClientEP(sim, net, params, drop, drop, srv, app)


def _summary(sim, clients, log, dev, gpus, t0, kills, net, miners_per_gpu) -> dict:
    done = [c.done_at - t0 for c in clients if c.done_at is not None]
    work = {}
    for _, data, lo, hi, s, e in log:
        work.setdefault((data, lo, hi), (s, e))
    total = sum(hi - lo + 1 for data, lo, hi in work)
    makespan = max(done) if done else float("inf")
    # the node's capacity over the run (a killed miner's GPU counts until the kill)
    cap = sum(gpus) * makespan
    if miners_per_gpu == 1:  # a shared GPU keeps working for the rest
        for t, i in kills:
            cap -= gpus[i] * max(0.0, makespan - t)
    first = min((s for *_, s, e in log), default=t0)
    last = max((e for *_, s, e in log), default=t0)
    return {
        "makespan": makespan,
        "done": sorted(done),
        "disconnected": sum(c.disconnected for c in clients),
        "results": [c.result for c in clients],
        "jobs": len(log),
        "duplicates": len(log) - len(work),
        "work": total,
        "efficiency": total / cap if cap else 0.0,     # useful nonces / node capacity
        "gpu_busy": [g.busy for g in dev],
        "window": last - first,
        "datagrams": net.datagrams,
    }
