"""Server -- bitcoin/server/server.go of the reference (stub at :15), written to p1.pdf
pp.13-15: split each client Request into jobs, farm them to miners, merge the Results,
answer the client.

Job chunking: the reference leaves "a suitable maximum job size"
open.  Default: fixed jobs of 2^34 nonces, ~0.5 s on one MI355X -- big enough that the
per-job overhead (one LSP round trip + one gpuhash_min call, ~ms, plus an epoch-long
stall whenever a message is dropped) stays small, small enough that a killed miner
loses half a second of work and 16 concurrent requests spread over 8 miners
(GPUHASH_JOB_SIZE overrides the size).

Per-miner sizing (GPUHASH_JOB_SECONDS=t, or Scheduler(sizing=Sizing(...))): each job is
sized for the miner that takes it, to last ~t.  A miner's rate is learned from its own
results (work and wall time of its recent jobs, halved at every new result); its first
job is a 2^22-nonce probe.  This serves miners of
very different speeds (a CPU miner running the reference loop next to MI355X miners: a
2^34 job on it takes minutes) and spreads the end of a lone big request over every
miner (no job larger than its uncut remainder over its share of the miners, down to a
quarter job).  It is not the default because with lossy links its jobs, shorter than
fixed 2^34 ones whenever miners share a GPU, pay more resend stalls: BASELINE config 5
as run on a 1-GPU box (8 miners on one GPU, 10% drops) measured 29.6-30.9 GH/s against
33.2-33.7 with fixed jobs.

Scheduler (p1.pdf p.15, "balances loads across all requests"): an idle miner always
gets the next job of the outstanding request that currently has the FEWEST jobs in
flight (ties: oldest request first), so the workers assigned to each request differ by
at most one whenever requests have work queued.

Failures (p1.pdf p.15): a lost miner's job goes back to the FRONT of its request's queue
(and waits for a miner if none is left); a lost client's requests are dropped -- queued
jobs are discarded, in-flight results are ignored when they arrive.  A job whose miners
keep dying (more than MAX_REQUEUES losses, e.g. a job that trips a device fault on every
GPU) is not handed to miner after miner: its request is abandoned and the client's
connection closed, so the client prints "Disconnected".

Validation: a Request is accepted only if 0 <= Lower <= Upper <= 2^64-1 (the uint64
fields are already range-checked by unmarshal, as Go's json.Unmarshal would) and its
Data fits the engine (GPUHASH_MAX_MSG bytes).  Anything else is rejected by closing the
client's connection: no job is cut and nothing is left in flight.

Merging: results fold with the lexicographic (hash, nonce) key, so the answer is the
same however the range is chunked (lowest nonce among equal hashes).

    python bitcoin-miner_amd/bin/server port
"""
from __future__ import annotations

import collections
import itertools
import os
import sys
import time
from dataclasses import dataclass, field

import lsp
import lsp.message
import lspnet
from gpuhash import GPUHASH_MAX_MSG  # a constant only: the server never loads the engine

from . import UINT64_MAX, MsgType, NewRequest, NewResult, marshal, params_from_env, unmarshal

DEFAULT_JOB_SIZE = 1 << 34
MAX_REQUEUES = 3
JOB_SECONDS = 0.5
MINER_DEPTH = 1  # jobs a miner holds at once (serve(); GPUHASH_MINER_DEPTH overrides)


@dataclass
class Sizing:
    """Per-miner job sizing: a job lasts about `target_s` on the miner that takes it."""
    target_s: float = JOB_SECONDS
    probe: int = 1 << 22          # first job of a miner whose rate is unknown
    min_job: int = 1 << 16
    max_job: int = 1 << 40


@dataclass
class MinerRate:
    """Work and time of a miner's recent jobs, both halved at every new result: the
    rate is dominated by its long recent jobs, so the round trip of a short probe does
    not drag it down, and it follows a GPU that other miners start sharing.  Time is
    wall time per job, so the rate includes the job's round trip and any LSP resend
    stall: a job then lasts ~target_s including them."""
    work: float = 0.0
    secs: float = 0.0

    def add(self, n: int, dt: float) -> None:
        self.work = 0.5 * self.work + n
        self.secs = 0.5 * self.secs + max(dt, 1e-6)

    @property
    def rate(self) -> float:
        return self.work / self.secs


def request_error(data: str, lower: int, upper: int) -> str | None:
    """Why a client Request cannot be served, or None if it can."""
    for name, v in (("Lower", lower), ("Upper", upper)):
        if isinstance(v, bool) or not isinstance(v, int) or not 0 <= v <= UINT64_MAX:
            return f"{name}={v!r} outside [0, 2^64-1]"
    if lower > upper:
        return f"empty range: Lower {lower} > Upper {upper}"
    n = len(data.encode())
    if n > GPUHASH_MAX_MSG:
        return f"Data is {n} bytes, over the engine's {GPUHASH_MAX_MSG}"
    # every job Request this server cuts from it must fit one LSP datagram (the reference
    # reads 2000-byte buffers, lspnet/conn.go:35): a job's bounds can have more digits than
    # the client's Lower, so a request that fit may yield jobs that do not, and a
    # truncated datagram is never acked -- the job would hang
    if len(job_frame_worst_case(data, upper)) > lspnet.MAX_DATAGRAM:
        return f"its jobs would not fit a {lspnet.MAX_DATAGRAM}-byte LSP datagram"
    return None


def job_frame_worst_case(data: str, upper: int = UINT64_MAX) -> bytes:
    """The longest LSP frame a job of this request can take: no job bound exceeds the
    request's Upper, so both bounds at Upper's digit count (pricing them at
    2^64-1 refused requests the reference serves), 10-digit ConnID and SeqNum."""
    return lsp.message.NewData(2**31 - 1, 2**31 - 1, marshal(NewRequest(data, upper, upper))).marshal()


@dataclass
class Job:
    req_id: int
    lower: int
    upper: int
    requeues: int = 0  # times a miner holding this job was lost
    sent: float = 0.0  # when it was last dispatched (Scheduler clock)


@dataclass
class Request:
    """One client request.  Jobs are cut lazily from [next_lo, upper] (a request may span
    all of [0, 2^64-1], i.e. 2^30 jobs, so they are never materialised); jobs of lost
    miners wait in `requeued` and go out first."""
    req_id: int
    client: int
    data: str
    next_lo: int = 0
    upper: int = -1       # next_lo > upper: nothing left to cut
    requeued: collections.deque = field(default_factory=collections.deque)
    inflight: int = 0
    best: tuple | None = None

    def has_pending(self) -> bool:
        return bool(self.requeued) or self.next_lo <= self.upper

    def uncut(self) -> int:
        """Nonces not yet cut into any job."""
        return max(0, self.upper - self.next_lo + 1)

    def remaining(self) -> int:
        """Nonces not yet handed to a miner: the uncut range plus requeued jobs."""
        return self.uncut() + sum(j.upper - j.lower + 1 for j in self.requeued)

    def pop_job(self, size: int) -> Job:
        if self.requeued:
            return self.requeued.popleft()
        lo = self.next_lo
        hi = min(self.upper, lo + size - 1)
        self.next_lo = hi + 1
        return Job(self.req_id, lo, hi)


def split_jobs(req_id: int, lower: int, upper: int, size: int):
    """Contiguous jobs of at most `size` nonces covering the inclusive range."""
    lo = lower
    while True:
        hi = min(upper, lo + size - 1)
        yield Job(req_id, lo, hi)
        if hi >= upper:
            return
        lo = hi + 1


class Scheduler:
    """Pure bookkeeping (no I/O): tests drive it directly.  `sizing` None = fixed jobs of
    `job_size`; otherwise jobs are sized per miner (Sizing), timed with `clock`.

    `depth` = jobs a miner may hold at once.  With 2, a miner's next Request is already
    queued in its LSP connection while it computes, so the Result -> Request round trip
    and any resend stall after a dropped message overlap the GPU's work instead of
    idling it.  A miner answers its Requests in order over an in-order connection, so a
    Result belongs to the oldest job the miner holds.  The default stays 1: on one GPU
    shared by 8 miners a stalled miner's share goes to the others anyway, and config 5
    measured no gain there (33.2 vs 32.2-33.2 GH/s, a killed miner then strands two
    jobs); the gain is for one miner per GPU over lossy links."""

    def __init__(self, job_size: int = DEFAULT_JOB_SIZE, max_requeues: int = MAX_REQUEUES,
                 sizing: Sizing | None = None, clock=time.monotonic, depth: int = 1):
        self.job_size = job_size
        self.max_requeues = max_requeues
        self.sizing = sizing
        self.clock = clock
        self.depth = max(1, depth)
        self.rates: dict[int, MinerRate] = {}
        self.done_at: dict[int, float] = {}   # miner -> when its last result arrived
        self.requests: dict[int, Request] = {}
        self.miners: dict[int, collections.deque] = {}  # miner conn -> its jobs, oldest first
        self.abandoned: collections.deque = collections.deque()  # clients to disconnect
        self._ids = itertools.count(1)
        self._tick = itertools.count()
        self._turn: dict[int, int] = {}       # miner -> when it last got a job

    def add_miner(self, conn: int) -> None:
        if conn not in self.miners:
            self.miners[conn] = collections.deque()
            self._turn[conn] = next(self._tick)

    def add_request(self, client: int, data: str, lower: int, upper: int) -> int:
        """Registers a request; ValueError (nothing registered) if request_error()."""
        err = request_error(data, lower, upper)
        if err is not None:
            raise ValueError(err)
        rid = next(self._ids)
        r = Request(rid, client, data, next_lo=lower, upper=upper)
        self.requests[rid] = r
        return rid

    def next_assignment(self):
        """(miner, job, data) for the next dispatch, or None.  The miner holding the
        fewest jobs goes first (then the one served longest ago); the request with the
        fewest jobs in flight gets it, then the one with the least work left to hand out,
        then the oldest.  The second key is shortest-remaining-first: a short request that
        arrives while a long one keeps every miner busy gets the next job instead of
        waiting for the long one to finish, and equal requests still finish one after
        another rather than all at the end (p1.pdf p.15)."""
        free = [m for m, q in self.miners.items() if len(q) < self.depth]
        if not free:
            return None
        cands = [r for r in self.requests.values() if r.has_pending()]
        if not cands:
            return None
        miner = min(free, key=lambda m: (len(self.miners[m]), self._turn[m]))
        r = min(cands, key=lambda x: (x.inflight, x.remaining(), x.req_id))
        job = r.pop_job(self.size_for(miner, r))
        job.sent = self.clock()
        r.inflight += 1
        self.miners[miner].append(job)
        self._turn[miner] = next(self._tick)
        return miner, job, r.data

    def size_for(self, miner: int, r: Request) -> int:
        """Nonces of the next job cut from `r` for `miner`."""
        if self.sizing is None:
            return self.job_size
        s = self.sizing
        mr = self.rates.get(miner)
        if mr is None:
            return s.probe
        size = int(mr.rate * s.target_s)
        # end game: what is left of the request is spread over its share of the miners
        # (all of them when it is the only request with work left), down to a quarter of
        # this miner's full job so the tail is not shredded into tiny jobs
        active = sum(1 for x in self.requests.values() if x.has_pending())
        miners = max(1, -(-len(self.miners) // max(1, active)))
        share = max(-(-r.uncut() // miners), size // 4)
        return max(s.min_job, min(s.max_job, size, share))

    def result(self, miner: int, h: int, n: int):
        """Folds a miner's result (for its oldest job); returns (client, (hash, nonce))
        when a request is done."""
        q = self.miners.get(miner)
        if not q:
            return None
        job = q.popleft()
        now = self.clock()
        # the job computed from when it was sent or the miner's previous result came back
        start = max(job.sent, self.done_at.get(miner, job.sent))
        self.done_at[miner] = now
        self.rates.setdefault(miner, MinerRate()).add(job.upper - job.lower + 1, now - start)
        r = self.requests.get(job.req_id)
        if r is None:  # the client is gone: ignore the result
            return None
        r.inflight -= 1
        if r.best is None or (h, n) < r.best:
            r.best = (h, n)
        if not r.has_pending() and r.inflight == 0:
            del self.requests[r.req_id]
            return r.client, r.best
        return None

    def lost(self, conn: int) -> str | None:
        """Forgets a lost connection; returns a log line describing what changed."""
        note = None
        if conn in self.miners:
            jobs = self.miners.pop(conn)
            self._turn.pop(conn, None)
            self.rates.pop(conn, None)
            self.done_at.pop(conn, None)
            notes = [f"miner {conn} lost"]
            for job in reversed(jobs):  # requeued oldest-first at the front
                r = self.requests.get(job.req_id)
                if r is None:
                    continue
                r.inflight -= 1
                job.requeues += 1
                if job.requeues > self.max_requeues:
                    # every miner that took this job died: stop feeding it to the rest
                    del self.requests[r.req_id]
                    self.abandoned.append(r.client)
                    notes.append(f"job [{job.lower}, {job.upper}] lost {job.requeues} miners: "
                                 f"request {r.req_id} abandoned, client {r.client} disconnected")
                    continue
                r.requeued.appendleft(job)
                notes.append(f"job [{job.lower}, {job.upper}] of request {job.req_id} requeued")
            note = "; ".join(notes)
        dropped = [rid for rid, r in self.requests.items() if r.client == conn]
        for rid in dropped:
            del self.requests[rid]
        if dropped:
            note = f"client {conn} lost; dropped request(s) {dropped}"
        return note


def serve(port: int, params=None, job_size: int | None = None, ready=None, log=None) -> None:
    """Runs the server until its LSP server is closed.  `log(str)` (or GPUHASH_SERVER_LOG=1
    for stderr) receives joins, requests and failure handling."""
    srv = lsp.NewServer(port, params or params_from_env())
    if log is None and os.environ.get("GPUHASH_SERVER_LOG"):
        def log(line):  # stderr only: stdout of the programs is graded (p1.pdf p.15)
            print(f"server: {line}", file=sys.stderr, flush=True)
    if ready is not None:
        ready(srv)
    secs = os.environ.get("GPUHASH_JOB_SECONDS")
    depth = int(os.environ.get("GPUHASH_MINER_DEPTH", MINER_DEPTH))
    if job_size is None and secs:
        sched = Scheduler(sizing=Sizing(target_s=float(secs)), depth=depth)
    else:
        sched = Scheduler(job_size or int(os.environ.get("GPUHASH_JOB_SIZE", DEFAULT_JOB_SIZE)), depth=depth)

    def disconnect_abandoned():
        while sched.abandoned:
            client = sched.abandoned.popleft()
            try:
                srv.CloseConn(client)
            except lsp.LSPError:
                pass

    def dispatch():
        disconnect_abandoned()
        while True:
            a = sched.next_assignment()
            if a is None:
                return
            miner, job, data = a
            try:
                srv.Write(miner, marshal(NewRequest(data, job.lower, job.upper)))
            except lsp.LSPError:
                note = sched.lost(miner)
                if log and note:
                    log(note)
                disconnect_abandoned()

    while True:
        try:
            conn, payload = srv.Read()
        except lsp.LSPError as e:
            if e.conn_id == 0:
                return  # server closed
            note = sched.lost(e.conn_id)
            if log:  # the LSP's reason (silent epochs, last heard) beside what it cost
                log(f"{e}: {note}" if note else str(e))
            dispatch()
            continue
        try:
            m = unmarshal(payload)
        except (ValueError, KeyError):
            continue
        if m.Type == MsgType.Join:
            sched.add_miner(conn)
        elif m.Type == MsgType.Request:
            try:
                sched.add_request(conn, m.Data, m.Lower, m.Upper)
            except ValueError as e:  # rejected: the client sees its connection close
                if log:
                    log(f"conn {conn}: request rejected ({e}); closing the connection")
                try:
                    srv.CloseConn(conn)
                except lsp.LSPError:
                    pass
                continue
        elif m.Type == MsgType.Result:
            done = sched.result(conn, m.Hash, m.Nonce)
            if done is not None:
                client, (h, n) = done
                try:
                    srv.Write(client, marshal(NewResult(h, n)))
                except lsp.LSPError:
                    pass
        if log and m.Type != MsgType.Result:
            log(f"conn {conn}: {m}")
        dispatch()


def main(argv=None) -> int:
    argv = sys.argv if argv is None else argv
    if len(argv) != 2:  # server.go:9-13
        print("Usage: ./server <port>")
        return 0
    serve(int(argv[1]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
