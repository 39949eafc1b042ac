"""Server -- bitcoin/server/server.go of the reference (stub at :15), written to p1.pdf
pp.13-15: split each client Request into jobs, farm them to miners, merge the Results,
answer the client.

Job chunking: the reference leaves "a suitable maximum job size"
open.  Default: fixed jobs of half a second of one MI355X (or one LSP epoch if shorter),
a power of two -- 2^34 nonces at the reference's 2 s epochs (default_job_size).  The
programs send every LSP datagram three times (bitcoin.SEND_COPIES), so a dropped Request
or Result rarely waits for the next epoch, and four jobs per 2^36-nonce config-5 request
spread it over a node's GPUs.  With single sends (LSP_SEND_COPIES=1, the protocol exactly
as specified) a dropped message stalls its window-1 connection until the next epoch
with p = 0.19 at config 5's drops, and jobs are one epoch long (2^36) so that the
stalls do not dominate.  A request's last sliver (under a quarter job) rides with the
job before it.  GPUHASH_JOB_SIZE overrides the size.

Depth and speculative copies: a miner holds up to MINER_DEPTH (3) jobs, so its next
Request is already there while a Result or a Request waits for a resend; when nothing is
left to hand out, a miner holding nothing takes a copy of a job that is overdue by its
holder's learned rate (up to COPIES live copies, the first Result wins), which covers a
dropped Result and a killed miner, which LSP reports only after EpochLimit silent epochs
(10 s by default).  DESIGN.md 6.2-6.4 has the model (tests/lsp_des.py) and the
measurements behind these defaults.

Per-miner sizing (GPUHASH_JOB_SECONDS=t, or Scheduler(sizing=Sizing(...))): each job is
sized for the miner that takes it, to last ~t.  A miner's rate is learned from its own
results (work and wall time of its recent jobs, halved at every new result); its first
job is a 2^22-nonce probe.  This serves miners of very different speeds (a CPU miner
running the reference loop next to MI355X miners) and spreads the end of a lone big
request over every miner.  It is not the default: on lossy links its shorter jobs pay
more resend stalls.

Scheduler (p1.pdf p.15, "balances loads across all requests"): an idle miner always
gets the next job of the outstanding request that currently has the FEWEST jobs in
flight (then the least work left, then the oldest), so the workers assigned to each
request differ by at most one whenever requests have work queued.

Failures (p1.pdf p.15): a lost miner's unfinished jobs go back to the FRONT of their
requests' queues (unless another miner holds a copy); a lost client's requests are
dropped -- queued jobs are discarded, in-flight results are ignored when they arrive.  A
job whose miners keep dying while computing it (more than MAX_REQUEUES such losses, e.g.
a job that trips a device fault on every GPU) is not handed to miner after miner: its
request is abandoned and the client's connection closed, so the client prints
"Disconnected".  Jobs queued behind the one a lost miner was computing never ran and are
not charged.

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
import math
import os
import sys
import time
from dataclasses import dataclass, field

import lsp
import lsp.message
import lspnet
from gpuhash import GPUHASH_MAX_MSG  # a constant only: the server never loads the engine

from . import UINT64_MAX, MsgType, NewRequest, NewResult, marshal, params_from_env, unmarshal

MAX_REQUEUES = 3
JOB_SECONDS = 0.5
# The server program's defaults (make_scheduler; DESIGN.md 6 has the measurements behind
# them).  Scheduler() itself defaults to the plain scheduler: fixed jobs, depth 1, no copies.
REF_RATE = 34.6e9  # nonces/s of one MI355X on config 2 (profiles/r05_bench_config2.json)
MINER_DEPTH = 3    # jobs a miner holds at once (GPUHASH_MINER_DEPTH)
COPIES = 3         # live copies of an overdue job (GPUHASH_COPIES; GPUHASH_BACKUP=0: 1)
SLACK = 0.1        # a copy is overdue this long after its expected answer ...
SLACK_FRAC = 0.25  # ... or this fraction of its job time, if longer


def default_job_size(epoch_s: float, send_copies: int = 1) -> int:
    """GPU work of one MI355X, to a power of two, for a job's wall time of: one LSP epoch
    when every datagram is sent once (2^36 at the reference's 2 s epochs, 2^33 at 200 ms)
    -- each job is a Request and a Result over a window-1 connection whose dropped
    messages wait for the next epoch, so a job much shorter than an epoch spends its time
    waiting on the connection; half a second, or one epoch if shorter, when the programs
    send copies (2^34 at 2 s, 2^33 at 200 ms) -- a stall is then rare, and shorter jobs
    spread config 5's 2^36-nonce requests over a node's GPUs."""
    secs = epoch_s if send_copies <= 1 else min(epoch_s, 0.5)
    b = math.floor(math.log2(max(1.0, REF_RATE * secs)) + 0.5)  # lround, as the C++ server
    return 1 << min(40, max(30, b))


DEFAULT_JOB_SIZE = default_job_size(2.0)  # 2^36 at lsp.params' DefaultEpochMillis, one copy


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


@dataclass(eq=False)
class Job:
    """A range of one request.  The same Job object sits in the queue of every miner that
    holds a copy of it (speculative copies, Scheduler); `done` once any copy answered."""
    req_id: int
    lower: int
    upper: int
    requeues: int = 0  # losses of a miner that was computing this job
    sent: float = 0.0  # when it was first dispatched (Scheduler clock)
    done: bool = False
    holders: dict = field(default_factory=dict)  # miner -> when its copy was sent

    @property
    def size(self) -> int:
        return self.upper - self.lower + 1


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
        """The next job: a requeued one, else the next `size` nonces -- or all that is
        left when less than a quarter job would remain (a sliver job costs a whole LSP
        round trip for no work, e.g. the one nonce of [0, 2^35] past 2^35)."""
        if self.requeued:
            return self.requeued.popleft()
        lo = self.next_lo
        hi = self.upper if self.upper - lo + 1 < size + size // 4 else lo + size - 1
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

    `depth` = jobs a miner may hold at once.  With 2 or more, a miner's next Request is
    already queued in its LSP connection while it computes, so the Result -> Request round
    trip and any resend stall after a dropped message overlap the GPU's work instead of
    idling it.  A miner answers its Requests in order over an in-order connection, so a
    Result belongs to the oldest job the miner holds.

    `copies` > 1 enables speculative copies (backup tasks): when no request has work left
    to hand out, a miner that holds nothing takes a copy of a job another miner still
    holds -- with hedge="overdue" only once every copy of it is past its expected answer
    (the holder's learned rate and queue, plus `slack`), with hedge="idle" at once.  The
    first Result of any copy completes the job; later ones are ignored.  That covers what
    LSP makes slow: a Result stuck behind drops (each costs up to an epoch, 2 s by
    default), and a killed miner, which LSP reports only after EpochLimit silent epochs
    (10 s by default)."""

    def __init__(self, job_size: int = DEFAULT_JOB_SIZE, max_requeues: int = MAX_REQUEUES,
                 sizing: Sizing | None = None, clock=time.monotonic, depth: int = 1,
                 copies: int = 1, hedge: str = "overdue", slack: float = 0.1, slack_frac: float = 0.5):
        self.job_size = job_size
        self.max_requeues = max_requeues
        self.sizing = sizing
        self.clock = clock
        self.depth = max(1, depth)
        self.copies = max(1, copies)
        if hedge not in ("overdue", "idle"):
            raise ValueError(f"hedge={hedge!r}: 'overdue' or 'idle'")
        self.hedge = hedge
        self.slack = slack            # seconds past a copy's expected answer ...
        self.slack_frac = slack_frac  # ... or this fraction of its job time, if longer
        self.rates: dict[int, MinerRate] = {}
        self.done_at: dict[int, float] = {}   # miner -> when its last result arrived
        self.requests: dict[int, Request] = {}
        self.miners: dict[int, collections.deque] = {}  # miner conn -> its jobs, oldest first
        self.abandoned: collections.deque = collections.deque()  # clients to disconnect
        self.speculated = 0                   # copies handed out
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
        another rather than all at the end (p1.pdf p.15).  With nothing left to hand out,
        a speculative copy (`copies`)."""
        free = [m for m, q in self.miners.items() if len(q) < self.depth]
        if not free:
            return None
        cands = [r for r in self.requests.values() if r.has_pending()]
        if not cands:
            return self._speculate()
        miner = min(free, key=lambda m: (len(self.miners[m]), self._turn[m]))
        r = min(cands, key=lambda x: (x.inflight, x.remaining(), x.req_id))
        job = r.pop_job(self.size_for(miner, r))
        job.sent = self.clock()
        job.holders[miner] = job.sent
        r.inflight += 1
        self.miners[miner].append(job)
        self._turn[miner] = next(self._tick)
        return miner, job, r.data

    # -- speculative copies ----------------------------------------------------------
    def _rate(self, miner: int) -> float | None:
        mr = self.rates.get(miner)
        if mr is not None:
            return mr.rate
        known = sorted(x.rate for x in self.rates.values())
        return known[len(known) // 2] if known else None  # a new miner: the median

    def _expected(self, job: Job, miner: int) -> float | None:
        """When `miner`'s Result for `job` is due: its queue worked in order at its rate,
        each job starting once sent and once the previous one is answered."""
        rate = self._rate(miner)
        if rate is None:
            return None
        t = self.done_at.get(miner, 0.0)
        for j in self.miners.get(miner, ()):
            t = max(t, j.holders.get(miner, j.sent)) + j.size / rate
            if j is job:
                return t + max(self.slack, self.slack_frac * j.size / rate)
        return None

    def _overdue_at(self, job: Job) -> float | None:
        """When every copy of `job` is overdue (None: some holder's rate is unknown)."""
        ts = [self._expected(job, m) for m in job.holders]
        return None if not ts or None in ts else max(ts)

    def _unfinished(self):
        seen = set()
        for q in self.miners.values():
            for j in q:
                if not j.done and id(j) not in seen and j.req_id in self.requests:
                    seen.add(id(j))
                    yield j

    def _speculate(self):
        if self.copies <= 1:
            return None
        idle = [m for m, q in self.miners.items() if not q]
        if not idle:
            return None
        now = self.clock()
        best = None
        for job in self._unfinished():
            if len(job.holders) >= self.copies:
                continue
            if self.hedge == "overdue":
                t = self._overdue_at(job)
                if t is None or t > now:
                    continue
                key = (t, job.sent)
            else:
                key = (len(job.holders), job.sent)
            if best is None or key < best[0]:
                best = (key, job)
        if best is None:
            return None
        job = best[1]
        miner = max(idle, key=lambda m: (self._rate(m) or 0.0, -self._turn[m]))  # the fastest
        job.holders[miner] = now
        self.miners[miner].append(job)
        self._turn[miner] = next(self._tick)
        self.speculated += 1
        return miner, job, self.requests[job.req_id].data

    def next_wakeup(self) -> float | None:
        """When (Scheduler clock) next_assignment() may have something new to hand out
        without any message arriving -- the next job to become overdue while a miner is
        idle -- or None: only a message can change that."""
        if self.copies <= 1 or self.hedge != "overdue":
            return None
        if not any(not q for q in self.miners.values()):
            return None
        if any(r.has_pending() for r in self.requests.values()):
            return None
        ts = [self._overdue_at(j) for j in self._unfinished() if len(j.holders) < self.copies]
        ts = [t for t in ts if t is not None]
        return min(ts) if ts else None

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
        when a request is done.  A copy that answers after another one is ignored."""
        q = self.miners.get(miner)
        if not q:
            return None
        job = q.popleft()
        now = self.clock()
        sent = job.holders.pop(miner, job.sent)
        # the job computed from when it was sent or the miner's previous result came back
        start = max(sent, self.done_at.get(miner, sent))
        self.done_at[miner] = now
        self.rates.setdefault(miner, MinerRate()).add(job.size, now - start)
        if job.done:
            return None
        job.done = True
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
        """Forgets a lost connection; returns a log line describing what changed.  A lost
        miner's unfinished jobs go back to the front of their requests' queues unless
        another miner holds a copy.  Only the job it was computing -- the oldest it held --
        counts toward that job's requeue cap: the ones queued behind it never ran, so a
        miner lost for any other reason does not use up their cap."""
        note = None
        if conn in self.miners:
            jobs = self.miners.pop(conn)
            self._turn.pop(conn, None)
            self.rates.pop(conn, None)
            self.done_at.pop(conn, None)
            current = jobs[0] if jobs else None
            notes = [f"miner {conn} lost"]
            for job in reversed(jobs):  # requeued oldest-first at the front
                job.holders.pop(conn, None)
                r = self.requests.get(job.req_id)
                if job.done or r is None:
                    continue
                if job is current:
                    job.requeues += 1
                    if job.requeues > self.max_requeues:
                        # every miner that computed this job died: stop feeding it to the rest
                        r.inflight -= 1
                        del self.requests[r.req_id]
                        self.abandoned.append(r.client)
                        notes.append(f"job [{job.lower}, {job.upper}] lost {job.requeues} miners: "
                                     f"request {r.req_id} abandoned, client {r.client} disconnected")
                        continue
                if job.holders:  # a copy is still out: nothing to hand out again
                    notes.append(f"job [{job.lower}, {job.upper}] of request {job.req_id} still held "
                                 f"by miner(s) {sorted(job.holders)}")
                    continue
                r.inflight -= 1
                r.requeued.appendleft(job)
                notes.append(f"job [{job.lower}, {job.upper}] of request {job.req_id} requeued")
            note = "; ".join(notes)
        dropped = [rid for rid, r in self.requests.items() if r.client == conn]
        for rid in dropped:
            del self.requests[rid]
        if dropped:
            note = f"client {conn} lost; dropped request(s) {dropped}"
        return note


class ServerCore:
    """The server program's event handling, free of I/O: serve() drives it from the LSP
    server's Read loop, tests/lsp_des.py from a discrete-event simulation of the same LSP
    endpoints.  `write(conn, payload)` raises lsp.LSPError for a lost connection;
    `close_conn(conn)` closes one."""

    def __init__(self, sched: Scheduler, write, close_conn, log=None):
        self.sched = sched
        self.write = write
        self.close_conn = close_conn
        self.log = log

    def _disconnect_abandoned(self) -> None:
        while self.sched.abandoned:
            client = self.sched.abandoned.popleft()
            try:
                self.close_conn(client)
            except lsp.LSPError:
                pass

    def dispatch(self) -> None:
        self._disconnect_abandoned()
        while True:
            a = self.sched.next_assignment()
            if a is None:
                return
            miner, job, data = a
            if self.log and len(job.holders) > 1:
                self.log(f"copy of job [{job.lower}, {job.upper}] of request {job.req_id} to miner {miner} "
                         f"(held by {sorted(m for m in job.holders if m != miner)}, overdue)")
            try:
                self.write(miner, marshal(NewRequest(data, job.lower, job.upper)))
            except lsp.LSPError:
                note = self.sched.lost(miner)
                if self.log and note:
                    self.log(note)
                self._disconnect_abandoned()

    def on_lost(self, conn: int, reason: str = "") -> None:
        note = self.sched.lost(conn)
        if self.log:  # the LSP's reason (silent epochs, last heard) beside what it cost
            self.log(f"{reason}: {note}" if note else reason)
        self.dispatch()

    def on_timer(self) -> None:
        self.dispatch()

    def on_payload(self, conn: int, payload: bytes) -> None:
        try:
            m = unmarshal(payload)
        except (ValueError, KeyError):
            return
        if m.Type == MsgType.Join:
            self.sched.add_miner(conn)
        elif m.Type == MsgType.Request:
            try:
                self.sched.add_request(conn, m.Data, m.Lower, m.Upper)
            except ValueError as e:  # rejected: the client sees its connection close
                if self.log:
                    self.log(f"conn {conn}: request rejected ({e}); closing the connection")
                try:
                    self.close_conn(conn)
                except lsp.LSPError:
                    pass
                return
        elif m.Type == MsgType.Result:
            done = self.sched.result(conn, m.Hash, m.Nonce)
            if done is not None:
                client, (h, n) = done
                try:
                    self.write(client, marshal(NewResult(h, n)))
                except lsp.LSPError:
                    pass
        if self.log and m.Type != MsgType.Result:
            self.log(f"conn {conn}: {m}")
        self.dispatch()


def make_scheduler(job_size: int | None = None, epoch_s: float = 2.0, send_copies: int = 1) -> Scheduler:
    """The Scheduler serve() runs (csrc/server_main.cpp builds the same one): jobs of
    default_job_size(epoch_s, send_copies), MINER_DEPTH jobs per miner, up to COPIES live copies of an
    overdue job.  GPUHASH_JOB_SIZE, GPUHASH_JOB_SECONDS (per-miner sizing),
    GPUHASH_MINER_DEPTH, GPUHASH_COPIES and GPUHASH_BACKUP=0 override them."""
    secs = os.environ.get("GPUHASH_JOB_SECONDS")
    depth = int(os.environ.get("GPUHASH_MINER_DEPTH", MINER_DEPTH))
    copies = 1 if os.environ.get("GPUHASH_BACKUP") == "0" else int(os.environ.get("GPUHASH_COPIES", COPIES))
    kw = dict(depth=depth, copies=copies, hedge="overdue", slack=SLACK, slack_frac=SLACK_FRAC)
    if job_size is None and secs:
        return Scheduler(sizing=Sizing(target_s=float(secs)), **kw)
    size = job_size or int(os.environ.get("GPUHASH_JOB_SIZE", 0)) or default_job_size(epoch_s, send_copies)
    return Scheduler(size, **kw)


def serve(port: int, params=None, job_size: int | None = None, ready=None, log=None) -> None:
    """Runs the server until its LSP server is closed.  `log(str)` (or GPUHASH_SERVER_LOG=1
    for stderr) receives joins, requests and failure handling."""
    params = params or params_from_env()
    srv = lsp.NewServer(port, params)
    if log is None and os.environ.get("GPUHASH_SERVER_LOG"):
        def log(line):  # stderr only: stdout of the programs is graded (p1.pdf p.15)
            print(f"server: {line}", file=sys.stderr, flush=True)
    if ready is not None:
        ready(srv)
    sched = make_scheduler(job_size, params.EpochMillis / 1000.0, params.SendCopies)
    core = ServerCore(sched, srv.Write, srv.CloseConn, log)
    if log:  # the configuration, in the words of csrc/server_main.cpp (tests compare the two)
        size = "per-miner" if sched.sizing is not None else str(sched.job_size)
        log(f"config: jobs of {size} nonces, depth {sched.depth}, {sched.copies} live copies of an overdue "
            f"job; LSP epoch {params.EpochMillis} ms, limit {params.EpochLimit}, window {params.WindowSize}, "
            f"send copies {params.SendCopies}")
    while True:
        wake = core.sched.next_wakeup()
        try:
            got = srv.read_until(wake)
        except lsp.LSPError as e:
            if e.conn_id == 0:
                return  # server closed
            core.on_lost(e.conn_id, str(e))
            continue
        if got is None:
            core.on_timer()
        else:
            core.on_payload(*got)


def main(argv=None) -> int:
    argv = sys.argv if argv is None else argv
    if len(argv) != 2:  # server.go:9-13
        print("Usage: ./server <port>")
        return 0
    serve(int(argv[1]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
