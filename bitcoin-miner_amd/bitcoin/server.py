"""Server -- bitcoin/server/server.go of the reference (stub at :15), written to p1.pdf
pp.13-15: split each client Request into jobs, farm them to miners, merge the Results,
answer the client.

Job chunking: the reference leaves "a suitable maximum job size"
open.  With GPU miners at ~34 GH/s each, a job of 2^34 nonces is ~0.5 s of GPU time:
big enough that per-job overhead (one LSP round trip + one gpuhash_min call, ~ms) is
<1%, small enough that a killed miner loses half a second of work and 16 concurrent
requests still spread over 8 miners.  GPUHASH_JOB_SIZE overrides it.

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
from dataclasses import dataclass, field

import lsp
from gpuhash import GPUHASH_MAX_MSG  # a constant only: the server never loads the engine

from . import UINT64_MAX, MsgType, NewRequest, NewResult, marshal, params_from_env, unmarshal

DEFAULT_JOB_SIZE = 1 << 34
MAX_REQUEUES = 3


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
    return None


@dataclass
class Job:
    req_id: int
    lower: int
    upper: int
    requeues: int = 0  # times a miner holding this job was lost


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
    """Pure bookkeeping (no I/O): tests drive it directly."""

    def __init__(self, job_size: int = DEFAULT_JOB_SIZE, max_requeues: int = MAX_REQUEUES):
        self.job_size = job_size
        self.max_requeues = max_requeues
        self.requests: dict[int, Request] = {}
        self.miners: dict[int, Job | None] = {}   # miner conn -> job in flight
        self.idle: collections.deque = collections.deque()
        self.abandoned: collections.deque = collections.deque()  # clients to disconnect
        self._ids = itertools.count(1)

    def add_miner(self, conn: int) -> None:
        if conn not in self.miners:
            self.miners[conn] = None
            self.idle.append(conn)

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
        """(miner, job, data) for the next dispatch, or None."""
        while self.idle:
            cands = [r for r in self.requests.values() if r.has_pending()]
            if not cands:
                return None
            r = min(cands, key=lambda x: (x.inflight, x.req_id))
            miner = self.idle.popleft()
            if miner not in self.miners:
                continue
            job = r.pop_job(self.job_size)
            r.inflight += 1
            self.miners[miner] = job
            return miner, job, r.data
        return None

    def result(self, miner: int, h: int, n: int):
        """Folds a miner's result; returns (client, (hash, nonce)) when a request is done."""
        job = self.miners.get(miner)
        if job is None:
            return None
        self.miners[miner] = None
        self.idle.append(miner)
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
            job = self.miners.pop(conn)
            try:
                self.idle.remove(conn)
            except ValueError:
                pass
            note = f"miner {conn} lost"
            if job is not None and job.req_id in self.requests:
                r = self.requests[job.req_id]
                r.inflight -= 1
                job.requeues += 1
                if job.requeues > self.max_requeues:
                    # every miner that took this job died: stop feeding it to the rest
                    del self.requests[r.req_id]
                    self.abandoned.append(r.client)
                    return (note + f"; job [{job.lower}, {job.upper}] lost {job.requeues} miners: "
                            f"request {r.req_id} abandoned, client {r.client} disconnected")
                r.requeued.appendleft(job)
                note += f"; job [{job.lower}, {job.upper}] of request {job.req_id} requeued"
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
    sched = Scheduler(job_size or int(os.environ.get("GPUHASH_JOB_SIZE", DEFAULT_JOB_SIZE)))

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
            if log and note:
                log(note)
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
