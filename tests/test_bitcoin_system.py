"""CPU: the bitcoin server / miner / client programs in-process.

The miners here search with the oracle (test infrastructure standing in for the GPU
engine, which tests/test_gpu_system.py uses for real); what is under test is the
server's job chunking, its load-balancing scheduler, failure handling (lost miner ->
job reassigned, lost client -> work dropped) and the lexicographic merge, over LSP with
packet drops.  Answers are checked against the oracle over the whole range.
"""
import threading
import time

import pytest

import bitcoin
import lsp
import lspnet
from bitcoin import client as bclient
from bitcoin import miner as bminer
from bitcoin import server as bserver

P = lsp.Params(EpochLimit=20, EpochMillis=40, WindowSize=1)


class OracleEngine:
    def __init__(self, oracle, delay=0.0):
        self.oracle, self.delay, self.calls = oracle, delay, []

    def min(self, msg, lo, hi):
        self.calls.append((lo, hi))
        if self.delay:
            time.sleep(self.delay)
        return self.oracle.min(msg.encode(), lo, hi)


@pytest.fixture(autouse=True)
def no_drops():
    yield
    lspnet.SetReadDropPercent(0)
    lspnet.SetWriteDropPercent(0)


def start_server(job_size):
    box = {}
    ready = threading.Event()

    def on_ready(srv):
        box["srv"] = srv
        ready.set()

    t = threading.Thread(target=bserver.serve, args=(0,), kwargs=dict(params=P, job_size=job_size, ready=on_ready),
                         daemon=True)
    t.start()
    ready.wait(5)
    return box["srv"], t


def close_quietly(srv):
    """Server.Close raises if a client is lost while closing (server_api.go:33-38); the
    clients here have already gone away, so that is expected."""
    try:
        srv.Close()
    except lsp.LSPError:
        pass


def start_miner(port, engine):
    t = threading.Thread(target=bminer.run, args=(f"127.0.0.1:{port}", engine, P), daemon=True)
    t.start()
    return t


# ---- scheduler bookkeeping ---------------------------------------------------------

def test_split_jobs_tiles_range():
    jobs = list(bserver.split_jobs(1, 5, 104, 10))
    assert [(j.lower, j.upper) for j in jobs][:2] == [(5, 14), (15, 24)]
    assert jobs[-1].upper == 104 and len(jobs) == 10
    top = list(bserver.split_jobs(1, (1 << 64) - 25, (1 << 64) - 1, 10))
    assert top[-1].upper == (1 << 64) - 1 and sum(j.upper - j.lower + 1 for j in top) == 25


def test_scheduler_balances_requests():
    s = bserver.Scheduler(job_size=10)
    r1 = s.add_request(client=100, data="a", lower=0, upper=999)
    r2 = s.add_request(client=101, data="b", lower=0, upper=999)
    for m in range(6):
        s.add_miner(m)
    got = [s.next_assignment() for _ in range(6)]
    per_req = {r1: 0, r2: 0}
    for miner, job, data in got:
        per_req[job.req_id] += 1
    assert per_req == {r1: 3, r2: 3}
    assert s.next_assignment() is None  # no idle miners left


def test_scheduler_does_not_starve_a_later_request():
    """One miner, a long request in progress: a short request that arrives later gets
    the next jobs (least work left first) and finishes; then the long one resumes."""
    s = bserver.Scheduler(job_size=10)
    big = s.add_request(client=100, data="a", lower=0, upper=10 ** 6)
    s.add_miner(1)
    m, job, _ = s.next_assignment()
    small = s.add_request(client=101, data="b", lower=0, upper=29)
    order = []
    for _ in range(6):
        s.result(m, 1, job.lower)
        m, job, _ = s.next_assignment()
        order.append(job.req_id)
    assert order == [small, small, small, big, big, big]


def test_scheduler_equal_requests_finish_in_turn():
    """Requests of equal size arriving together finish one after another (shortest
    remaining first), not all at once at the end."""
    s = bserver.Scheduler(job_size=10)
    a = s.add_request(client=100, data="a", lower=0, upper=29)
    b = s.add_request(client=101, data="b", lower=0, upper=29)
    s.add_miner(1)
    done, order = [], []
    m, job, _ = s.next_assignment()
    while True:
        order.append(job.req_id)
        r = s.result(m, 1, job.lower)
        if r is not None:
            done.append(r[0])
        nxt = s.next_assignment()
        if nxt is None:
            break
        m, job, _ = nxt
    assert order == [a, a, a, b, b, b] and done == [100, 101]


def test_scheduler_reassigns_lost_miner_job_first():
    s = bserver.Scheduler(job_size=10)
    s.add_request(client=100, data="a", lower=0, upper=29)
    s.add_miner(1)
    s.add_miner(2)
    m1, j1, _ = s.next_assignment()
    s.next_assignment()
    s.lost(m1)
    s.add_miner(3)
    m3, j3, _ = s.next_assignment()
    assert m3 == 3 and (j3.lower, j3.upper) == (j1.lower, j1.upper)


def test_scheduler_drops_lost_client_and_ignores_late_results():
    s = bserver.Scheduler(job_size=10)
    s.add_request(client=100, data="a", lower=0, upper=99)
    s.add_miner(1)
    m, job, _ = s.next_assignment()
    s.lost(100)
    assert s.requests == {}
    assert s.result(m, 5, 5) is None  # result for a dropped request: ignored
    assert s.next_assignment() is None


def test_full_u64_request_cuts_jobs_lazily():
    # [0, 2^64-1] is 2^30 jobs of 2^34: the scheduler must not materialise them
    import time
    s = bserver.Scheduler(job_size=1 << 34)
    t = time.time()
    rid = s.add_request(client=100, data="a", lower=0, upper=(1 << 64) - 1)
    assert time.time() - t < 0.1
    s.add_miner(1)
    s.add_miner(2)
    (m1, j1, _), (m2, j2, _) = s.next_assignment(), s.next_assignment()
    assert (j1.lower, j1.upper, j2.lower) == (0, (1 << 34) - 1, 1 << 34)
    s.lost(m1)  # the lost job goes out again before any new one
    s.add_miner(3)
    _, j3, _ = s.next_assignment()
    assert (j3.lower, j3.upper) == (j1.lower, j1.upper)
    r = s.requests[rid]
    r.next_lo = (1 << 64) - 10  # fast-forward to the top of the range
    s.result(m2, 9, 9)
    _, j4, _ = s.next_assignment()
    assert (j4.lower, j4.upper) == ((1 << 64) - 10, (1 << 64) - 1)
    assert not r.has_pending()


def test_merge_is_lexicographic():
    s = bserver.Scheduler(job_size=5)
    s.add_request(client=100, data="a", lower=0, upper=9)
    s.add_miner(1)
    s.add_miner(2)
    (ma, _, _), (mb, _, _) = s.next_assignment(), s.next_assignment()
    assert s.result(mb, 7, 9) is None
    assert s.result(ma, 7, 3) == (100, (7, 3))  # equal hash -> lower nonce wins


# ---- the three programs over LSP ------------------------------------------------------

def test_config1_shape(oracle):
    srv, t = start_server(job_size=2500)
    eng = OracleEngine(oracle)
    start_miner(srv.port, eng)
    res = bclient.request(f"127.0.0.1:{srv.port}", "bradfitz", 9999, P)
    assert res == (1419516646206828, 9898)
    assert sorted(eng.calls) == [(0, 2499), (2500, 4999), (5000, 7499), (7500, 9999)]
    close_quietly(srv)


def test_many_clients_miners_drops_and_a_killed_miner(oracle):
    srv, t = start_server(job_size=3000)
    lspnet.SetReadDropPercent(10)
    lspnet.SetWriteDropPercent(10)
    engines = [OracleEngine(oracle, delay=0.02) for _ in range(3)]
    for e in engines:
        start_miner(srv.port, e)
    # a fourth miner that dies mid-job: once it holds a job its transport goes silent
    # without a Close (the in-process analogue of SIGKILL)
    box = {}
    got_job = threading.Event()

    class Doomed:
        calls = []

        def min(self, msg, lo, hi):
            self.calls.append((msg, lo, hi))
            box["client"]._loop.stop()
            got_job.set()
            time.sleep(3600)

    threading.Thread(target=bminer.run, args=(f"127.0.0.1:{srv.port}", Doomed(), P),
                     kwargs=dict(on_client=lambda c: box.setdefault("client", c)), daemon=True).start()
    results = {}

    def cl(i):
        results[i] = bclient.request(f"127.0.0.1:{srv.port}", f"client-{i:02d}", 20000 + 777 * i, P)

    threads = [threading.Thread(target=cl, args=(i,)) for i in range(6)]
    for x in threads:
        x.start()
    for x in threads:
        x.join(120)
    lspnet.SetReadDropPercent(0)
    lspnet.SetWriteDropPercent(0)
    for i in range(6):
        assert results[i] == oracle.min(f"client-{i:02d}".encode(), 0, 20000 + 777 * i), i
    # the killed miner held a job, and that exact job was redone by a live miner
    assert got_job.is_set() and len(Doomed.calls) == 1
    msg, lo, hi = Doomed.calls[0]
    assert any((lo, hi) in e.calls for e in engines)
    close_quietly(srv)


def test_lost_client_work_is_dropped(oracle):
    srv, t = start_server(job_size=1000)
    eng = OracleEngine(oracle, delay=0.05)
    start_miner(srv.port, eng)
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", P)
    c.Write(bitcoin.marshal(bitcoin.NewRequest("gone", 0, 99999)))  # 100 jobs
    time.sleep(0.3)
    c._loop.stop()  # the client vanishes
    time.sleep(P.EpochLimit * P.EpochMillis / 1000 + 0.5)
    n = len(eng.calls)
    time.sleep(0.5)
    assert len(eng.calls) <= n + 1 and n < 100  # the server stopped farming its jobs
    # and the server still serves others
    assert bclient.request(f"127.0.0.1:{srv.port}", "bradfitz", 9999, P) == (1419516646206828, 9898)
    close_quietly(srv)
