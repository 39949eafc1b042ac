"""CPU: the server's speculative job copies and its requeue cap (bitcoin/server.py
Scheduler; csrc/server_main.cpp mirrors it and runs the same cases in
tests/test_native_server.py).  VERDICT r05 items 1-2: on the reference's LSP parameters a
dropped Result waits up to an epoch (2 s) and a killed miner is noticed only after
EpochLimit silent epochs (10 s), so once nothing is left to hand out an idle miner takes a
copy of a job that is overdue; and a miner lost for reasons unrelated to a job must not
use up that job's requeue cap.
"""
import pytest

from bitcoin import server as bserver

GPU = 34.6e9


def sched(**kw):
    now = [0.0]
    s = bserver.Scheduler(**{"job_size": 1 << 34, "depth": 1, "copies": 3, **kw})
    s.clock = lambda: now[0]
    return s, now


def test_no_copy_while_work_is_left_or_before_a_job_is_overdue():
    s, now = sched()
    for m in (1, 2, 3):
        s.add_miner(m)
    s.add_request(client=100, data="a", lower=0, upper=(1 << 36) - 1)  # 4 jobs of 2^34
    got = [s.next_assignment() for _ in range(3)]
    assert all(g is not None for g in got) and s.next_assignment() is None
    # miner 1 answers after its job's time: it learns its rate, and the fourth job goes out
    now[0] = (1 << 34) / GPU
    assert s.result(1, 5, 1) is None
    m, j4, _ = s.next_assignment()
    assert m == 1 and j4.lower == 3 << 34
    assert s.next_assignment() is None  # nothing idle
    now[0] += 0.01
    assert s.result(2, 7, 2) is None  # miner 2 done: idle, but no job is overdue yet
    assert s.next_assignment() is None
    # miner 3's job was due at ~0.50 s (+ slack of a quarter job): a copy goes out after
    due = s.next_wakeup()
    assert due is not None and 0.55 < due < 0.75, due
    now[0] = due + 1e-6
    m, j, _ = s.next_assignment()
    assert m == 2 and j.lower == 2 << 34 and sorted(j.holders) == [2, 3] and s.speculated == 1


def test_first_copy_wins_and_the_late_one_is_ignored():
    s, now = sched()
    s.add_miner(1)
    s.add_miner(2)
    s.add_request(client=100, data="a", lower=0, upper=(1 << 34) - 1)  # one job
    m, job, _ = s.next_assignment()
    assert m == 1
    # teach the scheduler miner 1's rate from an earlier job of another request
    s.rates[1] = bserver.MinerRate(work=1 << 34, secs=(1 << 34) / GPU)
    now[0] = 5.0  # long past due: its Result is lost in the network
    m2, copy, _ = s.next_assignment()
    assert m2 == 2 and copy is job
    assert s.result(2, 42, 17) == (100, (42, 17))  # the copy answers first: request done
    assert s.result(1, 1, 1) is None              # the original's answer is ignored
    assert not s.requests and not s.miners[1] and not s.miners[2]


def test_copies_are_capped():
    s, now = sched(copies=2)
    for m in (1, 2, 3):
        s.add_miner(m)
        s.rates[m] = bserver.MinerRate(work=1 << 34, secs=(1 << 34) / GPU)
    s.add_request(client=100, data="a", lower=0, upper=(1 << 34) - 1)
    s.next_assignment()
    now[0] = 5.0
    assert s.next_assignment() is not None   # one copy
    now[0] = 50.0
    assert s.next_assignment() is None       # two live copies: the cap
    assert s.next_wakeup() is None


def test_a_lost_miner_whose_job_has_a_copy_requeues_nothing():
    s, now = sched()
    for m in (1, 2):
        s.add_miner(m)
        s.rates[m] = bserver.MinerRate(work=1 << 34, secs=(1 << 34) / GPU)
    s.add_request(client=100, data="a", lower=0, upper=(1 << 34) - 1)
    s.next_assignment()
    now[0] = 5.0
    s.next_assignment()
    note = s.lost(1)
    assert "still held" in note and "requeued" not in note
    r = next(iter(s.requests.values()))
    assert not r.requeued and r.inflight == 1
    assert s.result(2, 9, 9) == (100, (9, 9))


def test_only_the_job_being_computed_counts_toward_the_cap():
    """four miners lost one after another, each computing a different
    job of a busy request with a healthy request's job queued behind it (two jobs per
    miner): the healthy job never ran, so it is requeued four times without using up its
    cap, and no job is abandoned.  A job that is being computed each time its miner dies
    -- the poison case the cap exists for -- still ends its request."""
    s, now = sched(depth=2, copies=1)
    s.add_request(client=100, data="busy", lower=0, upper=(1 << 40) - 1)
    for m in (10, 11, 12, 13):
        s.add_miner(m)
    busy = [s.next_assignment() for _ in range(4)]
    assert [a[0] for a in busy] == [10, 11, 12, 13] and len({a[1].lower for a in busy}) == 4
    healthy = s.add_request(client=200, data="healthy", lower=0, upper=(1 << 34) - 1)
    m, job, _ = s.next_assignment()
    assert (m, job.req_id) == (10, healthy)
    for k in range(4):
        miner = 10 + k
        assert [j.req_id for j in s.miners[miner]] == [1, healthy], k  # computing busy, healthy behind
        note = s.lost(miner)
        assert f"request {healthy} requeued" in note and "abandoned" not in note, note
        a = s.next_assignment()
        if k < 3:
            assert (a[0], a[1].req_id) == (miner + 1, healthy)
    assert healthy in s.requests and s.requests[healthy].requeued[0].requeues == 0
    assert all(a[1].requeues == 1 for a in busy) and not s.abandoned
    # the poison case: the job is what each miner computes when it dies
    s2, _ = sched(depth=1, copies=1)
    s2.add_request(client=300, data="poison", lower=0, upper=99)
    for k in range(bserver.MAX_REQUEUES + 1):
        s2.add_miner(50 + k)
        assert s2.next_assignment()[0] == 50 + k
        note = s2.lost(50 + k)
    assert "abandoned" in note and list(s2.abandoned) == [300]


def test_four_unrelated_miner_deaths_at_default_epochs_do_not_abandon_a_request():
    """The same through the whole system model (tests/lsp_des.py) at the reference's LSP
    parameters: 8 GPU miners, 10% drops, four miners killed one after another mid-run
    (each death noticed 10 s later); every client still gets its Result."""
    import lsp
    import lsp_des
    reqs = [(f"client-{i:02d}", 0, 1 << 36) for i in range(8)]
    sch = bserver.make_scheduler(epoch_s=2.0)
    sim_kills = [(0.5 + 1.5 * k, 7 - k) for k in range(4)]
    r = lsp_des.run_system(sch, [GPU] * 8, 1, reqs, params=lsp.NewParams(), drop=0.10, seed=3,
                           kills=sim_kills)
    assert r["disconnected"] == 0 and len(r["done"]) == 8, r
    assert not sch.abandoned


def test_program_defaults():
    s = bserver.make_scheduler(epoch_s=2.0)
    assert (s.job_size, s.depth, s.copies, s.hedge) == (1 << 36, bserver.MINER_DEPTH, bserver.COPIES, "overdue")
    assert bserver.make_scheduler(epoch_s=0.2).job_size == 1 << 33
    assert bserver.default_job_size(0.04) == 1 << 30  # clamped


def test_program_defaults_env(monkeypatch):
    monkeypatch.setenv("GPUHASH_BACKUP", "0")
    monkeypatch.setenv("GPUHASH_MINER_DEPTH", "1")
    monkeypatch.setenv("GPUHASH_JOB_SIZE", "1000")
    s = bserver.make_scheduler()
    assert (s.job_size, s.depth, s.copies) == (1000, 1, 1)


@pytest.mark.parametrize("hedge", ["nope"])
def test_bad_hedge(hedge):
    with pytest.raises(ValueError):
        bserver.Scheduler(hedge=hedge)
