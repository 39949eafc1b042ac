"""CPU: the server's job sizing, driven as a discrete-event simulation of miners with
given rates (no sockets, no GPU).  What is checked: every request's jobs tile its range
exactly, and the makespans of fixed-size and adaptive (per-miner, SURVEY 8(f) row 2:
"chunk sizes retuned for GPU-scale throughput") chunking on the shapes that matter:
  * one big request on an 8-GPU node (fixed 2^34 jobs leave half the GPUs idle);
  * GPU miners mixed with CPU miners running the reference's loop (a fixed GPU-sized
    job on a CPU miner takes minutes);
  * BASELINE config 5's shape, 16 clients x 2^36 on 8 GPU miners (adaptive must not
    lose to the fixed size that suits it).
Rates: one MI355X = 34.6 GH/s (profiles/r02_bench_config2.json); a CPU miner running
the reference loop on 16 cores = 0.08 GH/s (the bench's cpu_baseline_multicore).
"""
import heapq
import random

import pytest

from bitcoin import server as bserver

GPU = 34.6e9
CPU = 0.08e9
LATENCY = 0.002  # one LSP round trip + one gpuhash_min call


def leg(rng, drop, epoch, latency=LATENCY):
    """One direction of a job's round trip over LSP: half the latency, plus, for each of
    its two messages (Data, Ack) that lspnet drops, a wait for the next epoch's resend."""
    t = latency / 2
    for _ in range(2):
        if rng.random() < drop:
            t += rng.uniform(0, epoch)
            while rng.random() < drop:
                t += epoch
    return t


def simulate(sched, rates, requests, latency=LATENCY, drop=0.0, epoch=0.5, seed=1):
    """Runs `sched` until every request is answered; returns ({client: finish time},
    {req: [(lo, hi), ...]}, number of jobs).  A miner works its jobs in order (a job
    waits for the previous one); each leg of a round trip may lose messages."""
    rng = random.Random(seed)
    now = [0.0]
    sched.clock = lambda: now[0]
    for m in rates:
        sched.add_miner(m)
    for i, (lo, hi) in enumerate(requests):
        sched.add_request(client=1000 + i, data=f"r{i}", lower=lo, upper=hi)
    events, done, cuts, seq = [], {}, {}, 0
    free_at = {m: 0.0 for m in rates}

    def dispatch():
        nonlocal seq
        while True:
            a = sched.next_assignment()
            if a is None:
                return
            m, job, data = a
            cuts.setdefault(data, []).append((job.lower, job.upper))
            start = max(now[0] + leg(rng, drop, epoch, latency), free_at[m])
            free_at[m] = start + (job.upper - job.lower + 1) / rates[m]
            t = free_at[m] + leg(rng, drop, epoch, latency)
            seq += 1
            heapq.heappush(events, (t, seq, m, job))

    dispatch()
    while events:
        t, _, m, job = heapq.heappop(events)
        now[0] = t
        # any fixed (hash, nonce) per job: merging is tested elsewhere, timing here
        res = sched.result(m, (job.lower * 2654435761) % (1 << 64), job.lower)
        if res is not None:
            done[res[0]] = t
        dispatch()
    return done, cuts, seq


def tiles(cuts, lo, hi):
    c = sorted(cuts)
    return c[0][0] == lo and c[-1][1] == hi and all(a[1] + 1 == b[0] for a, b in zip(c, c[1:]))


def fixed():
    return bserver.Scheduler(job_size=1 << 34)


def adaptive():
    return bserver.Scheduler(sizing=bserver.Sizing())


def test_one_big_request_uses_every_gpu():
    rates = {m: GPU for m in range(8)}
    req = [(0, (1 << 36) - 1)]
    done_f, cuts_f, _ = simulate(fixed(), rates, req)
    done_a, cuts_a, njobs = simulate(adaptive(), rates, req)
    assert tiles(cuts_f["r0"], *req[0]) and tiles(cuts_a["r0"], *req[0])
    ideal = (1 << 36) / (8 * GPU)
    # fixed 2^34 jobs: 4 jobs for 8 GPUs, twice the ideal time
    assert done_f[1000] == pytest.approx(2 * ideal, rel=0.05)
    assert done_a[1000] < 1.25 * ideal, (done_a, ideal)  # measured 1.16
    assert njobs < 40  # and not by shredding the range


def test_gpu_and_cpu_miners_together():
    rates = {0: GPU, 1: GPU, 2: CPU, 3: CPU, 4: CPU}
    req = [(0, (1 << 36) - 1)]
    done_f, _, _ = simulate(fixed(), rates, req)
    done_a, cuts_a, _ = simulate(adaptive(), rates, req)
    assert tiles(cuts_a["r0"], *req[0])
    assert done_f[1000] > 200  # a 2^34 job on a CPU miner: ~215 s
    # adaptive: the GPUs do the bulk, CPU miners take jobs of ~0.5 s
    assert done_a[1000] < 1.3 * (1 << 36) / (2 * GPU + 3 * CPU) + 1.0, done_a


def test_two_big_requests_lose_little():
    # 2 x 2^36 on 8 GPUs: fixed 2^34 jobs are a perfect fit (8 jobs, 8 GPUs); the
    # adaptive probes and end game cost a few per cent at most
    rates = {m: GPU for m in range(8)}
    reqs = [(0, (1 << 36) - 1)] * 2
    done_f, _, _ = simulate(fixed(), rates, reqs)
    done_a, _, _ = simulate(adaptive(), rates, reqs)
    assert max(done_a.values()) <= 1.05 * max(done_f.values())


def test_config5_shape_is_not_slower():
    rates = {m: GPU for m in range(8)}
    reqs = [(0, 1 << 36) for _ in range(16)]
    done_f, _, _ = simulate(fixed(), rates, reqs)
    done_a, cuts_a, _ = simulate(adaptive(), rates, reqs)
    for i in range(16):
        assert tiles(cuts_a[f"r{i}"], 0, 1 << 36)
    assert max(done_a.values()) <= 1.01 * max(done_f.values()), (max(done_a.values()), max(done_f.values()))


def test_rate_follows_a_shared_gpu():
    """A miner whose GPU starts being shared (its rate halves) gets smaller jobs."""
    s = adaptive()
    now = [0.0]
    s.clock = lambda: now[0]
    s.add_miner(1)
    s.add_request(client=9, data="x", lower=0, upper=(1 << 50) - 1)
    sizes = []
    rate = GPU
    for k in range(12):
        m, job, _ = s.next_assignment()
        n = job.upper - job.lower + 1
        sizes.append(n)
        if k == 6:
            rate = GPU / 2
        now[0] += n / rate + LATENCY
        s.result(m, 1, job.lower)
    assert sizes[0] == bserver.Sizing().probe
    full = GPU * bserver.JOB_SECONDS
    assert 0.8 * full < sizes[6] < 1.05 * full, sizes
    assert sizes[-1] < 0.7 * full, sizes  # converged toward the halved rate


def test_lost_miner_forgets_its_rate_and_fixed_mode_is_unchanged():
    s = adaptive()
    s.add_miner(1)
    s.add_request(client=9, data="x", lower=0, upper=(1 << 40) - 1)
    m, job, _ = s.next_assignment()
    s.result(m, 1, job.lower)
    assert 1 in s.rates
    s.lost(1)
    assert 1 not in s.rates and 1 not in s.done_at
    f = fixed()
    f.add_miner(1)
    f.add_request(client=9, data="x", lower=0, upper=(1 << 40) - 1)
    assert f.next_assignment()[1].upper == (1 << 34) - 1


def test_depth_two_hides_round_trips_and_resends():
    """Two jobs per miner: the next Request waits in the miner's connection while it
    computes.  Config 5's shape with 10% drops on every message and 0.5 s epochs (the
    system bench's), on an 8-GPU node (one miner per GPU) and on one GPU shared by 8."""
    reqs = [(0, (1 << 36) - 1)] * 16
    total = 16 * (1 << 36)
    for rates, gain in (({m: GPU for m in range(8)}, 1.10), ({m: GPU / 8 for m in range(8)}, 1.01)):
        ghs = {}
        for depth in (1, 2):
            done, cuts, _ = simulate(bserver.Scheduler(job_size=1 << 34, depth=depth), rates, reqs,
                                     drop=0.1, epoch=0.5)
            assert all(tiles(cuts[f"r{i}"], 0, (1 << 36) - 1) for i in range(16))
            ghs[depth] = total / max(done.values()) / 1e9
        assert ghs[2] >= gain * ghs[1], ghs
    # lossless: depth 2 costs nothing
    rates = {m: GPU for m in range(8)}
    d1 = max(simulate(bserver.Scheduler(job_size=1 << 34, depth=1), rates, reqs)[0].values())
    d2 = max(simulate(bserver.Scheduler(job_size=1 << 34, depth=2), rates, reqs)[0].values())
    assert d2 <= 1.005 * d1


def test_depth_two_bookkeeping():
    s = bserver.Scheduler(job_size=10, depth=2)
    s.add_request(client=100, data="a", lower=0, upper=99)
    s.add_miner(1)
    s.add_miner(2)
    got = [s.next_assignment() for _ in range(4)]
    assert s.next_assignment() is None  # both miners hold two jobs
    assert sorted(m for m, _, _ in got) == [1, 1, 2, 2]
    first = [j for m, j, _ in got if m == 1]
    assert s.result(1, 7, first[0].lower) is None  # a Result is the OLDEST job's
    assert list(s.miners[1]) == [first[1]]
    two = [j for m, j, _ in got if m == 2]
    note = s.lost(2)  # both of its jobs go back, oldest first
    assert note.count("requeued") == 2
    r = next(iter(s.requests.values()))
    assert list(r.requeued) == two and r.inflight == 1
