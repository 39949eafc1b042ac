"""CPU: the N>1 path (one process per GPU) with world_size-2 gloo process groups.

The per-rank search is stood in for by the oracle (this file is test infrastructure);
what is under test is gpuhash.dist: contiguous sharding, the 24-byte all_gather and
the lexicographic merge -- the same code bench.py runs across ranks on the GPU box.
tests/test_gpu_dist.py runs the same path with the HIP engine as the per-rank search.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

import gpuhash.dist as gd

U64 = (1 << 64) - 1


def test_split_range_tiles():
    for lo, hi, w in [(0, 9, 2), (0, 0, 2), (5, 5, 8), (0, (1 << 40) - 1, 8), (U64 - 2, U64, 8), (0, U64, 3)]:
        s = gd.split_range(lo, hi, w)
        got = [x for x in s if x is not None]
        assert got[0][0] == lo and got[-1][1] == hi
        for a, b in zip(got, got[1:]):
            assert b[0] == a[1] + 1
        counts = [b - a + 1 for a, b in got]
        assert max(counts) - min(counts) <= 1


M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]


def test_cost_balanced_split_through_the_abi():
    """split_range(..., msg_len) = gpuhash_shard_range: the engine's cost model (VERDICT r02
    item 5).  m = 45 crosses 1 -> 2 SHA blocks at 10 digits, so of a window centred on
    10^9 the 2-block half costs more and its shard holds fewer nonces."""
    lo, hi = 10**9 - (1 << 27), 10**9 + (1 << 27)
    for w in (2, 3, 8):
        s = gd.split_range(lo, hi, w, msg_len=45)
        got = [x for x in s if x is not None]
        assert got[0][0] == lo and got[-1][1] == hi
        for a, b in zip(got, got[1:]):
            assert b[0] == a[1] + 1
    s2 = gd.split_range(lo, hi, 2, msg_len=45)
    assert s2[0][1] > 10**9  # the cheap 9-digit half plus part of the 10-digit one
    assert (s2[0][1] - s2[0][0]) > 1.2 * (s2[1][1] - s2[1][0])
    # a one-block message at one digit count: equal counts within one nonce
    s3 = gd.split_range(10**9, 2 * 10**9 - 1, 4, msg_len=8)
    counts = [b - a + 1 for a, b in s3]
    assert max(counts) - min(counts) <= 1
    # empty shards when the range has fewer nonces than ranks
    s4 = gd.split_range(5, 6, 4, msg_len=8)
    assert [x for x in s4 if x is not None] == [(5, 5), (6, 6)]
    with pytest.raises(Exception):
        gd.split_range(0, 1, 0, msg_len=8)


def test_split_under_a_layout_policy():
    """the cuts depend on the layout policy (a digit group's cost is its
    layout's), so gpuhash_shard_range_policy cuts as gpuhash_min does under that policy;
    AUTO is gpuhash_shard_range.  Over [0, 2^40) of 'bradfitz' the 12-digit groups run
    tail-digit launches under AUTO and not under TAIL_NEVER, so the two cut differently."""
    import gpuhash
    lo, hi = 0, (1 << 40) - 1
    auto = gd.split_range(lo, hi, 8, msg_len=8)
    assert gd.split_range(lo, hi, 8, msg_len=8, policy=gpuhash.LAYOUT_AUTO) == auto
    never = gd.split_range(lo, hi, 8, msg_len=8, policy=gpuhash.LAYOUT_TAIL_NEVER)
    assert never != auto
    for cuts in (auto, never):
        assert cuts[0][0] == lo and cuts[-1][1] == hi
        assert all(b[0] == a[1] + 1 for a, b in zip(cuts, cuts[1:]))
    with pytest.raises(gpuhash.GpuHashError):
        gpuhash.shard_range(8, 0, 10, 2, gpuhash.LAYOUT_TAIL_ALWAYS | gpuhash.LAYOUT_TAIL_NEVER)


def test_weak_range():
    assert gd.weak_range(0, 1 << 32, 0) == (0, (1 << 32) - 1)
    assert gd.weak_range(0, 1 << 37, 7) == (7 << 37, (1 << 40) - 1)
    with pytest.raises(ValueError):
        gd.weak_range(U64, 2, 0)


def test_merge_min_tie_goes_to_lowest_nonce():
    assert gd.merge_min([(5, 10), (3, 99), (3, 7), None, (4, 1)]) == (3, 7)
    assert gd.merge_min([(U64, U64), (U64, 3)]) == (U64, 3)
    with pytest.raises(ValueError):
        gd.merge_min([None, None])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q):
    import torch.distributed as dist
    import hash_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    oracle = hash_oracle.load_c_oracle()
    out = []
    for msg, lo, hi in cases:
        out.append(gd.distributed_min(lambda a, b: oracle.min(msg, a, b), lo, hi))
        # the engine's cost-balanced cut points (host-only ABI call, no device needed)
        out.append(gd.distributed_min(lambda a, b: oracle.min(msg, a, b), lo, hi, msg_len=len(msg)))
    # a rank with an empty shard still joins the gather
    out.append(gd.distributed_min(lambda a, b: oracle.min(b"x", a, b), 7, 7))
    q.put((rank, out))
    dist.destroy_process_group()


def test_gloo_world2_matches_single_range(oracle):
    cases = [(b"bradfitz", 0, 9999), (b"msg", 0, 2), (M120, 999999000, 1000001000), (b"", U64 - 5000, U64),
             (M120[:45], 999998000, 1000002000)]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [r for m, lo, hi in cases for r in [oracle.min(m, lo, hi)] * 2] + [oracle.min(b"x", 7, 7)]
    assert res[0] == res[1] == want
