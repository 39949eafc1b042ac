"""CPU: the N>1 path (one process per GPU) with world_size-2 gloo process groups.

The per-rank search is stood in for by the oracle (this file is test infrastructure);
what is under test is gpuhash.dist: contiguous sharding, the 24-byte all_gather and
the lexicographic merge -- the same code bench.py runs over RCCL on the GPU box.
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
    # a rank with an empty shard still joins the gather
    out.append(gd.distributed_min(lambda a, b: oracle.min(b"x", a, b), 7, 7))
    q.put((rank, out))
    dist.destroy_process_group()


def test_gloo_world2_matches_single_range(oracle):
    cases = [(b"bradfitz", 0, 9999), (b"msg", 0, 2), ((b"The quick brown fox jumps over the lazy dog. " * 3)[:120],
                                                      999999000, 1000001000), (b"", U64 - 5000, U64)]
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
    want = [oracle.min(m, lo, hi) for m, lo, hi in cases] + [oracle.min(b"x", 7, 7)]
    assert res[0] == res[1] == want
