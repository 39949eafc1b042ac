"""GPU: the lowest-nonce tie rule at every reduction level, with REAL ties.

Real 64-bit SHA ties are unreachable, so libgpuhash_tietest.so is the same source built
with -DGPUHASH_TIE_TEST_BITS=4: the kernels keep only the top 4 bits of H0 (and zero
H1), so about one nonce in 16 shares the minimal key.  The expected answer is the
lowest nonce with the minimal truncated key (np.argmin returns the first index), which
exercises the in-lane scan order, the wave slow path (a lane's later r can have a lower
nonce than the next lane's current one), the workgroup LDS reduce, the candidate reduce
across workgroups and launches, and the host merge across calls.
"""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]


@pytest.fixture(scope="module")
def tie_engine():
    import gpuhash
    if not os.path.exists(gpuhash.TIETEST_LIB_PATH):
        pytest.fail("libgpuhash_tietest.so not built (make -C bitcoin-miner_amd)")
    eng = gpuhash.Engine(lib_path=gpuhash.TIETEST_LIB_PATH)
    yield eng
    eng.close()


def truncated(oracle, msg, lo, count):
    h = oracle.hash_range(msg, lo, count)
    return (h >> np.uint64(60)) << np.uint64(32)


def expect(oracle, msg, lo, hi):
    k = truncated(oracle, msg, lo, hi - lo + 1)
    i = int(np.argmin(k))  # first occurrence = lowest nonce
    return int(k[i]), lo + i


def test_tietest_build_is_the_one_loaded(tie_engine):
    assert b"TIE-TEST" in tie_engine._lib.gpuhash_version()


def test_truncated_hash_range(tie_engine, oracle):
    for m, lo, n in [(b"bradfitz", 999990000, 20000), (M120, 9999990000, 20000), (b"x" * 53, 0, 20000)]:
        assert (tie_engine.hash_range(m, lo, n) == truncated(oracle, m, lo, n)).all()


@pytest.mark.parametrize("rchunk", [0, 1, 7, 100])
def test_lowest_nonce_wins_ties(tie_engine, oracle, rchunk):
    rng = random.Random(rchunk)
    cases = [(b"bradfitz", 0, 3_000_000), (b"bradfitz", 999_000_000, 1_002_000_000),
             (M120, 999_000_000, 1_001_500_000), (b"y" * 56, 123, 1_500_000)]
    for _ in range(6):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 130)))
        lo = rng.randrange(0, 10 ** 12)
        cases.append((m, lo, lo + rng.randrange(1, 2_000_000)))
    for m, lo, hi in cases:
        assert tie_engine.min(m, lo, hi, rchunk=rchunk) == expect(oracle, m, lo, hi), (m, lo, hi)


def test_ties_where_minimum_appears_late(tie_engine, oracle):
    # start just after a key-0 nonce so the first minimal nonce is far from `lo` and is
    # found by a later lane / workgroup than many higher-keyed candidates
    m = b"bradfitz"
    base = 4_000_000_000
    k = truncated(oracle, m, base, 200_000)
    zeros = np.nonzero(k == 0)[0]
    gaps = np.diff(zeros)
    j = int(np.argmax(gaps))
    lo = base + int(zeros[j]) + 1
    hi = lo + 150_000
    assert tie_engine.min(m, lo, hi) == expect(oracle, m, lo, hi)


def test_merge_of_split_calls_keeps_lowest_nonce(tie_engine, oracle):
    import gpuhash.dist as gd
    m, lo, hi = b"bradfitz", 10 ** 9, 10 ** 9 + 4_000_000
    parts = [tie_engine.min(m, a, b) for a, b in gd.split_range(lo, hi, 5)]
    assert gd.merge_min(parts) == tie_engine.min(m, lo, hi) == expect(oracle, m, lo, hi)
