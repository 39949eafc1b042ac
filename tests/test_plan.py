"""CPU: the host-side planner (bitcoin-miner_amd/csrc/plan.cpp) without a GPU.

libgpuhash_hostcheck.so exposes the launch plan libgpuhash.so would execute and replays
the per-nonce data flow of a scan kernel from each launch's descriptor (midstates,
uniform words, lane/loop digit insertion, extra padding block).  Checked against the
oracle: exact tiling of [lower, upper], every kernel variant, message lengths across
block boundaries, digit-count boundaries, and the 2^64-1 edge.
"""
import ctypes
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "bitcoin-miner_amd", "lib")
# tests/test_sanitizers.py reruns this module against the ASan/UBSan build
HC = os.environ.get("GPUHASH_HOSTCHECK_LIB") or os.path.join(LIBDIR, "libgpuhash_hostcheck.so")
U64 = (1 << 64) - 1
M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
u64 = ctypes.c_uint64


class Info(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_int) for n in "J C2 EX d q s".split()]
                + [(n, u64) for n in "lo hi base".split()]
                + [(n, ctypes.c_uint32) for n in "nblocks R rchunk nrchunks p_first p_last r_first r_last".split()]
                + [(n, ctypes.c_uint32) for n in "stride tail".split()])


@pytest.fixture(scope="module")
def hc():
    if not os.path.exists(HC):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "bitcoin-miner_amd"),
                               os.path.relpath(HC, os.path.join(ROOT, "bitcoin-miner_amd"))])
    lib = ctypes.CDLL(HC)
    cp, u32 = ctypes.c_char_p, ctypes.c_uint32
    lib.gpuhash_plan_count.argtypes = [cp, u64, u64, u64, u32]
    lib.gpuhash_plan_get.argtypes = [cp, u64, u64, u64, u32, ctypes.c_int, ctypes.POINTER(Info)]
    lib.gpuhash_plan_all.argtypes = [cp, u64, u64, u64, u32, ctypes.POINTER(Info), ctypes.c_int]
    lib.hostcheck_desc_hash.argtypes = [cp, u64, u64, u64, u32, ctypes.c_int, u64, ctypes.POINTER(u64)]
    lib.gpuhash_shard.argtypes = [u64, u64, u64, ctypes.c_int, ctypes.POINTER(u64),
                                  ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_int)]
    lib.gpuhash_plan_cost.argtypes = [cp, u64, u64, u64]
    lib.gpuhash_plan_cost.restype = ctypes.c_double
    lib.hostcheck_set_layout_policy.argtypes = [ctypes.c_int]
    lib.hostcheck_set_layout_policy(AUTO)
    return lib


AUTO, UNIFORM, CLASSIC, LANETABLE = 0, 1, 2, 3


def plan(hc, m, a, b, rchunk=0):
    n = hc.gpuhash_plan_count(m, len(m), a, b, rchunk)
    arr = (Info * n)()
    assert hc.gpuhash_plan_all(m, len(m), a, b, rchunk, arr, n) == n
    return list(arr)


def count(l):
    """Nonces of launch l (a tail-digit launch covers every stride-th nonce of [lo, hi])."""
    return (l.hi - l.lo) // l.stride + 1


def some_nonce(rng, l):
    return l.lo + l.stride * rng.randrange(count(l))


def assert_tiles(p, a, b):
    """The launches cover [a, b] exactly once, in order: plain launches tile it, and each
    run of tail-digit launches (one digit group) covers its span [A, B] as ten residue
    classes, class t's k = nonce / 10 ranges tiling [ceil((A-t)/10), floor((B-t)/10)]."""
    i, nxt = 0, a
    while i < len(p):
        l = p[i]
        if l.stride == 1:
            assert l.lo == nxt, (i, l.lo, nxt)
            nxt = l.hi + 1
            i += 1
            continue
        j = i
        while j < len(p) and p[j].stride != 1 and p[j].d == l.d:
            j += 1
        run = p[i:j]
        A, B = nxt, max(x.hi for x in run)
        assert min(x.lo for x in run) >= A and B <= b
        for t in range(10):
            ks = sorted(((x.lo - t) // 10, (x.hi - t) // 10) for x in run if x.tail == t)
            assert all(x.lo % 10 == t and x.hi % 10 == t and x.stride == 10 for x in run if x.tail == t)
            ka, kb = (A - t + 9) // 10 if A > t else 0, (B - t) // 10
            if ka > kb:
                assert not ks
                continue
            assert ks and ks[0][0] == ka and ks[-1][1] == kb, (t, ks, ka, kb)
            for (x0, x1), (y0, y1) in zip(ks, ks[1:]):
                assert y0 == x1 + 1
        assert sum(count(x) for x in run) == B - A + 1
        nxt = B + 1
        i = j
    assert nxt == b + 1


def desc_hash(hc, m, a, b, i, n, rchunk=0):
    o = u64()
    assert hc.hostcheck_desc_hash(m, len(m), a, b, rchunk, i, n, ctypes.byref(o)) == 0
    return o.value


def test_plan_tiles_range_and_layouts_are_legal(hc):
    rng = random.Random(11)
    for _ in range(600):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 200)))
        a = rng.randrange(0, U64)
        b = min(U64, a + rng.randrange(0, 10 ** rng.randrange(0, 13)))
        p = plan(hc, m, a, b)
        assert_tiles(p, a, b)
        for l in p:
            if l.C2 == 3:  # lane table: lanes = W_0/W_1 digits, loop = block B-1 digits
                assert l.J == 1 and 5 <= l.q <= 8 and 1 <= l.s <= 8 and not l.EX
                RQ = 10 ** l.q
                assert 1 <= l.R <= 1024 and l.r_first == 0 and l.r_last == l.R - 1
                assert l.lo == l.base + l.p_first and l.hi == l.base + (l.R - 1) * RQ + l.p_last
                assert l.p_first <= l.p_last < RQ
                # a rectangle: one loop value, or every lane value of each loop value
                assert l.R == 1 or (l.p_first == 0 and l.p_last == RQ - 1)
                assert l.nblocks == (l.p_last - l.p_first) // 256 + 1
                continue
            if l.C2 == 2:  # two-word uniform loop: W_0 (4 digits) + W_1 (1..4 digits)
                assert l.J == 1 and 5 <= l.q <= 8 and 3 <= l.s <= 8 and l.s + l.q <= 12
            else:
                assert 1 <= l.q <= 4 and 0 <= l.s <= 8 and l.s + l.q <= 10
            assert not (l.C2 and l.J > 1) and not (l.EX and l.J < 13) and not (l.C2 and l.EX)
            assert l.R == 10 ** l.q
            assert (l.lo - l.tail) // l.stride == l.base + l.p_first * l.R + l.r_first
            assert (l.hi - l.tail) // l.stride == l.base + l.p_last * l.R + l.r_last
            if l.stride != 1:  # tail-digit launch: plain, the loop word's four digits
                assert l.stride == 10 and l.q == 4 and not l.C2 and l.tail < 10
            assert l.nblocks == ((l.p_last - l.p_first) // 256 + 1) * l.nrchunks
            assert l.nrchunks * l.rchunk >= l.R


@pytest.mark.parametrize("policy", [AUTO, UNIFORM, CLASSIC, LANETABLE])
def test_descriptor_replay_matches_oracle(hc, oracle, policy):
    hc.hostcheck_set_layout_policy(policy)
    rng = random.Random(5)
    seen = set()
    for _ in range(1500):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 200)))
        d = rng.randrange(1, 21)
        lo = 0 if d == 1 else 10 ** (d - 1)
        hi = min(10 ** d - 1, U64)
        a = rng.randrange(lo, hi + 1)
        b = min(hi, a + rng.randrange(0, 10 ** rng.randrange(0, 12)))
        for i, l in enumerate(plan(hc, m, a, b)):
            seen.add((l.J, l.C2, l.EX))
            for n in {l.lo, l.hi, some_nonce(rng, l)}:
                assert desc_hash(hc, m, a, b, i, n) == oracle.hash(m, n), (m, a, b, i, n)
    hc.hostcheck_set_layout_policy(AUTO)
    # the reachable (J, C2, EX) variants of each policy were all exercised: 14 plain, 3
    # extra-block, the K+W table (C2 = 1, J = 0), and per policy the J = 1 straddles --
    # UNIFORM: C2 = 2 and 3; AUTO: C2 = 1 (narrow searches) and 3 (and 2 on searches of
    # > 65536 block B-1 values, which this test's ranges rarely reach); CLASSIC: C2 = 1;
    # LANETABLE: C2 = 3 only
    want = {UNIFORM: {(1, 2, 0), (1, 3, 0)}, AUTO: {(1, 1, 0), (1, 3, 0)},
            CLASSIC: {(1, 1, 0)}, LANETABLE: {(1, 3, 0)}}[policy]
    straddle = {v for v in seen if v[0] == 1 and v[1] >= 1}
    assert straddle <= want | {(1, 2, 0)} and want - {(1, 2, 0)} <= straddle, sorted(seen)
    assert len(seen - straddle) == 18, sorted(seen)


def _header_rule():
    """The layout-policy rule as include/gpuhash.h states it (the ONE statement of it,
    VERDICT r03 item 4): GPUHASH_LANETABLE_MAX and the four policy lines."""
    import re
    h = open(os.path.join(ROOT, "include", "gpuhash.h")).read()
    cap = int(re.search(r"#define GPUHASH_LANETABLE_MAX (\d+)u", h).group(1))
    block = h[h.index("Layout choice for a digit group"):h.index("#define GPUHASH_LAYOUT_AUTO")]
    rule = " ".join(" ".join(re.sub(r"^\s*\*\s?", "", ln) for ln in block.splitlines()).split())
    return cap, rule


def test_layout_policy_for_straddling_j1(hc):
    """J = 1 straddles (4 + q1 digits in block B's W_0/W_1, the rest in block B-1), checked
    against the rule include/gpuhash.h states: AUTO takes the classic layout (C2 = 1) when
    span < 2 * RQ, the two-word loop (C2 = 2) when block B-1 holds >= 3 digits and
    N = (span - 1) / RQ + 2 > GPUHASH_LANETABLE_MAX, else the lane table (C2 = 3); UNIFORM
    C2 = 2 whenever block B-1 holds >= 3 digits; CLASSIC C2 = 1; LANETABLE C2 = 3 up to
    the same cap, C2 = 2 beyond it (uncapped, a wide LANETABLE search asked
    for ~640 MB of p-table)."""
    cap, rule = _header_rule()
    assert cap == 65536
    for line in ("AUTO (default) span < 2 * RQ -> C2 = 1 (classic)",
                 "else nb1 >= 3 and N > GPUHASH_LANETABLE_MAX -> C2 = 2 (two-word loop)",
                 "else -> C2 = 3 (lane table)",
                 "UNIFORM nb1 >= 3 -> C2 = 2, else C2 = 3",
                 "CLASSIC C2 = 1 always",
                 "LANETABLE C2 = 3 up to N = GPUHASH_LANETABLE_MAX, C2 = 2 beyond it",
                 "N = (span - 1) / RQ + 2"):
        assert line in rule, line
    pick = lambda m, a, b: {(l.J, l.C2) for l in plan(hc, m, a, b)}
    # m = 59, d = 12: 4 digits in block 0, 8 in block 1 (RQ = 10^8): at most 9000 values
    m = b"y" * 59
    lo = 10 ** 11
    narrow, wide = (lo, lo + 10 ** 9), (lo, lo + 5 * 10 ** 11)
    assert pick(m, *narrow) == {(1, 3)} and pick(m, *wide) == {(1, 3)}
    # m = 56, d = 12: 7 digits in block 0 (nb1 = 7), 5 in block 1 (RQ = 10^5); the cap's
    # edge: N = cap -> lane table, N = cap + 1 -> two-word loop
    m56, RQ = b"z" * 56, 10 ** 5
    at_cap = lo + (cap - 1) * RQ - 1  # span - 1 = (cap - 1) * RQ - 1 -> N = cap
    assert pick(m56, lo, at_cap) == {(1, 3)}
    assert pick(m56, lo, at_cap + 1) == {(1, 2)}
    # fewer than 2 block B-1 values' worth of nonces: the classic layout
    assert pick(m, lo, lo + 10 ** 8) == {(1, 1)} and pick(m, lo, lo + 2 * 10 ** 8) == {(1, 3)}
    assert pick(m, lo, lo + 2 * 10 ** 8 - 2) == {(1, 1)}  # span = 2 * RQ - 1
    try:
        hc.hostcheck_set_layout_policy(UNIFORM)
        assert pick(m, *narrow) == {(1, 2)}
        assert pick(b"q" * 61, 10 ** 9, 10 ** 9 + 10 ** 7) == {(1, 3)}  # 2 digits in block 0
        hc.hostcheck_set_layout_policy(CLASSIC)
        assert pick(m, *wide) == {(1, 1)} and pick(m, *narrow) == {(1, 1)}
        hc.hostcheck_set_layout_policy(LANETABLE)
        assert pick(m, *wide) == {(1, 3)} and pick(m, lo, lo + 10 ** 8) == {(1, 3)}
        assert pick(m56, lo, at_cap) == {(1, 3)} and pick(m56, lo, at_cap + 1) == {(1, 2)}
        # ADVICE r03's example: q = 5 over 10^12 nonces stays bounded (C2 = 2, not a
        # 10^7-entry p-table)
        assert pick(m56, lo, lo + 10 ** 12) == {(1, 2)}
    finally:
        hc.hostcheck_set_layout_policy(AUTO)


@pytest.mark.parametrize("mlen", [0, 8, 44, 45, 53, 54, 55, 56, 63, 64, 110, 119, 120, 127, 128, 180])
def test_every_digit_count_and_message_length(hc, oracle, mlen):
    m = bytes((i * 37 + 11) % 256 for i in range(mlen))
    for d in range(1, 21):
        lo = 0 if d == 1 else 10 ** (d - 1)
        hi = min(10 ** d - 1, U64)
        for a, b in [(lo, min(hi, lo + 1234)), (max(lo, hi - 777), hi)]:
            for i, l in enumerate(plan(hc, m, a, b)):
                for n in (l.lo, l.hi):
                    assert desc_hash(hc, m, a, b, i, n) == oracle.hash(m, n)


@pytest.mark.parametrize("mlen", [1000, 1299, 1300, 4093, (1 << 20) - 5, 1 << 20])
def test_long_messages(hc, oracle, mlen):
    # the LSP packet budget caps real messages near 1.3 KB; the host
    # midstate covers every block before the digits, up to GPUHASH_MAX_MSG = 1 MiB
    m = bytes((i * 131 + 7) % 256 for i in range(mlen))
    for d in (1, 9, 10, 12, 20):
        lo = 0 if d == 1 else 10 ** (d - 1)
        hi = min(10 ** d - 1, U64)
        a, b = lo, min(hi, lo + 99_999)
        for i, l in enumerate(plan(hc, m, a, b)):
            for n in (l.lo, l.hi):
                assert desc_hash(hc, m, a, b, i, n) == oracle.hash(m, n)


def test_wide_ranges_plan(hc):
    for a, b in [(0, (1 << 40) - 1), (0, (1 << 32) - 1), (U64 - 10 ** 12, U64)]:
        p = plan(hc, b"bradfitz", a, b)
        assert_tiles(p, a, b)
        assert sum(count(l) for l in p) == b - a + 1


def test_rchunk_override(hc, oracle):
    m = b"bradfitz"
    for rc in (1, 7, 10, 33, 1000):
        for i, l in enumerate(plan(hc, m, 123456789, 123499999, rc)):
            assert l.rchunk == min(rc, l.R)
            assert desc_hash(hc, m, 123456789, 123499999, i, l.hi, rc) == oracle.hash(m, l.hi)


def shards(hc, mlen, a, b, n):
    lo, hi, em = (u64 * n)(), (u64 * n)(), (ctypes.c_int * n)()
    assert hc.gpuhash_shard(mlen, a, b, n, lo, hi, em) == 0
    return [None if em[i] else (lo[i], hi[i]) for i in range(n)]


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_shards_tile_range(hc, n):
    rng = random.Random(n)
    cases = [(0, (1 << 40) - 1), (0, (1 << 32) - 1), (5, 9), (0, 0), (U64 - 3, U64), (0, U64)]
    cases += [(x, x + rng.randrange(0, 10 ** 15)) for x in (rng.randrange(0, 10 ** 18) for _ in range(20))]
    for a, b in cases:
        s = [x for x in shards(hc, 8, a, b, n) if x is not None]
        assert s[0][0] == a and s[-1][1] == b
        for x, y in zip(s, s[1:]):
            assert y[0] == x[1] + 1
        assert all(lo <= hi for lo, hi in s)


def test_shards_balance_config4(hc):
    # config 4: [0, 2^40) over 8 GPUs.  d=12 and d=13 layouts cost within a few %,
    # so the cost-balanced shards hold nearly equal nonce counts
    s = shards(hc, 8, 0, (1 << 40) - 1, 8)
    counts = [hi - lo + 1 for lo, hi in s]
    assert max(counts) / min(counts) < 1.03


def _shard_costs(hc, msg, a, b, n):
    return [hc.gpuhash_plan_cost(msg, len(msg), lo, hi) for lo, hi in
            (x for x in shards(hc, len(msg), a, b, n) if x is not None)]


@pytest.mark.parametrize("policy", [AUTO, AUTO | 16, AUTO | 32])
def test_shard_costs_follow_each_shards_plan(hc, policy):
    """a shard is priced by the layouts ITS plan uses.  Mid-size ranges (2^33 to
    2^36 over 8 devices) give shards below the tail-digit span (2^33), so their 8- and
    12-digit 'bradfitz' nonces run the plain one-digit-loop layout, not the tail-digit
    launches a whole digit group would get; under TAIL_ALWAYS / TAIL_NEVER the plans follow
    the flag.  Across a digit boundary whose two groups run different layouts, the cost
    of every shard's own plan (plan_cost, the same model) stays within 0.5% of the mean."""
    hc.hostcheck_set_layout_policy(policy)
    try:
        for msg, a, b in [(b"bradfitz", 10 ** 11 - (1 << 34), 10 ** 11 + (1 << 34)),
                          (b"bradfitz", 10 ** 11 - (1 << 32), 10 ** 11 + (1 << 35)),
                          (b"bradfitz", 10 ** 7 - (1 << 22), 10 ** 7 + (1 << 33)),
                          (M120[:45], 10 ** 9 - (1 << 29), 10 ** 9 + (1 << 33)),
                          (b"bradfitz", 0, (1 << 40) - 1)]:
            costs = _shard_costs(hc, msg, a, b, 8)
            mean = sum(costs) / len(costs)
            assert max(costs) / mean < 1.005 and min(costs) / mean > 0.995, (msg, a, b, costs)
    finally:
        hc.hostcheck_set_layout_policy(AUTO)


@pytest.mark.parametrize("mlen", [61, 62, 125, 126])
def test_lane_table_straddles(hc, oracle, mlen):
    """The layouts C2 = 3 is for: block B-1 holds 1-2 digits (message lengths = 61, 62 mod
    64, 6-10 digits), with rectangles split at partial first/last loop values, and long
    loops split at 1024 p-table entries."""
    m = bytes((i * 29 + 3) % 256 for i in range(mlen))
    seen = 0
    for d in range(5, 12):
        lo, hi = 10 ** (d - 1), 10 ** d - 1
        rng = random.Random(d * 1000 + mlen)
        for a, b in [(lo, hi), (lo + 12345, hi - 54321), (rng.randrange(lo, hi), None)]:
            if b is None:
                b = min(hi, a + rng.randrange(1, 10 ** 6))
            p = plan(hc, m, a, b)
            assert_tiles(p, a, b)
            for i, l in enumerate(p):
                seen += l.C2 == 3
                pts = {l.lo, l.hi, some_nonce(rng, l)}
                for n in pts:
                    assert desc_hash(hc, m, a, b, i, n) == oracle.hash(m, n), (mlen, d, a, b, i, n)
    assert seen > 0


TAIL_ALWAYS, TAIL_NEVER = 16, 32


def test_tail_digit_layouts_replay(hc, oracle):
    """Tail-digit launches (include/gpuhash.h): with the last digit fixed
    per launch, every launch of every qualifying digit group -- message lengths 0-129, so
    the one-digit last word lands in every word position and block, extra padding block
    included -- replays bit-exact against the oracle, and the ten residue classes tile
    the range."""
    rng = random.Random(37)
    hc.hostcheck_set_layout_policy(AUTO | TAIL_ALWAYS)
    try:
        tails, variants = 0, set()
        for mlen in range(0, 130):
            m = bytes(rng.randrange(256) for _ in range(mlen))
            for d in range(6, 21):
                lo_d, hi_d = 10 ** (d - 1), min(10 ** d - 1, U64)
                a = rng.randrange(lo_d, hi_d + 1)
                b = min(hi_d, a + rng.randrange(0, 10 ** rng.randrange(1, 6)))
                p = plan(hc, m, a, b)
                assert_tiles(p, a, b)
                for i, l in enumerate(p):
                    if l.stride == 1:
                        continue
                    tails += 1
                    variants.add((l.J, l.EX))
                    for n in {l.lo, l.hi, some_nonce(rng, l)}:
                        assert desc_hash(hc, m, a, b, i, n) == oracle.hash(m, n), (mlen, a, b, i, n)
        assert tails > 1000 and (13, 1) in variants and (14, 1) in variants, (tails, sorted(variants))
        # the top of the uint64 range (ceil((a - t) / 10) must not overflow at a = 2^64-1)
        for m in (b"", b"bradfitz", b"x" * 42):
            for a, b in ((U64 - 5, U64), (U64, U64), (U64 - 123456, U64 - 17)):
                p = plan(hc, m, a, b)
                assert_tiles(p, a, b)
                for i, l in enumerate(p):
                    for n in {l.lo, l.hi}:
                        assert desc_hash(hc, m, a, b, i, n) == oracle.hash(m, n), (m, a, b, i, n)
    finally:
        hc.hostcheck_set_layout_policy(AUTO)


def test_tail_digit_span_rule(hc):
    """AUTO takes the tail-digit launches only for a digit group the search spans
    GPUHASH_TAIL_MIN_SPAN (2^33) nonces of; the flags force either way."""
    import re
    h = open(os.path.join(ROOT, "include", "gpuhash.h")).read()
    assert int(re.search(r"#define GPUHASH_TAIL_MIN_SPAN (\d+)ull", h).group(1)) == 1 << 33
    assert int(re.search(r"#define GPUHASH_LAYOUT_TAIL_ALWAYS (\d+)", h).group(1)) == TAIL_ALWAYS
    assert int(re.search(r"#define GPUHASH_LAYOUT_TAIL_NEVER (\d+)", h).group(1)) == TAIL_NEVER
    import sys
    sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
    import gpuhash
    assert (gpuhash.LAYOUT_TAIL_ALWAYS, gpuhash.LAYOUT_TAIL_NEVER, gpuhash.TAIL_MIN_SPAN) == (TAIL_ALWAYS, TAIL_NEVER, 1 << 33)
    m = b"bradfitz"  # 12 digits: W_4 = 4 digits, W_5 = the 12th digit + 0x80
    a = 10 ** 11
    strides = lambda p: {l.stride for l in p}
    assert strides(plan(hc, m, a, a + (1 << 33) - 2)) == {1}
    p = plan(hc, m, a, a + (1 << 33) - 1)
    assert strides(p) == {10} and {(l.J, l.q) for l in p} == {(4, 4)} and {l.tail for l in p} == set(range(10))
    assert_tiles(p, a, a + (1 << 33) - 1)
    # 10- and 11-digit bradfitz groups (3 and 4 digits in W_4) never qualify
    assert strides(plan(hc, m, 10 ** 9, 10 ** 11 - 1)) == {1}
    try:
        hc.hostcheck_set_layout_policy(AUTO | TAIL_NEVER)
        assert strides(plan(hc, m, 0, (1 << 40) - 1)) == {1}
        hc.hostcheck_set_layout_policy(AUTO | TAIL_ALWAYS)
        assert 10 in strides(plan(hc, m, a, a + 99))
    finally:
        hc.hostcheck_set_layout_policy(AUTO)
