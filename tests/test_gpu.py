"""GPU parity: the HIP path (through the C ABI) against the oracle and the goldens.

Bar: bit-exact (hash, nonce) for every search and bit-exact per-nonce hashes, on the
same inputs, at sizes the C oracle finishes in seconds; the committed golden fixtures
(tests/golden/golden.json, incl. the full 2^32 config-2 range); and at full sizes
through size-independent properties (split/merge invariance, winner re-hash).
"""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

U64 = (1 << 64) - 1
M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]


def test_spec_kats_through_kernels(engine):
    # p1.pdf p.12: Hash("msg", 0..2)
    got = engine.hash_range(b"msg", 0, 3)
    assert [int(x) for x in got] == [13781283048668101583, 4754799531757243342, 5611725180048225792]
    assert engine.min(b"msg", 0, 2) == (4754799531757243342, 1)


def test_golden_ranges(engine, golden):
    # the HUGE fixtures (oracle/golden_scan.c: config 4's 2^40 and config 5's 2^36
    # requests) have their own tests: test_config4_full_range, test_gpu_system.py
    for r in golden["ranges"]:
        if "computed_by" in r:
            continue
        got = engine.min(bytes.fromhex(r["msg_hex"]), r["lower"], r["upper"])
        assert got == (r["hash"], r["nonce"]), r["name"]


def test_config1_miner_request(engine):
    import gpuhash as g
    miner = g.Miner(engine=engine)
    res = miner.handle(g.NewRequest("bradfitz", 0, 9999))
    assert (res.Type, res.Hash, res.Nonce) == (g.MsgType.Result, 1419516646206828, 9898)
    assert g.Hash("bradfitz", res.Nonce) == res.Hash


def variant_cases():
    """(msg, lower, count) windows that straddle digit-count and block boundaries for
    message lengths 0..140, so every (J, C2, EX) kernel variant and both lane-word
    placements run."""
    rng = random.Random(42)
    cases = []
    for mlen in list(range(0, 70)) + list(range(100, 141, 3)):
        m = bytes(rng.randrange(256) for _ in range(mlen))
        d = rng.choice([3, 5, 7, 9, 10, 11, 12, 13])
        cases.append((m, max(0, 10 ** d - rng.randrange(1, 3000)), rng.randrange(1000, 6000)))
    for m in (b"", b"bradfitz", M120, M120[:44], M120[:45]):
        cases.append((m, 0, 12000))
        cases.append((m, U64 - 4999, 5000))
        cases.append((m, 10 ** 19 - 2500, 5000))
    return cases


def test_hash_range_bit_exact(engine, oracle):
    for m, lo, cnt in variant_cases():
        got = engine.hash_range(m, lo, cnt)
        want = oracle.hash_range(m, lo, cnt)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (len(m), lo, cnt, int(bad[0]) + lo)


@pytest.mark.parametrize("mlen,d,j", [
    (8, 12, 4), (8, 8, 3), (12, 12, 5), (27, 9, 8),     # plain: last word = 1 digit
    (42, 14, 13), (46, 14, 14), (42, 18, 14),           # the extra-padding-block kernels
])
def test_tail_digit_launches(engine, oracle, mlen, d, j, request):
    """Tail-digit launches (include/gpuhash.h), forced on small ranges:
    per-nonce parity across the last-digit residues, the loop word's roll-overs and the
    lane rows (the kernel maps k back to nonce = 10 k + t), and min parity, on the J-1
    kernel the layout moves the group to."""
    import gpuhash
    request.addfinalizer(lambda: engine.set_layout_policy(gpuhash.LAYOUT_AUTO))
    engine.set_layout_policy(gpuhash.LAYOUT_AUTO | gpuhash.LAYOUT_TAIL_ALWAYS)
    rng = random.Random(mlen * 100 + d)
    m = bytes(rng.randrange(32, 127) for _ in range(mlen))
    base = 10 ** (d - 1) + rng.randrange(10 ** (d - 2))
    for lo in (base - base % 10 ** 5 - 4321, base + 7):
        got = engine.hash_range(m, lo, 60000)
        assert {(r["J"], r["digits"]) for r in engine.launches()} == {(j, d)}, engine.launches()
        want = oracle.hash_range(m, lo, 60000)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mlen, d, lo, int(bad[0]) + lo if bad.size else None)
    for lo, hi in ((base, base + 400_000), (base - base % 10 ** 6 - 13, base - base % 10 ** 6 + 250_000)):
        assert engine.min(m, lo, hi) == oracle.min(m, lo, hi, threads=16), (mlen, d, lo, hi)


def test_tail_digit_launches_top_of_u64(engine, oracle, request):
    """Tail-digit launches at 20 digits up to 2^64-1 (nonce = 10 k + t at the top of the
    uint64 range), per nonce and min, against the oracle."""
    import gpuhash
    request.addfinalizer(lambda: engine.set_layout_policy(gpuhash.LAYOUT_AUTO))
    engine.set_layout_policy(gpuhash.LAYOUT_AUTO | gpuhash.LAYOUT_TAIL_ALWAYS)
    for m in (b"", b"bradfitz"):  # 20 digits end W_5 / W_7 byte 0: one digit in the last word
        lo = U64 - 59999
        got = engine.hash_range(m, lo, 60000)
        assert {r["digits"] for r in engine.launches()} == {20}
        assert (got == oracle.hash_range(m, lo, 60000)).all()
        for a, b in ((U64 - 5, U64), (U64, U64), (U64 - 300_000, U64 - 17)):
            assert engine.min(m, a, b) == oracle.min(m, a, b), (m, a, b)


@pytest.mark.parametrize("mlen,d,c2,j", [
    (58, 10, 2, 1), (59, 10, 2, 1), (60, 10, 2, 1), (56, 12, 2, 1), (59, 12, 2, 1),  # two-word loop
    (120, 10, 1, 0), (54, 10, 1, 0), (119, 12, 1, 0),                                # K+W table
])
def test_uniform_schedule_layouts(engine, oracle, mlen, d, c2, j, request):
    """Layouts whose final block holds loop digits only (its schedule is built once per
    loop value: C2=1/J=0 from the k_ktab table, C2=2/J=1 in LDS): per-nonce parity over
    windows where the W_1 and W_0 loop digits roll over, and min parity."""
    import gpuhash
    rng = random.Random(mlen * 100 + d)
    m = bytes(rng.randrange(32, 127) for _ in range(mlen))
    base = 10 ** (d - 1) + rng.randrange(10 ** (d - 2))
    engine.set_layout_policy(gpuhash.LAYOUT_UNIFORM)  # small ranges would pick C2=1 under AUTO
    request.addfinalizer(lambda: engine.set_layout_policy(gpuhash.LAYOUT_AUTO))
    engine.min(m, base, base + 1000)
    assert any(r["C2"] == c2 and r["J"] == j for r in engine.launches()), engine.launches()
    for lo in (base - base % 10 ** 4 - 700, base - base % 10 ** 8 - 3000, base + 12345):
        got = engine.hash_range(m, lo, 6000)
        want = oracle.hash_range(m, lo, 6000)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mlen, d, lo, int(bad[0]) + lo if bad.size else None)
    for lo, hi in ((base, base + 2_000_000), (base - base % 10 ** 6 - 77, base - base % 10 ** 6 + 300_000)):
        assert engine.min(m, lo, hi) == oracle.min(m, lo, hi), (mlen, d, lo, hi)


@pytest.mark.parametrize("mlen,d", [(61, 10), (61, 7), (62, 8), (62, 6), (125, 9), (126, 9)])
def test_lane_table_layout(engine, oracle, mlen, d, request):
    """C2 = 3 (lane table): block B-1 holds 1-2 digits (message lengths =
    61, 62 mod 64), the lanes take block B's W_0/W_1 digits and keep its schedule in
    registers, the loop walks the block B-1 values from the p-table (k_ptab).  AUTO picks
    it for these lengths once a search covers >= 2 block B-1 values; the parity windows
    below are smaller, so they force it.  Per-nonce parity across loop-value (p-table
    entry) boundaries and W_0 / W_1 roll-overs, and min parity over whole and partial
    rectangles."""
    import gpuhash
    rng = random.Random(mlen * 100 + d)
    m = bytes(rng.randrange(32, 127) for _ in range(mlen))
    nb1 = (mlen + 1) % 64 and 64 - (mlen + 1) % 64
    RQ = 10 ** (d - nb1)  # lane values per loop value
    lo_d, hi_d = 10 ** (d - 1), 10 ** d - 1
    request.addfinalizer(lambda: engine.set_layout_policy(gpuhash.LAYOUT_AUTO))
    engine.min(m, lo_d, lo_d + 3 * RQ)
    assert {(r["C2"], r["J"]) for r in engine.launches()} == {(3, 1)}, engine.launches()
    engine.min(m, lo_d, lo_d + RQ // 2)
    assert {(r["C2"], r["J"]) for r in engine.launches()} == {(1, 1)}, engine.launches()
    engine.set_layout_policy(gpuhash.LAYOUT_LANETABLE)
    p = rng.randrange(lo_d // RQ + 1, hi_d // RQ)
    for lo in (p * RQ - 2500, p * RQ + RQ // 2 - 3333, p * RQ + 9_990_000 % RQ - 100):
        got = engine.hash_range(m, lo, 6000)
        want = oracle.hash_range(m, lo, 6000)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mlen, d, lo, int(bad[0]) + lo if bad.size else None)
    cases = [(p * RQ - 1_000_000, p * RQ + 1_000_000), (p * RQ + 17, p * RQ + 17)]
    if hi_d - lo_d < 10 ** 6:
        cases.append((lo_d, hi_d))  # the whole digit group: full rectangles + partial ends
    for lo, hi in cases:
        lo, hi = max(lo, lo_d), min(hi, hi_d)
        assert engine.min(m, lo, hi) == oracle.min(m, lo, hi, threads=8), (mlen, d, lo, hi)


def test_lane_table_long_loops_split(engine, oracle, request):
    """Under LANETABLE a straddle with 5 digits in block B-1 (m = 58, d = 10) loops over
    up to 10^5 block B-1 values; launches take at most 1024 p-table entries each."""
    import gpuhash
    request.addfinalizer(lambda: engine.set_layout_policy(gpuhash.LAYOUT_AUTO))
    engine.set_layout_policy(gpuhash.LAYOUT_LANETABLE)
    m = M120[:58]
    lo, hi = 12345 * 10 ** 5 + 678, (12345 + 1100) * 10 ** 5 + 4321
    assert engine.min(m, lo, hi) == oracle.min(m, lo, hi, threads=16)
    assert {(r["C2"], r["J"]) for r in engine.launches()} == {(3, 1)}, engine.launches()
    got = engine.hash_range(m, (12345 + 1024) * 10 ** 5 - 3000, 6000)
    want = oracle.hash_range(m, (12345 + 1024) * 10 ** 5 - 3000, 6000)
    assert (got == want).all()


def test_idle_waves_of_partial_rows(engine, oracle, request):
    """A row is 256 lane values (4 waves); a wave whose lanes all lie past the search's
    last lane value skips the row (scan_kernel.h), and in the two-word uniform layout it
    still walks the LDS batch barriers. 140 lane values: waves 0-1 full, wave 2 with 12
    lanes, wave 3 idle, in both the two-word (C2=2) and the plain layout."""
    import gpuhash
    request.addfinalizer(lambda: engine.set_layout_policy(gpuhash.LAYOUT_AUTO))
    engine.set_layout_policy(gpuhash.LAYOUT_UNIFORM)
    # m = 58, d = 10: 5 lane digits end block B-1, 5 loop digits fill W_0/W_1 (R = 10^5)
    m = M120[:58]
    lo, hi = 12345 * 10 ** 5 + 678, (12345 + 139) * 10 ** 5 + 4321
    assert engine.min(m, lo, hi) == oracle.min(m, lo, hi, threads=16)
    assert {(r["C2"], r["J"]) for r in engine.launches()} == {(2, 1)}, engine.launches()
    # bradfitz, d = 10: loop digits in W_4 (R = 10^3), lanes in W_2/W_3
    lo, hi = 1234567 * 10 ** 3 + 5, (1234567 + 139) * 10 ** 3 + 998
    assert engine.min(b"bradfitz", lo, hi) == oracle.min(b"bradfitz", lo, hi)
    assert {(r["C2"], r["J"]) for r in engine.launches()} == {(0, 4)}, engine.launches()


def test_layout_policies_agree(engine, request):
    """The straddling J=1 digit groups under UNIFORM, CLASSIC and AUTO: same answers
    (each is bit-exact against the oracle elsewhere; here at sizes past the oracle's)."""
    import gpuhash
    request.addfinalizer(lambda: engine.set_layout_policy(gpuhash.LAYOUT_AUTO))
    for m, lo, n in ((b"y" * 59, 10 ** 11 + 12345, 3 * 10 ** 10), (M120[:58], 10 ** 9 + 7, 2 * 10 ** 9)):
        got = {}
        pols = (gpuhash.LAYOUT_UNIFORM, gpuhash.LAYOUT_CLASSIC, gpuhash.LAYOUT_AUTO, gpuhash.LAYOUT_LANETABLE)
        for pol in pols:
            engine.set_layout_policy(pol)
            got[pol] = engine.min(m, lo, lo + n)
            got[(pol, "c2")] = {r["C2"] for r in engine.launches()}
        assert len({got[pol] for pol in pols}) == 1, got
        assert 2 in got[(gpuhash.LAYOUT_UNIFORM, "c2")] and 2 not in got[(gpuhash.LAYOUT_CLASSIC, "c2")]
        assert got[(gpuhash.LAYOUT_LANETABLE, "c2")] == {3} and got[(gpuhash.LAYOUT_CLASSIC, "c2")] == {1}
        assert gpuhash.Hash(m, got[gpuhash.LAYOUT_AUTO][1]) == got[gpuhash.LAYOUT_AUTO][0]
    with pytest.raises(gpuhash.GpuHashError):
        engine.set_layout_policy(7)


def test_ktab_several_digit_groups_in_one_call(engine, oracle):
    # m = 55: d = 9, 10, 11 are all C2/J=0 layouts, so a window across 10^9 (or 10^10)
    # builds two K+W tables (one per digit count) for the same launch group
    m = M120[:55]
    for x in (10 ** 9, 10 ** 10):
        assert engine.min(m, x - 40_000, x + 40_000) == oracle.min(m, x - 40_000, x + 40_000)
        recs = [r for r in engine.launches() if r["C2"] == 1 and r["J"] == 0]
        assert recs and recs[0]["nonces"] == 80_001, engine.launches()
        got = engine.hash_range(m, x - 3000, 6000)
        assert (got == oracle.hash_range(m, x - 3000, 6000)).all()


def test_min_matches_oracle_random(engine, oracle):
    rng = random.Random(9)
    for _ in range(120):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 160)))
        kind = rng.randrange(4)
        if kind == 0:
            lo = rng.randrange(0, 10 ** rng.randrange(1, 20))
        elif kind == 1:
            lo = 10 ** rng.randrange(1, 20) - rng.randrange(0, 50000)
        elif kind == 2:
            lo = rng.randrange(0, U64)
        else:
            lo = U64 - rng.randrange(0, 100000)
        lo = max(0, lo)
        hi = min(U64, lo + rng.randrange(0, 120000))
        assert engine.min(m, lo, hi) == oracle.min(m, lo, hi), (m, lo, hi)


@pytest.mark.parametrize("mlen", [1000, 1300])
def test_long_messages(engine, oracle, mlen):
    m = bytes((i * 131 + 7) % 256 for i in range(mlen))
    for lo in (0, 999_990_000, 10 ** 12 - 5000):
        assert engine.min(m, lo, lo + 300_000) == oracle.min(m, lo, lo + 300_000)
        assert (engine.hash_range(m, lo, 3000) == oracle.hash_range(m, lo, 3000)).all()


@pytest.mark.parametrize("short", [0, 5, 9, 19])
def test_maximum_message_size(engine, oracle, short):
    # The largest Data the ABI accepts (GPUHASH_MAX_MSG = 1 MiB = 16,384 whole blocks,
    # compressed into the host midstate once per call), and 5 / 9 / 19 bytes less: m = 59,
    # 55 and 45 mod 64 put the 10-digit nonces in the lane-table, K+W-table and
    # extra-block layouts.  The naive C oracle re-hashes the whole MiB per nonce (hash.go
    # has no midstate), so the ranges stay short.
    import gpuhash
    m = bytes((i * 2654435761 >> 13) & 0xFF for i in range(gpuhash.GPUHASH_MAX_MSG - short))
    lo = 10 ** 9 - 32  # 9 -> 10 digits
    assert (engine.hash_range(m, lo, 64) == oracle.hash_range(m, lo, 64)).all()
    lo = 10 ** 12 - 256  # 12 -> 13 digits
    assert engine.min(m, lo, lo + 511) == oracle.min(m, lo, lo + 511, threads=8)


def test_single_nonce_ranges(engine, oracle):
    rng = random.Random(1)
    for n in [0, 1, 9, 10, 99, 100, 12345, 10 ** 9 - 1, 10 ** 9, 2 ** 32 - 1, 10 ** 19, U64 - 1, U64] + \
            [rng.randrange(0, U64) for _ in range(40)]:
        for m in (b"bradfitz", M120, b""):
            assert engine.min(m, n, n) == (oracle.hash(m, n), n)


@pytest.mark.parametrize("rchunk", [1, 3, 10, 64, 100, 1000, 10000])
def test_work_item_granularity_is_invisible(engine, oracle, rchunk):
    for m, lo, hi in [(b"bradfitz", 123456789, 123656789), (M120, 9999990000, 10000040000),
                      (M120[:45], 999990000, 1000020000), (b"x" * 53, 0, 60000)]:
        assert engine.min(m, lo, hi, rchunk=rchunk) == oracle.min(m, lo, hi, threads=8)


def test_config2_full_range_golden(engine, golden):
    g = {r["name"]: r for r in golden["ranges"]}["cfg2_bradfitz_2p32"]
    assert engine.min(b"bradfitz", 0, (1 << 32) - 1) == (g["hash"], g["nonce"])
    st = engine.stats()
    assert st["nonces"] == 1 << 32 and st["kernel_ms"] > 0


def test_split_merge_invariance_at_scale(engine, oracle):
    # 2^36 nonces of config-4 shape: the argmin of the whole equals the lexicographic
    # min of the argmins of any split, and the winner re-hashes to the same value
    lo, hi = 3 << 36, (4 << 36) - 1
    whole = engine.min(b"bradfitz", lo, hi)
    rng = random.Random(4)
    cut = rng.randrange(lo, hi)
    parts = [engine.min(b"bradfitz", lo, cut), engine.min(b"bradfitz", cut + 1, hi)]
    assert whole == min(parts)
    assert oracle.hash(b"bradfitz", whole[1]) == whole[0]
    assert lo <= whole[1] <= hi


def test_config4_full_range(engine, oracle, golden):
    # Config 4 at full size: [0, 2^40) of "bradfitz" (~33 s on one MI355X), against the
    # CPU golden `cfg4_bradfitz_2p40` that oracle/golden_scan.c (SHA-NI/AVX-512, a
    # restatement sharing no code with the kernels) computed over the whole range on the
    # container's 8 cores (tests/golden/make_golden.py --huge).  Also: the winner
    # re-hashes through the plain-C oracle, and the 2^22 nonces around it hold nothing
    # lower (lowest nonce on ties).
    g = {r["name"]: r for r in golden["ranges"]}["cfg4_bradfitz_2p40"]
    assert (g["lower"], g["upper"]) == (0, (1 << 40) - 1)
    h, n = engine.min(b"bradfitz", 0, (1 << 40) - 1)
    assert (h, n) == (g["hash"], g["nonce"])
    assert oracle.hash(b"bradfitz", n) == h
    assert oracle.min(b"bradfitz", n - (1 << 21), n + (1 << 21), threads=8) == (h, n)


def test_errors_are_loud(engine):
    import gpuhash
    with pytest.raises(gpuhash.GpuHashError) as e:
        engine.min(b"x", 10, 9)
    assert e.value.rc == gpuhash.GPUHASH_EINVAL
    with pytest.raises(gpuhash.GpuHashError):
        gpuhash.Engine([0, 99])
    with pytest.raises(gpuhash.GpuHashError):
        engine.hash_range(b"x", U64, 2)  # wraps past 2^64-1
    assert e.value.is_argument_error
    with pytest.raises(gpuhash.GpuHashError) as e:
        engine.min(b"x" * (gpuhash.GPUHASH_MAX_MSG + 1), 0, 9)
    assert e.value.rc == gpuhash.GPUHASH_ETOOLONG and e.value.is_argument_error
    # bounds outside uint64 never reach ctypes (which would wrap 2^64+5 to 5)
    with pytest.raises(ValueError):
        engine.min(b"x", 0, U64 + 6)
    with pytest.raises(ValueError):
        engine.min(b"x", -1, 5)
    # and the context is still usable after every refused call
    assert engine.min(b"msg", 0, 2) == (4754799531757243342, 1)


def test_calls_leave_the_current_device_alone(engine, oracle):
    """Every entry point restores the calling thread's HIP device (include/gpuhash.h).
    With one GPU only device 0 exists, so this checks the guard does not disturb it or
    the torch-side current device across single- and multi-shard calls."""
    import ctypes

    import gpuhash
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime libgpuhash.so links (same handle)
    dev = ctypes.c_int(-1)
    assert hip.hipSetDevice(0) == 0
    with gpuhash.Engine([0, 0]) as two:
        assert two.min(b"bradfitz", 0, 9999) == (1419516646206828, 9898)
    engine.min(b"bradfitz", 0, 9999)
    engine.hash_range(b"bradfitz", 0, 16)
    assert hip.hipGetDevice(ctypes.byref(dev)) == 0 and dev.value == 0


def test_multi_device_sharding_and_host_argmin(engine, oracle):
    """The in-process multi-device path (static cost-balanced shards, one host thread +
    stream per entry, 16-byte host argmin) run as 3 shards on the one GPU of the box."""
    import gpuhash
    with gpuhash.Engine([0, 0, 0]) as multi:
        assert multi.ndevices == 3
        for m, lo, hi in [(b"bradfitz", 0, (1 << 32) - 1), (M120, 999_000_000, 1_001_000_000),
                          (b"x", 5, 7), (b"y" * 50, U64 - 10 ** 7, U64)]:
            assert multi.min(m, lo, hi) == engine.min(m, lo, hi)
        st = multi.stats()
        assert st["ndevices"] == 3 and st["launches"] >= 3
        # the launch records name their shard and the stream's runtime device
        recs = multi.launches()
        assert {r["shard"] for r in recs} == {0, 1, 2}
        assert all(r["device"] == 0 and r["stream_device"] == 0 for r in recs)
        assert multi.min(b"bradfitz", 0, 9999) == oracle.min(b"bradfitz", 0, 9999)


def _check_distinct_shards(recs, devs, lo, hi):
    """Every launch ran on the device its shard names (record ordinal == the context's
    entry, the stream's runtime ordinal == that device), and the shards tile [lo, hi]."""
    for r in recs:
        assert r["device"] == devs[r["shard"]] and r["stream_device"] == r["device"], r
    wins = sorted({(r["lo"], r["hi"], r["shard"]) for r in recs})
    assert wins[0][0] == lo and wins[-1][1] == hi
    assert all(b[0] == a[1] + 1 for a, b in zip(wins, wins[1:]))
    assert [w[2] for w in wins] == sorted(w[2] for w in wins)  # shard k < shard k+1 in range order


def test_distinct_devices(oracle, golden):
    """the multi-device path with DISTINCT ordinals -- every visible
    GPU in one context.  A bug that only shows with distinct devices (a buffer, stream or
    event on the wrong device, occupancy queried on another ordinal) cannot surface in the
    repeated-ordinal tests above.  Runs wherever >= 2 GPUs are visible; skips on one."""
    import gpuhash
    n = gpuhash.device_count()
    if n < 2:
        pytest.skip(f"{n} HIP device visible: distinct-device sharding needs >= 2 "
                    "(repeated-ordinal rehearsals: test_multi_device_sharding_and_host_argmin)")
    devs = list(range(n))
    with gpuhash.Engine(devs) as multi:
        # a 1 -> 2 SHA block straddle (m = 45 at 9 -> 10 digits), against the oracle
        m, lo, hi = M120[:45], 10 ** 9 - (1 << 22), 10 ** 9 + (1 << 22)
        assert multi.min(m, lo, hi) == oracle.min(m, lo, hi, threads=8)
        _check_distinct_shards(multi.launches(), devs, lo, hi)
        # a whole config-5 request [0, 2^36] split over every device, against its CPU golden
        g = next(r for r in golden["ranges"] if r["name"] == "cfg5_client-00_2p36")
        got = multi.min(bytes.fromhex(g["msg_hex"]), g["lower"], g["upper"])
        assert got == (g["hash"], g["nonce"])
        recs = multi.launches()
        _check_distinct_shards(recs, devs, g["lower"], g["upper"])
        assert {r["device"] for r in recs} == set(devs)  # every GPU took a shard
        assert multi.stats()["ndevices"] == n


def _bench(args, env=None, timeout=300):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.Popen([sys.executable, os.path.join(root, "bench.py"), *args], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True, env=e, cwd=root)


def test_distinct_devices_bench_inproc():
    """bench.py's in-process path over every visible GPU (distinct
    ordinals, one context), the search leg over config 2's [0, 2^32) against its golden,
    with shards on distinct PCI devices and the same-run scaling field."""
    import json
    import gpuhash
    n = gpuhash.device_count()
    if n < 2:
        pytest.skip(f"{n} HIP device visible: the distinct-device bench path needs >= 2")
    p = _bench(["--gpus", str(n), "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--search", "0:2^32-1"])
    out, err = p.communicate(timeout=300)
    assert p.returncode == 0, err[-2000:]
    line = json.loads(out.strip().splitlines()[-1])
    s = line["search_2p40"]
    assert s["golden_name"] == "cfg2_bradfitz_2p32" and s["matches_golden"] is True
    assert [x["device"] for x in s["shards"]] == list(range(n))
    assert len({x["pci"] for x in s["shards"]}) == n and "device_check" not in line
    assert 0 < s["scaling"]["scaling_efficiency"] <= 1.2


def test_distinct_devices_bench_ranks_one_visible_gpu_each():
    """VERDICT r04 item 6 / ADVICE r04: one bench.py process per GPU, each started with
    HIP_VISIBLE_DEVICES naming only its own GPU (every rank sees ordinal 0); distinct GPUs
    are proven by PCI id, and the gloo-merged search over [0, 2^32) equals its golden."""
    import json
    import socket
    import gpuhash
    n = gpuhash.device_count()
    if n < 2:
        pytest.skip(f"{n} HIP device visible: one-GPU-per-rank launches need >= 2")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [_bench(["--gpus", str(n), "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--search",
                     "0:2^32-1"],
                    env=dict(RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(n), LOCAL_WORLD_SIZE="1",
                             MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HIP_VISIBLE_DEVICES=str(r)))
             for r in range(n)]
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-1500:] for o in outs]
    line = json.loads([x for x in outs[0][0].splitlines() if x.startswith("{")][-1])
    assert [d["device"] for d in line["rank_devices"]] == [0] * n
    assert len({d["pci"] for d in line["rank_devices"]}) == n and "device_check" not in line
    s = line["search_2p40"]
    assert s["golden_name"] == "cfg2_bradfitz_2p32" and s["matches_golden"] is True


def test_more_shards_than_nonces(oracle):
    """8 device entries (the 8-GPU shape, on the box's one GPU) over ranges of 1-7 nonces:
    the shards without nonces stay idle and the host argmin takes only the others."""
    import gpuhash
    with gpuhash.Engine([0] * 8) as multi:
        for m, lo, hi in [(b"w", 7, 7), (b"z", 42, 43), (b"q", 0, 4), (b"r", 9, 15), (b"e", U64, U64),
                          (b"msg", 0, 2)]:
            assert multi.min(m, lo, hi) == oracle.min(m, lo, hi), (m, lo, hi)
            assert 1 <= multi.stats()["ndevices"] <= min(8, hi - lo + 1)


def test_multi_device_sliced(engine, oracle, monkeypatch):
    """Slices (gpuhash_min_ex) over several devices: each slice is sharded over the 3
    entries and merged into the running argmin."""
    import gpuhash
    monkeypatch.setenv("GPUHASH_SLICE_NONCES", "3000")
    with gpuhash.Engine([0, 0, 0]) as multi:
        for m, lo, hi in [(b"bradfitz", 0, 99_999), (M120[:45], 9_999_990_000, 10_000_020_000),
                          (b"edge", U64 - 50_000, U64)]:
            assert multi.min(m, lo, hi) == oracle.min(m, lo, hi), (m, lo, hi)
            assert multi.stats()["nonces"] == hi - lo + 1


def test_plain_c_client_through_the_abi(oracle):
    """gpuhash_cli: a C process with no Python/torch, making the cgo binding's calls."""
    import os
    import subprocess
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "bitcoin-miner_amd", "lib", "gpuhash_cli")
    out = subprocess.run([cli, "bradfitz", "0", "9999"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "Result 1419516646206828 9898"
    m = M120[:58].decode()
    out = subprocess.run([cli, m, "999000000", "1001000000"], capture_output=True, text=True, timeout=120)
    h, n = oracle.min(m.encode(), 999000000, 1001000000)
    assert out.returncode == 0 and out.stdout.strip() == f"Result {h} {n}", out.stderr
    out = subprocess.run([cli, "--range", "msg", "0", "3"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.split() == ["13781283048668101583", "4754799531757243342",
                                                          "5611725180048225792"]
    out = subprocess.run([cli, "bradfitz", "10", "5"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 3 and "invalid argument" in out.stderr


def test_native_library_is_the_one_loaded(engine):
    import gpuhash
    maps = open("/proc/self/maps").read()
    assert gpuhash.LIB_PATH in maps


@pytest.mark.parametrize("slice_nonces", [1, 999, 250000])
def test_sliced_search_matches_oracle(engine, oracle, monkeypatch, slice_nonces):
    """Searches longer than one slice run as consecutive slices merged on the host
    (gpuhash_min_ex).  A small GPUHASH_SLICE_NONCES drives that loop over oracle-sized
    ranges: across digit-count boundaries, ending exactly at 2^64-1 (the loop's overflow
    edge), and with the minimum in a late slice."""
    monkeypatch.setenv("GPUHASH_SLICE_NONCES", str(slice_nonces))
    cases = [(b"bradfitz", 999_000, 1_001_000), (M120, 10 ** 9 - 700, 10 ** 9 + 700),
             (b"edge", U64 - 600_000, U64)]
    if slice_nonces == 1:
        cases = [(b"bradfitz", 0, 60), (b"edge", U64 - 40, U64)]
    for m, lo, hi in cases:
        assert engine.min(m, lo, hi) == oracle.min(m, lo, hi), (m, lo, hi)
        st = engine.stats()
        assert st["nonces"] == hi - lo + 1
        assert st["launches"] >= (hi - lo + 1 + slice_nonces - 1) // slice_nonces


def test_top_of_u64_range_in_slices(engine, monkeypatch):
    """Unsliced, a span this close to 2^64 would plan one descriptor per 10^10 nonces
    over the whole call (a full [0, 2^64-1] search threw std::bad_alloc through the C
    ABI).  The top 3 slices of the range run 20-digit plans and end the slice loop at
    2^64-1; the winner re-hashes to the reported hash on the host."""
    import gpuhash
    monkeypatch.setenv("GPUHASH_SLICE_NONCES", str(1 << 20))
    lo = U64 - 3 * (1 << 20) + 1
    h, n = engine.min(b"bradfitz", lo, U64)
    assert lo <= n <= U64 and gpuhash.Hash(b"bradfitz", n) == h


def test_concurrent_calls_on_one_context_are_serialised(engine, oracle):
    """Several host threads sharing one context (e.g. goroutines sharing a Go Engine)
    each get their own correct answer."""
    import threading
    jobs = [(b"bradfitz", i * 50_000, i * 50_000 + 49_999) for i in range(8)]
    got = [None] * len(jobs)

    def run(i):
        got[i] = engine.min(*jobs[i])

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(jobs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert got == [oracle.min(*j) for j in jobs]


def test_host_wait_does_not_spin(engine):
    """A miner spends its life waiting inside gpuhash_min.  On this ROCm both
    hipStreamSynchronize and a blocking-sync event keep the waiting thread running (1.0
    host core per miner, profiles/r05_host_wait.jsonl); the engine's default wait sleeps
    between event queries, so a 0.5-s search costs the host almost nothing."""
    import resource
    import time
    engine.min(b"bradfitz", 0, 1 << 20)
    r0, t0 = resource.getrusage(resource.RUSAGE_SELF), time.perf_counter()
    engine.min(b"bradfitz", 1 << 36, (1 << 36) + (1 << 34) - 1)
    wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    assert wall > 0.2 and cpu / wall < 0.15, (cpu, wall)
