"""CPU: pin the oracle before trusting it.

The reference's only pins for the hot path are the handout's known-answer values
(p1.pdf p.12).  Both restatements in oracle/ (C from FIPS 180-4, Python over hashlib /
OpenSSL) must reproduce them, agree with each other, and reproduce the committed
golden fixtures (tests/golden/golden.json, made by tests/golden/make_golden.py).
"""
import random

import hash_oracle as ho
import pytest


def test_spec_kats_c_and_hashlib(oracle):
    for msg, nonce, want in ho.SPEC_KATS:
        assert oracle.hash(msg, nonce) == want
        assert ho.hash_py(msg, nonce) == want


def test_spec_min_msg_0_2(oracle):
    # p1.pdf p.12: "the final result consists of least hash value 4754799531757243342 and nonce 1"
    assert oracle.min(b"msg", 0, 2) == (4754799531757243342, 1)
    assert ho.min_py(b"msg", 0, 2) == (4754799531757243342, 1)


def test_c_matches_hashlib_random():
    c = ho.load_c_oracle()
    rng = random.Random(7)
    for _ in range(3000):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 260)))
        n = rng.choice([rng.randrange(0, 100), rng.randrange(0, 1 << 64),
                        10 ** rng.randrange(0, 20) + rng.randrange(-2, 3)])
        n = max(0, min(n, (1 << 64) - 1))
        assert c.hash(m, n) == ho.hash_py(m, n), (m, n)


def test_golden_kats(golden, oracle):
    for k in golden["kats"]:
        assert oracle.hash(bytes.fromhex(k["msg_hex"]), k["nonce"]) == k["hash"]


def test_golden_small_ranges(golden, oracle):
    for r in golden["ranges"]:
        if r["upper"] - r["lower"] > 300000:
            continue
        got = oracle.min(bytes.fromhex(r["msg_hex"]), r["lower"], r["upper"])
        assert got == (r["hash"], r["nonce"]), r["name"]
        if r["upper"] - r["lower"] <= 20000:
            assert ho.min_py(bytes.fromhex(r["msg_hex"]), r["lower"], r["upper"]) == got


def test_survey_table_values(golden):
    # SURVEY.md 8(c) table, computed independently with hashlib while surveying
    want = {
        "cfg1_bradfitz_9999": (1419516646206828, 9898),
        "empty_msg_0_9": (611964081730071533, 9),
        "m44_9to10": (7116205622147787, 1000000849),
        "m44_10to11": (365873096250872, 9999999756),
        "m45_9to10": (10081557034389177, 1000000155),
        "m45_10to11": (4046047097157241, 9999999183),
        "m120_9to10": (2329720969182228, 999999133),
        "m120_10to11": (3511599402080292, 9999999544),
    }
    by = {r["name"]: (r["hash"], r["nonce"]) for r in golden["ranges"]}
    for k, v in want.items():
        assert by[k] == v, k
    assert ho.hash_py(b"bradfitz", (1 << 64) - 1) == 18191378931277043848


def test_multithreaded_min_equals_scan(oracle):
    rng = random.Random(3)
    for _ in range(20):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 130)))
        lo = rng.randrange(0, 10 ** 12)
        hi = lo + rng.randrange(0, 50000)
        assert oracle.min(m, lo, hi, threads=7) == oracle.min(m, lo, hi)


def test_tie_rule_lowest_nonce():
    # strict '<' ascending scan keeps the FIRST (lowest) nonce of equal hashes: check
    # the restatement on a synthetic key stream (real 64-bit ties are unreachable)
    keys = [(5, 9), (3, 4), (3, 2), (7, 1), (3, 8)]
    best = None
    for h, n in sorted(keys, key=lambda x: x[1]):  # ascending nonce order
        if best is None or h < best[0]:
            best = (h, n)
    assert best == min(keys) == (3, 2)


def test_lower_gt_upper_is_error(oracle):
    with pytest.raises(ValueError):
        oracle.min(b"x", 5, 4)


# FIPS 180-4 / NIST CSRC example digests for SHA-256 (independent of hashlib): pins the
# oracle's compression function itself, not just its agreement with OpenSSL.
FIPS_VECTORS = [
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqr"
     b"lmnopqrsmnopqrstnopqrstu",
     "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
    (b"a" * 1_000_000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]


@pytest.mark.parametrize("data,digest", FIPS_VECTORS, ids=["empty", "abc", "448bit", "896bit", "million_a"])
def test_c_sha256_fips_vectors(oracle, data, digest):
    import ctypes
    out = (ctypes.c_uint32 * 8)()
    oracle.lib.oracle_sha256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
    oracle.lib.oracle_sha256(data, len(data), out)
    assert "".join(f"{w:08x}" for w in out) == digest


def test_cpu_baseline_matches_the_oracle(oracle):
    """bench.py's CPU baseline (oracle/cpu_baseline.c, OpenSSL SHA-256) computes the same
    Hash and argmin as the checker: the KATs (p1.pdf p.12), config 1's answer, a range
    across the 9->10 digit boundary, and its threaded merge."""
    import hash_oracle as ho
    b = ho.load_cpu_baseline()
    if not b.available():
        pytest.skip("no libcrypto on this host")
    assert [b.hash(b"msg", n) for n in range(3)] == [13781283048668101583, 4754799531757243342,
                                                     5611725180048225792]
    assert b.min(b"bradfitz", 0, 9999) == (1419516646206828, 9898)
    m = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
    assert b.min(m, 999_990_000, 1_000_010_000) == oracle.min(m, 999_990_000, 1_000_010_000)
    assert b.min(b"bradfitz", 0, 200_000, threads=7) == oracle.min(b"bradfitz", 0, 200_000)
    with pytest.raises(ValueError):
        b.min(b"x", 5, 4)


@pytest.fixture(scope="module")
def golden_scan():
    gs = ho.GoldenScan()
    if not gs.available():
        pytest.skip("no x86 SHA extensions on this host")
    return gs


def test_golden_scan_matches_the_oracle(golden_scan, oracle):
    """oracle/golden_scan.c (SHA-NI midstates + AVX-512 or SHA-NI scan), which computes
    the HUGE fixtures, against the plain-C oracle: KATs, random single hashes, and range
    argmins over every digit count, block straddles, 1..3 threads (chunks of 2^22 never
    split these, so the segment loop, the lane padding and the digit carries are what is
    checked) and one range of several chunks."""
    for msg, n, h in ho.SPEC_KATS:
        assert golden_scan.hash(msg, n) == h
    rng = random.Random(11)
    for _ in range(1500):
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 200)))
        n = rng.choice([rng.randrange(1 << 64), rng.randrange(10 ** rng.randrange(1, 20))])
        assert golden_scan.hash(m, n) == oracle.hash(m, n), (m, n)
    for _ in range(150):
        m = bytes(rng.randrange(32, 127) for _ in range(rng.randrange(0, 140)))
        lo = rng.randrange(10 ** rng.randrange(1, 20))
        hi = min(lo + rng.randrange(0, 3000), (1 << 64) - 1)
        assert golden_scan.min(m, lo, hi, threads=rng.randrange(1, 4)) == oracle.min(m, lo, hi), (m, lo, hi)
    assert golden_scan.min(b"bradfitz", 0, 9999) == (1419516646206828, 9898)
    assert golden_scan.min(b"msg", (1 << 64) - 70, (1 << 64) - 1) == oracle.min(b"msg", (1 << 64) - 70, (1 << 64) - 1)
    lo, hi = 10**9 - 5_000_000, 10**9 + 5_000_000  # 3 chunks, 9 -> 10 digits
    assert golden_scan.min(b"client-03", lo, hi, threads=4) == oracle.min(b"client-03", lo, hi, threads=8)


def test_huge_goldens_rehash(golden, oracle):
    """Every HUGE fixture's winner re-hashes to its hash under the two other
    restatements (the full ranges are the GPU tests' job)."""
    huge = [r for r in golden["ranges"] if "computed_by" in r]
    names = {r["name"] for r in huge}
    # config 4's [0, 2^40) and every one of config 5's 16 client requests;
    # since round 5 the timed steps of config 2 at N = 2, 4, 8 and config 4 at N = 1, so
    # bench.py checks those lines too (step_check)
    assert names == {"cfg4_bradfitz_2p40", "cfg4_bradfitz_2p37"} | {f"cfg5_client-{i:02d}_2p36" for i in range(16)} \
        | {f"cfg2_bradfitz_{n}gpu" for n in (2, 4, 8)}
    for r in huge:
        m = bytes.fromhex(r["msg_hex"])
        assert r["lower"] <= r["nonce"] <= r["upper"]
        assert oracle.hash(m, r["nonce"]) == r["hash"] == ho.hash_py(m, r["nonce"]), r["name"]
