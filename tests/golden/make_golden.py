#!/usr/bin/env python3
"""Generate tests/golden/golden.json -- the committed parity fixtures.

Every expected (hash, nonce) here is computed by the CPU restatements in oracle/
(hash_oracle.c, cross-checked by the hashlib restatement for every range small
enough for Python).  The first group restates the only reference-provided pins, the
known-answer values of p1.pdf p.12; the rest are the SURVEY.md 8(c) table and the
BASELINE configs at full size where the C oracle can finish (2^32 nonces on 8 cores
takes a few minutes).

    python tests/golden/make_golden.py            # small + big (several minutes)
    python tests/golden/make_golden.py --small    # just the quick cases
    python tests/golden/make_golden.py --huge cfg5_client-00_2p36 ...   # named HUGE cases
    python tests/golden/make_golden.py --huge all                        # every HUGE case

HUGE cases (2^36-2^40 nonces) are computed by oracle/golden_scan.c, the SHA-NI/AVX-512
restatement (~190 MH/s on the container's 8 cores: 2^36 in ~6 min, 2^40 in ~1.6 h).
Each is merged into the existing golden.json as soon as it finishes, so the other
fixtures are kept.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import hash_oracle as ho  # noqa: E402

M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
M44, M45 = M120[:44], M120[:45]
U64 = (1 << 64) - 1

SMALL = [
    # (name, msg, lower, upper, note)
    ("spec_msg_0_2", b"msg", 0, 2, "p1.pdf p.12: min over n=0..2 is (4754799531757243342, 1)"),
    ("cfg1_bradfitz_9999", b"bradfitz", 0, 9999, "config 1: client must print Result 1419516646206828 9898"),
    ("empty_msg_0_9", b"", 0, 9, "empty message, L = 2"),
    ("bradfitz_u64max", b"bradfitz", U64, U64, "20-digit nonce"),
    ("m44_9to10", M44, 999999000, 1000001000, "9->10 digits, stays 1 block"),
    ("m44_10to11", M44, 9999999000, 10000001000, "10->11 digits, 1->2 blocks"),
    ("m45_9to10", M45, 999999000, 1000001000, "9->10 digits, 1->2 blocks"),
    ("m45_10to11", M45, 9999999000, 10000001000, "10->11 digits, 2 blocks"),
    ("m120_9to10", M120, 999999000, 1000001000, "config 3, 9->10"),
    ("m120_10to11", M120, 9999999000, 10000001000, "config 3, 10->11"),
    ("bradfitz_top", b"bradfitz", U64 - 1000, U64, "range ending at 2^64-1 (loop overflow edge)"),
    ("bradfitz_19to20", b"bradfitz", 10**19 - 500, 10**19 + 500, "19->20 digit boundary"),
    ("zero_only", b"bradfitz", 0, 0, "single nonce 0"),
    ("m55_pad", b"x" * 53, 0, 20000, "L crosses 55/56/64 bytes: extra padding block"),
    ("m63", b"y" * 63, 5, 123456, "prefix fills a block"),
    ("m64", b"z" * 64, 99990, 100010, "prefix = 64 bytes + space"),
    ("m119", M120[:119], 123456789, 123476789, "digits straddle block 1/2"),
]

BIG = [
    ("cfg2_bradfitz_2p32", b"bradfitz", 0, (1 << 32) - 1, "config 2 full range"),
    ("cfg3_m120_1e9", M120, 10**9 - (1 << 28), 10**9 + (1 << 28), "config 3 throughput window 9->10"),
    ("cfg3_m120_1e10", M120, 10**10 - (1 << 28), 10**10 + (1 << 28), "config 3 throughput window 10->11"),
    ("m45_2p28", M45, 10**9 - (1 << 27), 10**9 + (1 << 27), "1->2 blocks at 10 digits"),
]


# config 5 (BASELINE configs[4]): 16 clients "client-00".."client-15", each sending
# Request(msg, 0, maxNonce = 2^36) -- inclusive, p1.pdf p.14; config 4 (configs[3]):
# "bradfitz" over [0, 2^40).
CFG5_CLIENTS = [f"client-{i:02d}" for i in range(16)]
HUGE = [(f"cfg5_{c}_2p36", c.encode(), 0, 1 << 36, "config 5: one client's whole request")
        for c in CFG5_CLIENTS] + [
    ("cfg4_bradfitz_2p40", b"bradfitz", 0, (1 << 40) - 1, "config 4: [0, 2^40) of bradfitz"),
] + [
    # the timed step of bench.py's config 2 at N = 2, 4, 8 GPUs searches [0, N * 2^32) (weak
    # scaling, rank r on [r * 2^32, (r + 1) * 2^32)), so the driver's scaling lines are
    # golden-checked too; and config 4's one-GPU step, [0, 2^37)
    (f"cfg2_bradfitz_{n}gpu", b"bradfitz", 0, (n << 32) - 1, f"config 2's timed step at N = {n}")
    for n in (2, 4, 8)
] + [("cfg4_bradfitz_2p37", b"bradfitz", 0, (1 << 37) - 1, "config 4's timed step at N = 1")]


def run_huge(names: list[str], threads: int) -> None:
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    gs = ho.GoldenScan()
    if not gs.available():
        raise SystemExit("golden_scan needs the x86 SHA extensions")
    c = ho.load_c_oracle()
    for msg, n, h in ho.SPEC_KATS:
        assert gs.hash(msg, n) == h
    todo = [x for x in HUGE if "all" in names or x[0] in names]
    for name, msg, lo, hi, note in todo:
        t0 = time.time()
        h, n = gs.min(msg, lo, hi, threads=threads, progress=True)
        # the winner re-hashed by the two other restatements
        assert c.hash(msg, n) == h == ho.hash_py(msg, n), name
        out = json.load(open(dst))
        out["ranges"] = [r for r in out["ranges"] if r["name"] != name]
        out["ranges"].append({"name": name, "msg_hex": msg.hex(), "lower": lo, "upper": hi,
                              "hash": h, "nonce": n, "note": note,
                              "computed_by": "oracle/golden_scan.c (SHA-NI/AVX-512)",
                              "seconds": round(time.time() - t0, 1)})
        with open(dst, "w") as f:
            json.dump(out, f, indent=1)
        print(f"{name:24s} [{lo},{hi}] -> ({h}, {n})  {time.time() - t0:.1f}s", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--huge", nargs="+", default=None)
    args = ap.parse_args()
    if args.huge:
        run_huge(args.huge, args.threads)
        return
    c = ho.load_c_oracle()
    out = {"generated_by": "tests/golden/make_golden.py (oracle/hash_oracle.c, checked by oracle/hash_oracle.py)",
           "kats": [], "ranges": []}
    for msg, n, h in ho.SPEC_KATS:
        assert c.hash(msg, n) == h == ho.hash_py(msg, n)
        out["kats"].append({"msg_hex": msg.hex(), "nonce": n, "hash": h, "source": "p1.pdf p.12"})
    cases = SMALL + ([] if args.small else BIG)
    for name, msg, lo, hi, note in cases:
        t0 = time.time()
        h, n = c.min(msg, lo, hi, threads=args.threads if hi - lo > 100000 else 1)
        if hi - lo <= 200000:
            assert (h, n) == ho.min_py(msg, lo, hi), name
        out["ranges"].append({"name": name, "msg_hex": msg.hex(), "lower": lo, "upper": hi,
                              "hash": h, "nonce": n, "note": note})
        print(f"{name:24s} [{lo},{hi}] -> ({h}, {n})  {time.time() - t0:.1f}s", flush=True)
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    if os.path.exists(dst):
        # keep previously generated big cases (--small) and always the HUGE ones, which
        # only --huge recomputes
        old = json.load(open(dst))
        keep = {x[0] for x in HUGE} | ({x[0] for x in BIG} if args.small else set())
        have = {r["name"] for r in out["ranges"]}
        out["ranges"] += [r for r in old["ranges"] if r["name"] in keep and r["name"] not in have]
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main()
