#!/usr/bin/env python3
"""Randomised GPU-vs-oracle parity soak (run on the GPU box; not part of the test suite).

Draws (message, range) cases across message lengths 0-300 (plus a few 1-4 KB), every
digit count 1-20, ranges of 1 to ~2e6 nonces placed at random or straddling a digit-count
boundary, under every layout policy (a third of the cases with the tail-digit launches
forced), and compares gpuhash_min with the C oracle's scan.  Since round 5 a fifth of the
cases run on a context with 2, 3 or 8 entries of the one GPU, so the in-process shard cuts
(the cost model of plan.cpp shard_range, priced per shard span and policy) are soaked too,
and a tenth also compare every nonce's hash (gpuhash_hash_range, the kernels' MODE 1) over
up to 2^16 nonces of the case with the oracle's.
Prints one JSON line per 100 cases and a summary; exits 1 on the first mismatch.
"""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gpuhash  # noqa: E402
import hash_oracle  # noqa: E402

U64 = (1 << 64) - 1
seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 12345
rng = random.Random(seed)
oracle = hash_oracle.load_c_oracle()
threads = min(16, len(os.sched_getaffinity(0)))


def case():
    mlen = rng.choice([rng.randrange(0, 301)] * 9 + [rng.randrange(1000, 4097)])
    d = rng.randrange(1, 21)
    if rng.random() < 0.25:  # round 3: the J = 1 straddles (lane table, two-word, classic)
        mlen = 64 * rng.randrange(0, 4) + rng.choice([55, 56, 57, 58, 59, 60, 61, 62])
        d = rng.randrange(6, 13)
    m = bytes(rng.randrange(256) for _ in range(mlen))
    lo_d = 0 if d == 1 else 10 ** (d - 1)
    hi_d = U64 if d == 20 else 10 ** d - 1
    n = int(10 ** rng.uniform(0, 6.3))
    if rng.random() < 0.4 and d > 1:  # straddle the boundary into d digits
        lo = max(0, lo_d - rng.randrange(0, n + 1))
    else:
        lo = rng.randrange(lo_d, hi_d + 1)
    hi = min(U64, lo + n - 1)
    return m, lo, hi


t0 = time.time()
count = nonces = multi_cases = per_nonce = 0
multis = [gpuhash.Engine([0] * k) for k in (2, 3, 8)]
with gpuhash.Engine([0]) as one:
    while time.time() - t0 < seconds:
        m, lo, hi = case()
        eng = one
        if rng.random() < 0.2:
            eng = rng.choice(multis)
            multi_cases += 1
        policy = rng.choice([gpuhash.LAYOUT_AUTO, gpuhash.LAYOUT_UNIFORM, gpuhash.LAYOUT_CLASSIC,
                             gpuhash.LAYOUT_LANETABLE])
        # round 4: the tail-digit launches (AUTO takes them only above 2^33 nonces per
        # digit group, far beyond a soak case) forced on a third of the cases
        if rng.random() < 1 / 3:
            policy |= gpuhash.LAYOUT_TAIL_ALWAYS
        eng.set_layout_policy(policy)
        got = eng.min(m, lo, hi)
        want = oracle.min(m, lo, hi, threads=threads)
        count += 1
        nonces += hi - lo + 1
        if got != want:
            print(json.dumps({"MISMATCH": True, "msg_hex": m.hex(), "lower": lo, "upper": hi,
                              "policy": policy, "entries": eng.ndevices, "got": list(got),
                              "want": list(want)}), flush=True)
            sys.exit(1)
        if rng.random() < 0.1:  # per-nonce parity over the first <= 2^16 nonces of the case
            k = min(hi - lo + 1, 1 << 16)
            g = eng.hash_range(m, lo, k)
            w = oracle.hash_range(m, lo, k)
            per_nonce += k
            if not (g == w).all():
                bad = int((g != w).argmax())
                print(json.dumps({"MISMATCH": True, "per_nonce": True, "msg_hex": m.hex(), "nonce": lo + bad,
                                  "policy": policy, "got": int(g[bad]), "want": int(w[bad])}), flush=True)
                sys.exit(1)
        if count % 100 == 0:
            print(json.dumps({"cases": count, "nonces": nonces, "elapsed_s": round(time.time() - t0, 1)}),
                  flush=True)
for e in multis:
    e.close()
print(json.dumps({"summary": True, "cases": count, "multi_device_cases": multi_cases, "nonces": nonces,
                  "per_nonce_hashes_compared": per_nonce,
                  "mismatches": 0, "seed": seed, "build_id": gpuhash.build_id(),
                  "elapsed_s": round(time.time() - t0, 1)}), flush=True)
