#!/usr/bin/env python3
"""Times each tools/variants/<name>/libgpuhash.so (tools/build_variants.sh) on config 2
(bradfitz, 2^32 nonces) and config 3's 10^9 window, one subprocess per variant (each
loads its own code object), interleaved over rounds so clock drift hits all alike.
Checks every variant returns the same (hash, nonce)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "tools", "variants")

CHILD = r'''
import json, os, sys, time
sys.path.insert(0, sys.argv[2])
import gpuhash
M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
with gpuhash.Engine([0], lib_path=sys.argv[1]) as e:
    out = {}
    cases = [("c2", b"bradfitz", 0, (1 << 32) - 1),
             ("c3", M120, 10**9 - (1 << 28), 10**9 + (1 << 28)),
             ("u2", b"u" * 58, 10**11, 10**11 + (1 << 31)),        # C2=2 (two-word uniform loop)
             ("ex", b"x" * 44, 10**11, 10**11 + (1 << 30)),        # EX (extra padding block)
             ("j13", b"y" * 44, 10**9, 10**9 + (1 << 31)),         # plain, late loop word
             ("j2", b"", 10**9, 10**9 + (1 << 31)),                # plain, early loop word
             ("cj1", b"c" * 61, 10**9, 10**9 + (1 << 31)),         # classic straddle C2=1, J=1
             ("u2f", b"u" * 58, 10240 * 10**7, 10240 * 10**7 + 256 * 10**7 - 1),  # C2=2, one full row
             ("u2p", b"u" * 60, 10**9, (1 << 32) - 1),  # C2=2, 430 lane values: wave 3 of row 2 idle
             ("lt61", b"t" * 61, 10**9, 10**9 + (1 << 31)),        # C2=3 lane table, 2 digits in B-1
             ("lt58", b"t" * 58, 10**11, 10**11 + (1 << 32)),     # C2=3 lane table, 5 digits in B-1
             ("q1", b"bradfitz", 10**11, 10**11 + (1 << 34) - 1)]  # 12 digits: one in the last word (tail-digit launches)
    only = os.environ.get("VCASES")
    if only:
        cases = [next(c for c in cases if c[0] == n) for n in only.split(",")]
    for name, msg, lo, hi in cases:
        e.min(msg, lo, hi)
        best, res, sclk = 1e9, None, None
        for _ in range(4):
            t = time.perf_counter(); res = e.min(msg, lo, hi); dt = time.perf_counter() - t
            if dt < best:
                best = dt
                # in-kernel shader clock of the launch with the most nonces (workgroup 0's
                # s_memtime / s_memrealtime over the persistent launch)
                top = max(e.launches(), key=lambda l: l["nonces"])
                sclk = top["sclk_mhz"]
        out[name] = {"GHs": (hi - lo + 1) / best / 1e9, "res": list(res), "sclk": sclk}
    print(json.dumps(out))
'''

names = sorted(n for n in os.listdir(VDIR) if os.path.exists(os.path.join(VDIR, n, "libgpuhash.so")))
if len(sys.argv) > 2:
    names = [n for n in names if n in sys.argv[2].split(",")]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
results = {n: [] for n in names}
for rnd in range(rounds):
    for n in names:
        r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(VDIR, n, "libgpuhash.so"),
                            os.path.join(ROOT, "bitcoin-miner_amd")], capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            print(json.dumps({"variant": n, "error": r.stderr[-500:]}), flush=True)
            continue
        d = json.loads(r.stdout.strip().splitlines()[-1])
        results[n].append(d)
        print(json.dumps({"variant": n, "round": rnd, **{k: round(v["GHs"], 3) for k, v in d.items()}}), flush=True)
        print(json.dumps({"variant": n, "round": rnd, "sclk_mhz": {k: v["sclk"] and round(v["sclk"]) for k, v in d.items()}}), flush=True)
ref = None
for n, ds in results.items():
    if not ds:
        continue
    res = [tuple(v["res"]) for d in ds for v in d.values()]
    ref = ref or res
    best = {k: round(max(d[k]["GHs"] for d in ds), 3) for k in ds[0]}
    print(json.dumps({"variant": n, "best": best, "same_results": res == ref}), flush=True)
