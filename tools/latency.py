#!/usr/bin/env python3
"""Per-call latency of gpuhash_min for small to mid-size jobs (one MI355X).

A miner makes one blocking call per job.  For small jobs (config 1 is 10^4 nonces) the
call's fixed cost dominates: planning on the host, one descriptor copy, 1-3 scan launches,
a reduce per launch, and a 16-byte copy back.  This prints the median wall time per call
and the implied rate, so DESIGN.md can state where throughput takes over from latency.
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
import gpuhash  # noqa: E402

with gpuhash.Engine([0]) as eng:
    for n in [1, 10 ** 4, 10 ** 6, 10 ** 8, 10 ** 9]:
        reps = 50 if n <= 10 ** 6 else 10
        eng.min(b"bradfitz", 10 ** 9, 10 ** 9 + n - 1)  # warm
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            eng.min(b"bradfitz", 10 ** 9, 10 ** 9 + n - 1)
            ts.append(time.perf_counter() - t)
        med = statistics.median(ts)
        st = eng.stats()
        print(json.dumps({"nonces": n, "median_ms": round(med * 1e3, 4), "GHs": round(n / med / 1e9, 4),
                          "kernel_ms": round(st["kernel_ms"], 4), "launches": st["launches"]}), flush=True)
