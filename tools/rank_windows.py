#!/usr/bin/env python3
"""Each rank's window of the N-GPU config-2 bench, timed alone on one GPU: rank r searches
[r*2^32, (r+1)*2^32) of 'bradfitz', so ranks differ in digit counts (rank 0: d=1..10,
rank 1: d=10, rank 2: d=10/11, ranks 3-7: d=11) and hence in scan variants.  The N-GPU
bench takes the max over ranks, so the slowest window sets its per-GPU rate.

  python tools/rank_windows.py [--ranks 0,1,2,3,7] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))

PER_GPU = 1 << 32


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="0,1,2,3,7")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import gpuhash
    eng = gpuhash.Engine([0])
    for r in [int(x) for x in args.ranks.split(",")]:
        lo, hi = r * PER_GPU, (r + 1) * PER_GPU - 1
        eng.min(b"bradfitz", lo, hi)  # warm-up
        best, launches = None, []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            res = eng.min(b"bradfitz", lo, hi)
            dt = time.perf_counter() - t0
            launches = eng.launches()
            best = dt if best is None else min(best, dt)
        row = {"rank": r, "window": [lo, hi], "GHs": round(PER_GPU / best / 1e9, 3), "ms": round(best * 1e3, 2),
               "result": list(res),
               "launches": [{"J": x["J"], "C2": x["C2"], "EX": x["EX"], "nonces": x["nonces"],
                             "ms": round(x["ms"], 3),
                             "GHs": round(x["nonces"] / (x["ms"] * 1e-3) / 1e9, 3) if x["ms"] else None}
                            for x in launches]}
        print(json.dumps(row), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
