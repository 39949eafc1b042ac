#!/usr/bin/env python3
"""Every message length 0-63 (and 64-127 with --long) at 10-13 digits: one AUTO search of
2^33 nonces inside the digit group, its GH/s, in-kernel clock and the kernel variants it
ran.  Finds (length, digits) pairs that run below their layout family's rate.  One JSON
line per case (tools/gpu_session.sh lsweep)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
import gpuhash  # noqa: E402

N = 1 << 33
lens = range(64, 128) if "--long" in sys.argv else range(0, 64)
with gpuhash.Engine([0]) as e:
    for m in lens:
        msg = bytes(0x61 + (i % 26) for i in range(m))
        for d in (10, 11, 12, 13):
            lo = 10 ** (d - 1) + 12345
            e.min(msg, lo, lo + (1 << 24))  # warm
            t = time.perf_counter()
            res = e.min(msg, lo, lo + N - 1)
            dt = time.perf_counter() - t
            recs = e.launches()
            top = max(recs, key=lambda r: r["nonces"])
            kms = sum(r["ms"] for r in recs)
            ops = sum(r["nonces"] * 1378 * gpuhash.compressions_per_nonce(r) for r in recs)
            print(json.dumps({"msg_len": m, "digits": d, "GHs": round(N / dt / 1e9, 3),
                              "kernel_GHs": round(N / kms / 1e6, 3),
                              "variants": sorted({(r["J"], r["C2"], r["EX"]) for r in recs}),
                              "compressions_per_nonce": round(ops / 1378 / N, 3),
                              # algorithmic ops (1,378 per compression, c + EX) over the kernels'
                              # HIP-event time, against the 78.6 T VALU peak (bench.py)
                              "frac": round(ops / (kms * 1e-3) / (256 * 128 * 2.4e9), 4),
                              "sclk_mhz": round(top["sclk_mhz"]), "result": list(res)}), flush=True)
