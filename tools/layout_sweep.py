#!/usr/bin/env python3
"""Kernel throughput per message layout: for message lengths m and nonce digit counts d,
time gpuhash_min over 2^bits nonces of d digits and report the scan kernel's GH/s with
its variant (J, C2, EX) and loop digits q -- shows which layouts the planner handles
well and which cost more (extra padding block, J=0 chains, q=1 setups).

  python tools/layout_sweep.py [--bits 31] [--lens 0,8,20,44,45,53,56,60,64,100,120]
                               [--policies auto,classic,lanetable,uniform]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))


def loop_digits(m: int, d: int) -> int:
    """Digits in the last digit-bearing 32-bit word (the per-nonce word), as plan.cpp."""
    e_abs = m + d  # index of the last digit byte (L - 1 with L = m + 1 + d)
    wstart = 64 * (e_abs // 64) + 4 * ((e_abs % 64) // 4)
    return e_abs - max(wstart, m + 1) + 1


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=31)
    ap.add_argument("--lens", default="0,8,12,20,30,44,45,50,53,54,56,58,60,63,64,100,119,120")
    ap.add_argument("--digits", default="10,12")
    ap.add_argument("--policies", default="auto")
    args = ap.parse_args()
    import gpuhash
    eng = gpuhash.Engine([0])
    pols = {"auto": gpuhash.LAYOUT_AUTO, "uniform": gpuhash.LAYOUT_UNIFORM,
            "classic": gpuhash.LAYOUT_CLASSIC, "lanetable": gpuhash.LAYOUT_LANETABLE}
    rows = []
    for m, d, pol in [(m, d, pol) for m in [int(x) for x in args.lens.split(",")]
                      for d in [int(x) for x in args.digits.split(",")] for pol in args.policies.split(",")]:
        eng.set_layout_policy(pols[pol])
        msg = bytes((i * 37 + 11) % 94 + 32 for i in range(m))
        if True:
            lo = 10 ** (d - 1)
            hi = min(lo + (1 << args.bits) - 1, 10 ** d - 1)
            eng.min(msg, lo, lo + 10 ** 6)  # warm
            eng.min(msg, lo, hi)
            recs = eng.launches()
            ms = sum(r["ms"] for r in recs)
            r0 = max(recs, key=lambda r: r["nonces"])
            row = {"msg_len": m, "digits": d, "policy": pol, "nonces": hi - lo + 1, "J": r0["J"], "C2": r0["C2"], "EX": r0["EX"], "c": r0["c"],
                   "q": loop_digits(m, d), "GHs": round((hi - lo + 1) / ms / 1e6, 3)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
