#!/usr/bin/env python3
"""Does the planner's AUTO layout choice ever lose to a forced one?  For the message
lengths whose nonce digits straddle a block boundary (where AUTO chooses between the
two-word uniform layout, the lane table and the classic one, plan.cpp), several digit
counts and search widths, time the same search under AUTO and every forced policy
(UNIFORM, CLASSIC, LANETABLE) and report AUTO's rate over
the best forced one (1.0 = AUTO picked the faster layout).  Answers must agree.

  python tools/planner_regret.py [--lens 54,...] [--digits 10,11,12] [--bits 26,29,32]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="54,55,56,57,58,59,60,61,62,118,120,122")
    ap.add_argument("--digits", default="10,11,12")
    ap.add_argument("--bits", default="26,29,32")
    args = ap.parse_args()
    import gpuhash
    eng = gpuhash.Engine([0])
    pols = {"auto": gpuhash.LAYOUT_AUTO, "uniform": gpuhash.LAYOUT_UNIFORM, "classic": gpuhash.LAYOUT_CLASSIC,
            "lanetable": gpuhash.LAYOUT_LANETABLE}
    worst = 1e9
    for m in [int(x) for x in args.lens.split(",")]:
        msg = bytes((i * 37 + 11) % 94 + 32 for i in range(m))
        for d in [int(x) for x in args.digits.split(",")]:
            for bits in [int(x) for x in args.bits.split(",")]:
                lo = 10 ** (d - 1) + 12345
                hi = lo + (1 << bits) - 1
                row = {"msg_len": m, "digits": d, "bits": bits}
                res = set()
                for name, pol in pols.items():
                    eng.set_layout_policy(pol)
                    eng.min(msg, lo, hi)
                    best = 1e9
                    for _ in range(3):
                        t = time.perf_counter()
                        r = eng.min(msg, lo, hi)
                        best = min(best, time.perf_counter() - t)
                    res.add(r)
                    row[name] = round((hi - lo + 1) / best / 1e9, 3)
                    if name == "auto":
                        row["auto_C2"] = sorted({x["C2"] for x in eng.launches()})
                row["same"] = len(res) == 1
                row["auto_over_best"] = round(row["auto"] / max(row[k] for k in pols if k != "auto"), 3)
                worst = min(worst, row["auto_over_best"])
                print(json.dumps(row), flush=True)
    eng.set_layout_policy(gpuhash.LAYOUT_AUTO)
    eng.close()
    print(json.dumps({"summary": True, "worst_auto_over_best": worst}), flush=True)


if __name__ == "__main__":
    main()
