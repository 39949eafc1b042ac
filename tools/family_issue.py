#!/usr/bin/env python3
"""Issue rate per layout family: every kernel variant the planner can pick,
each on one search of its own, timed with the library's HIP events and in-kernel shader
clock, then run again under rocprofv3 --pmc for its VALU instructions per nonce.  Answers
whether the families' different GH/s come from their instruction counts (same issue
rate) or from how well each one issues.

  python3 tools/family_issue.py [--reps 3] > fam.jsonl          timing pass (JSON lines)
  rocprofv3 --pmc SQ_INSTS_VALU ... -d DIR -o pmc --output-format csv -- \
      python3 tools/family_issue.py --once                       counter pass
  python3 tools/family_issue.py --summarize DIR fam.jsonl         joined table (JSON lines)

Every case is a range inside one digit group, so each search makes exactly one k_scan
dispatch; the counter pass runs the cases in the same order, and the summary pairs the
k-th scan dispatch with the k-th case.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))

CUS = 256
LANES = 64
OPS_PER_BLOCK = 1378                  # bench.py / SURVEY 8(d): one compression
VALU_PEAK = CUS * 128 * 2.4e9         # bench.py VALU_PEAK_T, lane-ops/s

# (family, message length, digits, policy, log2 nonces)
CASES = [
    ("plain J=2", 0, 10, "auto", 31),
    ("plain J=4 (config 2)", 8, 10, "auto", 31),
    ("plain J=8", 24, 10, "auto", 31),
    ("plain J=13", 44, 10, "auto", 31),
    ("extra block J=13", 45, 10, "auto", 30),
    ("extra block J=15", 53, 10, "auto", 30),
    ("K+W table C2=1 J=0 (config 3)", 120, 10, "auto", 31),
    ("classic straddle C2=1 J=1", 61, 10, "classic", 31),
    ("two-word C2=2", 58, 12, "uniform", 31),
    ("lane table C2=3", 61, 10, "auto", 31),
    ("lane table C2=3", 58, 12, "auto", 31),
]


def case_range(d: int, bits: int) -> tuple[int, int]:
    lo = 10 ** (d - 1) + 12345
    return lo, lo + (1 << bits) - 1


def run(reps: int) -> None:
    import gpuhash
    pols = {"auto": gpuhash.LAYOUT_AUTO, "uniform": gpuhash.LAYOUT_UNIFORM,
            "classic": gpuhash.LAYOUT_CLASSIC, "lanetable": gpuhash.LAYOUT_LANETABLE}
    with gpuhash.Engine([0]) as eng:
        for fam, m, d, pol, bits in CASES:
            msg = bytes((0x61 + i % 26) for i in range(m))
            lo, hi = case_range(d, bits)
            eng.set_layout_policy(pols[pol])
            if reps > 1:
                eng.min(msg, lo, hi)  # warm-up (code object load, buffers)
            recs = []
            for _ in range(reps):
                res = eng.min(msg, lo, hi)
                scans = eng.launches()
                assert len(scans) == 1, (fam, scans)  # one variant, one dispatch
                recs.append(scans[0])
            r = recs[0]
            ms = statistics.median(x["ms"] for x in recs)
            sclk = statistics.median(x["sclk_mhz"] for x in recs)
            ghs = (hi - lo + 1) / ms / 1e6
            comp = gpuhash.compressions_per_nonce(r)
            print(json.dumps({"family": fam, "msg_len": m, "digits": d, "policy": pol,
                              "lower": lo, "upper": hi, "nonces": hi - lo + 1,
                              "variant": f"J={r['J']},C2={r['C2']},EX={r['EX']}",
                              "kernel_ms": round(ms, 3), "sclk_mhz": round(sclk, 1),
                              "GHs": round(ghs, 3),
                              # algorithmic ops: OPS_PER_BLOCK per compression (c + EX), with
                              # SURVEY 8(d)'s c-based count beside it
                              "compressions_per_nonce": comp,
                              "ops_per_nonce": OPS_PER_BLOCK * comp,
                              "ops_per_nonce_c_based": OPS_PER_BLOCK * r["c"],
                              "frac": round(ghs * 1e9 * OPS_PER_BLOCK * comp / VALU_PEAK, 4),
                              "frac_c_based": round(ghs * 1e9 * OPS_PER_BLOCK * r["c"] / VALU_PEAK, 4),
                              "result": list(res)}),
                  flush=True)


def summarize(pmc_dir: str, timing: str) -> None:
    rows = [json.loads(l) for l in open(timing) if l.startswith("{")]
    path = glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True)
    assert path, f"no counter csv under {pmc_dir}"
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path[0])):
        if "k_scan" not in r["Kernel_Name"]:
            continue
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] += float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    disp = sorted(per)
    assert len(disp) == len(rows), (len(disp), len(rows))
    for row, i in zip(rows, disp):
        c = per[i]
        instr = c["SQ_INSTS_VALU"] * LANES / row["nonces"]
        # lane-instructions per CU per clock over the timed launch (in-kernel clock)
        rate = c["SQ_INSTS_VALU"] * LANES / (row["kernel_ms"] * 1e-3 * row["sclk_mhz"] * 1e6 * CUS)
        out = dict(row)
        out.update({"kernel": names[i].split("(")[0][-40:],
                    "valu_lane_instr_per_nonce": round(instr, 1),
                    "salu_instr_per_wave_nonce": round(c["SQ_INSTS_SALU"] / row["nonces"] * LANES, 1),
                    "issue_lane_instr_per_clk_per_cu": round(rate, 2),
                    "issue_frac_of_simd32_peak": round(rate / 128.0, 4)})
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            if k in c:
                out[k] = c[k]
        print(json.dumps(out))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--once", action="store_true", help="counter pass: one search per case")
    ap.add_argument("--summarize", nargs=2, metavar=("PMC_DIR", "TIMING_JSONL"))
    a = ap.parse_args()
    if a.summarize:
        summarize(*a.summarize)
    else:
        run(1 if a.once else a.reps)


if __name__ == "__main__":
    main()
