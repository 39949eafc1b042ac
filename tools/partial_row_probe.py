#!/usr/bin/env python3
"""Rate of the two-word uniform layout (C2 = 2) against the classic straddle layout when
a search covers only part of a 256-lane row: m = 60, d = 10 (3 lane digits in block B-1,
7 loop digits in block B, R = 10^7 loop values per lane), searches of `lanes` lane
values from 10^9.  One subprocess per library (tools/variants/<name>/libgpuhash.so),
interleaved over rounds; prints GH/s per (lanes, policy) and checks all answers agree.

  python tools/partial_row_probe.py [rounds] [variant,variant,...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "tools", "variants")
LANES = [32, 45, 64, 100, 128, 160, 192, 215, 256, 300, 330, 400, 512]

CHILD = r'''
import json, sys, time
sys.path.insert(0, sys.argv[2])
import gpuhash
m = b"u" * 60
out = {}
with gpuhash.Engine([0], lib_path=sys.argv[1]) as e:
    for lanes in json.loads(sys.argv[3]):
        lo, hi = 10**9, 10**9 + lanes * 10**7 - 1
        for pol, name in ((gpuhash.LAYOUT_UNIFORM, "u2"), (gpuhash.LAYOUT_CLASSIC, "cj1"), (gpuhash.LAYOUT_AUTO, "auto")):
            e.set_layout_policy(pol)
            e.min(m, lo, hi)
            best, res = 1e9, None
            for _ in range(2):
                t = time.perf_counter(); res = e.min(m, lo, hi); dt = time.perf_counter() - t
                best = min(best, dt)
            c2 = sorted({r["C2"] for r in e.launches()})
            out[f"{lanes}/{name}"] = {"GHs": round((hi - lo + 1) / best / 1e9, 3), "res": list(res), "C2": c2}
print(json.dumps(out))
'''

names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["product"]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 1
best = {n: {} for n in names}
answers = {}
for rnd in range(rounds):
    for n in names:
        r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(VDIR, n, "libgpuhash.so"),
                            os.path.join(ROOT, "bitcoin-miner_amd"), json.dumps(LANES)],
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(json.dumps({"variant": n, "error": r.stderr[-800:]}), flush=True)
            sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        for k, v in d.items():
            best[n][k] = max(best[n].get(k, 0.0), v["GHs"])
            lanes = k.split("/")[0]
            answers.setdefault(lanes, set()).add(tuple(v["res"]))
            if k.endswith("auto"):
                best[n][k + "_C2"] = v["C2"]
        print(json.dumps({"variant": n, "round": rnd}), flush=True)
for n in names:
    for lanes in LANES:
        row = {"variant": n, "lanes": lanes}
        row.update({p: best[n][f"{lanes}/{p}"] for p in ("u2", "cj1", "auto")})
        row["auto_C2"] = best[n][f"{lanes}/auto_C2"]
        print(json.dumps(row), flush=True)
print(json.dumps({"same_answers": all(len(v) == 1 for v in answers.values())}), flush=True)
