#!/usr/bin/env python3
"""Does SIGKILLing one process whose kernel is running on a shared GPU disturb the
others?  (in one config-5 run a second miner went silent the moment the
first was killed.)  N worker processes share the one GPU, each calling gpuhash_min on
2^JOB_BITS-nonce ranges in a loop and printing every call's outcome; after KILL_AFTER
seconds worker 1 is SIGKILLed, the rest keep going for AFTER seconds and are then
stopped.  One JSON line per round: which workers' calls failed, and how.

  python tools/kill_probe.py [--rounds 4] [--workers 8] [--job-bits 34]
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import sys, time
sys.path.insert(0, sys.argv[1])
import gpuhash
bits = int(sys.argv[2])
eng = gpuhash.Engine([0])
print("ready", flush=True)
k = 0
while True:
    lo = (k << bits)
    t = time.time()
    try:
        r = eng.min(b"kill-probe", lo, lo + (1 << bits) - 1)
        print(f"ok {k} {time.time() - t:.3f}", flush=True)
    except Exception as e:  # the probe's question: does this ever happen?
        print(f"error {k} {type(e).__name__}: {e}", flush=True)
        eng.close()
        eng = gpuhash.Engine([0])
    k += 1
'''


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--job-bits", type=int, default=34)
    ap.add_argument("--kill-after", type=float, default=3.0)
    ap.add_argument("--after", type=float, default=10.0)
    a = ap.parse_args()
    for rnd in range(a.rounds):
        procs, outs = [], []
        for i in range(a.workers):
            p = subprocess.Popen([sys.executable, "-u", "-c", WORKER, os.path.join(ROOT, "bitcoin-miner_amd"),
                                  str(a.job_bits)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            lines: list = []
            threading.Thread(target=lambda p=p, lines=lines: [lines.append((time.time(), ln.strip())) for ln in p.stdout],
                             daemon=True).start()
            procs.append(p)
            outs.append(lines)
        t0 = time.time()
        while time.time() - t0 < 60 and not all(any(ln == "ready" for _, ln in o) for o in outs):
            time.sleep(0.1)
        time.sleep(a.kill_after)
        t_kill = time.time()
        procs[1].send_signal(signal.SIGKILL)
        time.sleep(a.after)
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(20)
            except subprocess.TimeoutExpired:
                p.kill()
        time.sleep(0.2)
        rows = []
        for i, o in enumerate(outs):
            ok_after = sum(1 for t, ln in o if ln.startswith("ok") and t > t_kill)
            errors = [ln for t, ln in o if ln.startswith("error") or "Traceback" in ln or "rror" in ln]
            rows.append({"worker": i, "killed": i == 1, "returncode": procs[i].returncode,
                         "calls_ok_after_kill": ok_after, "errors": errors[:4]})
        print(json.dumps({"round": rnd, "workers": a.workers, "job_bits": a.job_bits,
                          "disturbed": [r["worker"] for r in rows if not r["killed"] and r["errors"]],
                          "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
