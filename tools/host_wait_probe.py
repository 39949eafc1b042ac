#!/usr/bin/env python3
"""tools/host_wait_probe.py -- host CPU a miner burns while it waits for the GPU
(VERDICT r04 item 1, step 3).

A miner spends nearly all its time inside gpuhash_min waiting for its scan kernels.  For
each host-wait mode of the engine (GPUHASH_HOST_WAIT = stream | event | poll, csrc/
gpuhash.cpp), this runs P processes at once that share the GPU like config 5's miners, each
doing `jobs` searches of `bradfitz` over 2^span nonces, and reports per process: wall time,
CPU time (getrusage: user + sys, every thread), CPU / wall, the busiest thread's CPU, the
GH/s, and the result (which must agree across modes).  The cgroup's cpu.stat throttling
counters are sampled around each mode.  One JSON line per mode.

  python tools/host_wait_probe.py [--procs 8] [--span 34] [--jobs 3] [--modes stream,event,poll]
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _thread_cpu() -> dict:
    """tid -> (name, utime + stime seconds) of every thread of this process."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
            name = st[st.index("(") + 1:st.rindex(")")]
            f_ = st[st.rindex(")") + 2:].split()
            out[tid] = (name, (int(f_[11]) + int(f_[12])) / tick)
        except (OSError, ValueError):
            pass
    return out


def child(span: int, jobs: int) -> None:
    sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
    import gpuhash
    eng = gpuhash.Engine([0])
    eng.min(b"bradfitz", 0, 1 << 24)  # load the code objects
    n = 1 << span
    th0, r0, t0 = _thread_cpu(), resource.getrusage(resource.RUSAGE_SELF), time.perf_counter()
    res = []
    for j in range(jobs):
        res.append(eng.min(b"bradfitz", j * n, (j + 1) * n - 1))
    wall = time.perf_counter() - t0
    r1, th1 = resource.getrusage(resource.RUSAGE_SELF), _thread_cpu()
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    per = sorted(((th1[t][1] - th0.get(t, ("", 0.0))[1], th1[t][0]) for t in th1), reverse=True)
    print(json.dumps({"wall_s": round(wall, 3), "cpu_s": round(cpu, 3), "cpu_per_wall": round(cpu / wall, 3),
                      "busiest_thread": [round(per[0][0], 3), per[0][1]] if per else None,
                      "threads": len(th1), "GHs": round(jobs * n / wall / 1e9, 3), "results": res}), flush=True)
    eng.close()


def cgroup_stat() -> dict:
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return {}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--span", type=int, default=34)
    ap.add_argument("--jobs", type=int, default=3)
    ap.add_argument("--modes", default="stream,event,poll")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a.span, a.jobs)
    for mode in a.modes.split(","):
        env = dict(os.environ, GPUHASH_HOST_WAIT=mode)
        c0, t0 = cgroup_stat(), time.perf_counter()
        ps = [subprocess.Popen([sys.executable, __file__, "--child", "--span", str(a.span), "--jobs", str(a.jobs)],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
              for _ in range(a.procs)]
        outs = [p.communicate(timeout=600) for p in ps]
        wall = time.perf_counter() - t0
        c1 = cgroup_stat()
        rows = []
        for p, (o, e) in zip(ps, outs):
            if p.returncode != 0:
                print(json.dumps({"mode": mode, "error": e[-1500:]}), flush=True)
                sys.exit(1)
            rows.append(json.loads(o.strip().splitlines()[-1]))
        res = {tuple(map(tuple, r["results"])) for r in rows}
        d = {k: c1.get(k, 0) - c0.get(k, 0) for k in ("usage_usec", "nr_throttled", "throttled_usec", "nr_periods")}
        print(json.dumps({"mode": mode, "procs": a.procs, "span": a.span, "jobs": a.jobs, "wall_s": round(wall, 2),
                          "sum_cpu_s": round(sum(r["cpu_s"] for r in rows), 2),
                          "cpu_per_wall_each": [r["cpu_per_wall"] for r in rows],
                          "busiest_thread_each": [r["busiest_thread"] for r in rows],
                          "GHs_total": round(sum(r["GHs"] for r in rows), 2),
                          "results_agree": len(res) == 1, "cgroup_delta": d}), flush=True)


if __name__ == "__main__":
    main()
