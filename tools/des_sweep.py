#!/usr/bin/env python3
"""Runs server policies (Scheduler keyword sets) through the discrete-event model of
tests/lsp_des.py (the real LSP state machine and server core; modelled network, GPUs and
epochs) on the system shapes that matter, and prints one JSON line per (shape, policy).

  python tools/des_sweep.py --shapes node,one --policies '[{"job_size": 68719476736, "depth": 2}]'
  python tools/des_sweep.py --shape one --sizes 34,35,36 --depths 1,2,3     # a size x depth grid
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import lsp  # noqa: E402
import lsp_des  # noqa: E402
from bitcoin import server as bserver  # noqa: E402

GPU = 34.6e9

SHAPES = {
    # gpus, miners per gpu, clients, request bits, kill (s after the clients start, miner)
    "one": ([GPU], 1, 4, 35, None),                 # VERDICT r05 item 1's measurement
    "node": ([GPU] * 8, 1, 16, 36, (1.5, 7)),       # config 5 on an 8-GPU node
    "node_nokill": ([GPU] * 8, 1, 16, 36, None),
    "shared": ([GPU], 8, 16, 36, (3.0, 7)),         # config 5 as run on the 1-GPU box
    "node_big": ([GPU] * 8, 1, 16, 38, (6.0, 7)),   # 16 x 2^38: 16 s of node work
}


class SplitTail(bserver.Scheduler):
    """A measured alternative (not the product): once less than one job per idle miner is
    left to hand out, cut the request's remainder over the idle miners, down to
    job_size / split_frac (policy key "split_frac")."""

    def __init__(self, *a, split_frac: int = 4, **kw):
        super().__init__(*a, **kw)
        self.split_frac = split_frac

    def size_for(self, miner, r):
        size = self.job_size
        idle = sum(1 for q in self.miners.values() if not q)
        pend = sum(x.uncut() for x in self.requests.values() if x.has_pending())
        if idle > 1 and pend < idle * size:
            active = sum(1 for x in self.requests.values() if x.has_pending())
            share = -(-r.uncut() // max(1, idle // max(1, active)))
            size = max(size // self.split_frac, min(size, share))
        return size


def run(shape: str, policy: dict, seeds: int, epoch_ms: int, drop: float, copies: int = 1) -> dict:
    gpus, mpg, nclients, bits, kill = SHAPES[shape]
    params = lsp.NewParams()
    params.EpochMillis = epoch_ms
    params.SendCopies = copies
    reqs = [(f"client-{i:02d}", 0, 1 << bits) for i in range(nclients)]
    ms, eff, avail, spec, disc = [], [], [], [], []
    for seed in range(seeds):
        kw = dict(policy)
        cls = SplitTail if "split_frac" in kw else bserver.Scheduler
        r = lsp_des.run_system(cls(**kw), gpus, mpg, reqs, params=params, drop=drop, kill=kill, seed=seed)
        disc.append(r["disconnected"])  # LSP's own losses: 5 epochs of 19%-lossy silence
        ms.append(r["makespan"])
        eff.append(r["efficiency"])
        avail.append(r["busy_avail"])
        spec.append(r["speculated"])
    ms.sort()
    return {"shape": shape, "epoch_ms": epoch_ms, "drop": drop, "send_copies": copies, "policy": policy,
            "makespan_mean": round(statistics.mean(ms), 3), "makespan_p90": round(ms[int(0.9 * len(ms))], 3),
            "eff_mean": round(statistics.mean(eff), 4), "busy_avail_mean": round(statistics.mean(avail), 4),
            "busy_avail_min": round(min(avail), 4), "copies_mean": round(statistics.mean(spec), 1),
            "disconnected": sum(disc)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", "--shape", default="one")
    ap.add_argument("--policies", default="", help="JSON list of Scheduler keyword dicts")
    ap.add_argument("--sizes", default="34,35,36", help="grid mode: job bits")
    ap.add_argument("--depths", default="1,2,3", help="grid mode: depths")
    ap.add_argument("--extra", default="", help="grid mode: JSON dict added to every policy")
    ap.add_argument("--seeds", type=int, default=20)
    ap.add_argument("--epoch-ms", type=int, default=2000)
    ap.add_argument("--drop", type=float, default=0.10)
    ap.add_argument("--copies", default="1", help="LSP SendCopies values, comma-separated")
    args = ap.parse_args()
    if args.policies:
        policies = json.loads(args.policies)
    else:
        extra = json.loads(args.extra) if args.extra else {}
        policies = [dict(job_size=1 << int(b), depth=int(d), **extra)
                    for b in args.sizes.split(",") for d in args.depths.split(",")]
    for shape in args.shapes.split(","):
        for copies in (int(c) for c in args.copies.split(",")):
            for pol in policies:
                print(json.dumps(run(shape, pol, args.seeds, args.epoch_ms, args.drop, copies)), flush=True)


if __name__ == "__main__":
    main()
