#!/usr/bin/env python3
"""Checks the discrete-event model (tests/lsp_des.py) against real runs of the system:
the same shape run K times through tools/system_bench.py -- real server, real LSP over
UDP with lspnet's drops, real clients, and miners that are either the GPU miner (on the
GPU box) or tools/emu_miner.py (a miner that sleeps n / rate: CPU only) -- and N seeds of
the model, per server policy.  Prints one JSON line per policy with both distributions.

  python tools/validate_des.py --emulate --runs 24 --parallel 6     # CPU, here
  python tools/validate_des.py --runs 8                              # GPU box: one miner, real GPU
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

GPU = 34.6e9
POLICIES = {
    # name: (system_bench args, Scheduler kwargs for the model (None: make_scheduler's), LSP send copies)
    "round5": (["--job-bits", "34", "--depth", "1", "--copies", "1", "--send-copies", "1"],
               dict(job_size=1 << 34, depth=1), 1),
    "single": (["--send-copies", "1"], None, 1),  # today's scheduler, every datagram sent once
    "defaults": ([], None, 3),                    # the programs' defaults (bitcoin.SEND_COPIES)
}


def stats(xs: list[float]) -> dict:
    xs = sorted(xs)
    return {"n": len(xs), "mean": round(statistics.mean(xs), 3), "median": round(xs[len(xs) // 2], 3),
            "p90": round(xs[min(len(xs) - 1, int(0.9 * len(xs)))], 3), "min": round(xs[0], 3),
            "max": round(xs[-1], 3)}


def real_run(args, extra: list[str], k: int) -> dict:
    cmd = [sys.executable, os.path.join(ROOT, "tools", "system_bench.py"), "--clients", str(args.clients),
           "--bits", str(args.bits), "--miners", str(args.miners), "--kill-after", str(args.kill_after),
           "--label", f"run {k}"] + extra
    if args.emulate:
        cmd += ["--emulate", str(GPU)]
    if args.compiled_server:
        cmd += ["--compiled-server"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def model(policy, seeds: int, clients: int, bits: int, client_start: float, miners: int = 1,
          kill_after: float = -1.0, send_copies: int = 1) -> list[dict]:
    import lsp
    import lsp_des
    from bitcoin import server as bserver
    reqs = [(f"client-{i:02d}", 0, 1 << bits) for i in range(clients)]
    kill = (kill_after, miners - 1) if kill_after >= 0 and miners > 1 else None  # system_bench kills the last
    out = []
    for s in range(seeds):
        sch = (bserver.make_scheduler(epoch_s=2.0, send_copies=send_copies) if policy is None
               else bserver.Scheduler(**policy))
        params = lsp.NewParams()
        params.SendCopies = send_copies
        out.append(lsp_des.run_system(sch, [GPU] * miners, 1, reqs, params=params, drop=0.10, seed=s,
                                      client_start=client_start, kill=kill))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--seeds", type=int, default=400)
    ap.add_argument("--parallel", type=int, default=1)
    ap.add_argument("--emulate", action="store_true")
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--bits", type=int, default=35)
    ap.add_argument("--miners", type=int, default=1, help="one GPU each (emulated: one 34.6 GH/s miner each)")
    ap.add_argument("--kill-after", type=float, default=-1.0, help="SIGKILL the last miner this long after the clients start")
    ap.add_argument("--policies", default="round5,single,defaults")
    ap.add_argument("--out", default=None, help="also append each real run's line here")
    ap.add_argument("--compiled-server", action="store_true", help="lib/gpuhash_server instead of bin/server")
    args = ap.parse_args()
    for name in args.policies.split(","):
        extra, kw, send_copies = POLICIES[name]
        def one(k):
            r = real_run(args, extra, k)
            # progress on stdout and the run's line in --out as each run ends (a GPU box
            # kills a command that writes nothing for 3 minutes)
            print(f"{name} run {k}: wall {r['wall_s']} s, busy {r['busy_frac_wall']}, "
                  f"busy while available {r['busy_frac_avail']}", flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(dict(r, policy=name)) + "\n")
            return r

        with cf.ThreadPoolExecutor(args.parallel) as ex:
            runs = list(ex.map(one, range(args.runs)))
        # system_bench.py starts the clients 1.5 s (emulated) or 5 s (GPU) after the miners
        sims = model(kw, args.seeds, args.clients, args.bits, 1.5 if args.emulate else 5.0, args.miners,
                     args.kill_after, send_copies)
        work = args.clients * ((1 << args.bits) + 1)
        print(json.dumps({
            "policy": name, "send_copies": send_copies, "miners": "emulated (sleep n/34.6e9)" if args.emulate else "GPU",
            "server": "lib/gpuhash_server" if args.compiled_server else "bin/server",
            "shape": f"{args.miners} miner(s), {args.clients} clients x [0, 2^{args.bits}], 2 s epochs, limit 5, "
                     f"10% drops" + (f", last miner killed {args.kill_after} s in" if args.kill_after >= 0 else ""),
            "real_makespan_s": stats([r["wall_s"] for r in runs]),
            "model_makespan_s": stats([s["makespan"] for s in sims]),
            "real_GHs": stats([work / r["wall_s"] / 1e9 for r in runs]),
            "model_GHs": stats([work / s["makespan"] / 1e9 for s in sims]),
            "real_busy_frac_wall": stats([r["busy_frac_wall"] for r in runs]),
            "model_busy_frac_wall": stats([work / GPU / args.miners / s["makespan"] for s in sims]),
            "real_busy_frac_avail": stats([r["busy_frac_avail"] or 0.0 for r in runs]),
            "model_busy_frac_avail": stats([s["busy_avail"] for s in sims]),
            "real_all_verified": all(r["all_results_verified"] in (True, None) for r in runs),
        }), flush=True)


if __name__ == "__main__":
    main()
