#!/usr/bin/env python3
"""CPU soak of the compiled programs: lib-less builds of the server, client and miner
(the miner on the oracle-backed ABI shim, tests/native_programs.py), under a sanitizer,
over LSP/UDP with lspnet drops on every role.  Waves of clients with random messages
(non-ASCII, JSON-escaped characters) and random ranges run against a server with a random
job size while miners are SIGKILLed and replaced; every printed "Result h n" must equal
the oracle's argmin of the client's range, and no process may report a sanitizer error.

  python tools/cpu_system_soak.py [--seconds 300] [--seed 1] [--san address,undefined]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import signal
import sys
import tempfile
import time
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

ALPHABET = "abcXYZ019 _-\"\\/<>&\t\né✓€ "


def free_port() -> int:
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--san", default="address,undefined", help="'' for plain builds")
    ap.add_argument("--drop", type=int, default=15)
    args = ap.parse_args()
    import hash_oracle
    from native_programs import Procs, build_client, build_miner, build_server
    rng = random.Random(args.seed)
    oracle = hash_oracle.load_c_oracle()
    san = args.san or None
    d = Path(tempfile.mkdtemp(prefix="cpu_soak_"))
    server_bin, client_bin, miner_bin = build_server(d, san), build_client(d, san), build_miner(d, san)
    lsp_env = {"LSP_EPOCH_LIMIT": "20", "LSP_EPOCH_MILLIS": "40", "LSP_WINDOW_SIZE": str(rng.choice([1, 2, 5]))}
    drops = {f"LSPNET_{r}_{w}_DROP": args.drop for r in ("SERVER", "CLIENT") for w in ("READ", "WRITE")}
    stats = {"waves": 0, "requests": 0, "nonces": 0, "mismatches": 0, "no_result": 0, "kills": 0}
    t_end = time.time() + args.seconds
    pr = Procs()
    try:
        while time.time() < t_end:
            port = free_port()
            job = rng.choice([1, 7, 100, 997, 5000, 30000])
            depth = rng.choice([1, 1, 2])
            server = pr.start([server_bin, str(port)],
                              dict(lsp_env, GPUHASH_JOB_SIZE=job, GPUHASH_MINER_DEPTH=depth, GPUHASH_SERVER_LOG=1, **drops))
            time.sleep(0.2)
            miners = [pr.start([miner_bin, f"127.0.0.1:{port}"], dict(lsp_env, **drops))
                      for _ in range(rng.randint(1, 4))]
            reqs = []
            for _ in range(rng.randint(1, 8)):
                msg = "".join(rng.choice(ALPHABET) for _ in range(rng.randint(0, 70)))
                # at most ~150 jobs per request: each costs a few LSP round trips, and with
                # drops on every role a round trip averages tens of ms
                max_nonce = rng.randint(0, min(40000, 150 * job))
                c = pr.start([client_bin, f"127.0.0.1:{port}", msg, str(max_nonce)], lsp_env)
                reqs.append((c, msg, max_nonce))
            time.sleep(rng.uniform(0.05, 0.5))
            if rng.random() < 0.5 and len(miners) > 1:  # lose a miner mid-wave, start a fresh one
                v = rng.choice(miners)
                v.send_signal(signal.SIGKILL)
                stats["kills"] += 1
                miners.append(pr.start([miner_bin, f"127.0.0.1:{port}"], dict(lsp_env, **drops)))
            for c, msg, max_nonce in reqs:
                try:
                    out, _ = c.communicate(timeout=120)
                except Exception:
                    c.kill()
                    out = ""
                want = oracle.min(msg.encode(), 0, max_nonce)
                stats["requests"] += 1
                stats["nonces"] += max_nonce + 1
                if not out.startswith("Result "):
                    stats["no_result"] += 1
                    print(json.dumps({"no_result": out, "msg": msg, "max": max_nonce}), flush=True)
                elif tuple(int(x) for x in out.split()[1:3]) != want:
                    stats["mismatches"] += 1
                    print(json.dumps({"mismatch": out, "want": want, "msg": msg, "max": max_nonce}), flush=True)
            bad = stats["no_result"] + stats["mismatches"]
            server.send_signal(signal.SIGTERM)
            pr.stop_all()
            if bad:
                print(json.dumps({"wave": stats["waves"], "job": job, "depth": depth, "window": lsp_env,
                                  "miner_rcs": [m.returncode for m in miners]}), flush=True)
                print("server log tail:\n" + pr.errs[0][-3000:], flush=True)
                break
            if pr.sanitizer_reports():
                print(pr.sanitizer_reports()[0][-4000:], flush=True)
                stats["sanitizer_reports"] = len(pr.sanitizer_reports())
                break
            pr = Procs()
            stats["waves"] += 1
            print(json.dumps(stats), flush=True)
    finally:
        pr.stop_all()
    stats["ok"] = stats["mismatches"] == 0 and stats["no_result"] == 0 and "sanitizer_reports" not in stats
    print(json.dumps(stats), flush=True)
    sys.exit(0 if stats["ok"] else 1)


if __name__ == "__main__":
    main()
