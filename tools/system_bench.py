#!/usr/bin/env python3
"""System-level run of BASELINE config 5 (or a scaled version): server + GPU miners +
clients as separate processes over LSP/UDP on localhost, with lspnet drops and one miner
SIGKILLed mid-run.  Prints one JSON line: wall time, system GH/s, and whether every
client's printed result equals a direct search of its range (verified on the GPU engine,
itself parity-tested against the oracle) and re-hashes on the oracle.

  python tools/system_bench.py                       # config 5: 16 clients x 2^36, 8 miners
  python tools/system_bench.py --clients 4 --bits 32 --miners 2
  python tools/system_bench.py --native                # miners = the compiled lib/gpuhash_miner
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bitcoin-miner_amd", "bin")
LIB = os.path.join(ROOT, "bitcoin-miner_amd", "lib")
NATIVE_MINER = os.path.join(LIB, "gpuhash_miner")
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--miners", type=int, default=8)
    ap.add_argument("--bits", type=int, default=36, help="maxNonce = 2^bits per client")
    ap.add_argument("--drop", type=int, default=10, help="lspnet read+write drop %% on every role")
    ap.add_argument("--job-bits", type=int, default=34)
    ap.add_argument("--kill-after", type=float, default=3.0, help="SIGKILL one miner after s (<0: never)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--adaptive", action="store_true",
                    help="the server sizes jobs per miner (GPUHASH_JOB_SECONDS=0.5) instead of fixed 2^job-bits jobs")
    ap.add_argument("--native", action="store_true",
                    help="miners are the compiled program (lib/gpuhash_miner) instead of bin/miner")
    ap.add_argument("--compiled", action="store_true",
                    help="server, miners and clients all compiled (lib/gpuhash_{server,miner,client})")
    args = ap.parse_args()

    env = dict(os.environ, LSP_EPOCH_MILLIS="500", LSP_EPOCH_LIMIT="10",
               LSPNET_CLIENT_READ_DROP=str(args.drop), LSPNET_CLIENT_WRITE_DROP=str(args.drop),
               LSPNET_SERVER_READ_DROP=str(args.drop), LSPNET_SERVER_WRITE_DROP=str(args.drop))
    port = free_port()
    procs = []

    def start(argv, native=False, **kw):
        p = subprocess.Popen(argv if native else [sys.executable] + argv, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, text=True, **kw)
        procs.append(p)
        return p

    try:
        senv = dict(env, GPUHASH_SERVER_LOG="1")
        if args.adaptive:
            senv["GPUHASH_JOB_SECONDS"] = "0.5"
        else:
            senv["GPUHASH_JOB_SIZE"] = str(1 << args.job_bits)
        if args.compiled:
            args.native = True
            server = start([os.path.join(LIB, "gpuhash_server"), str(port)], native=True, env=senv)
        else:
            server = start([os.path.join(BIN, "server"), str(port)], env=senv)
        time.sleep(0.5)
        ngpu = int(os.environ.get("SYSTEM_BENCH_GPUS", "0"))
        miners = []
        for i in range(args.miners):
            e = dict(env)
            if ngpu:
                e["GPUHASH_DEVICES"] = str(i % ngpu)
            if args.native:
                miners.append(start([NATIVE_MINER, f"127.0.0.1:{port}"], native=True, env=e))
            else:
                miners.append(start([os.path.join(BIN, "miner"), f"127.0.0.1:{port}"], env=e))
        time.sleep(5.0)  # miners open their GPU and join
        max_nonce = (1 << args.bits)
        t0 = time.perf_counter()
        if args.compiled:
            clients = [start([os.path.join(LIB, "gpuhash_client"), f"127.0.0.1:{port}", f"client-{i:02d}",
                              str(max_nonce)], native=True, env=env) for i in range(args.clients)]
        else:
            clients = [start([os.path.join(BIN, "client"), f"127.0.0.1:{port}", f"client-{i:02d}", str(max_nonce)],
                             env=env) for i in range(args.clients)]
        killed = None
        if args.kill_after >= 0 and args.miners > 1:
            time.sleep(args.kill_after)
            miners[-1].send_signal(signal.SIGKILL)
            killed = args.kill_after
        outs = []
        for c in clients:
            out, _ = c.communicate(timeout=1800)
            outs.append(out.strip())
            print(f"client done: {out.strip()}", file=sys.stderr, flush=True)
        wall = time.perf_counter() - t0
        server.send_signal(signal.SIGTERM)
        log = server.communicate(timeout=30)[1]
        requeued = log.count("requeued")
        ok = None
        if not args.no_verify:
            import gpuhash
            import hash_oracle
            oracle = hash_oracle.load_c_oracle()
            ok = True
            with gpuhash.Engine([0]) as eng:
                for i, out in enumerate(outs):
                    parts = out.split()
                    msg = f"client-{i:02d}".encode()
                    good = (len(parts) == 3 and parts[0] == "Result"
                            and (int(parts[1]), int(parts[2])) == eng.min(msg, 0, max_nonce)
                            and oracle.hash(msg, int(parts[2])) == int(parts[1]))
                    ok = ok and good
        total = args.clients * (max_nonce + 1)
        print(json.dumps({
            "workload": f"config 5: {args.clients} clients x [0, 2^{args.bits}], {args.miners} GPU miners "
                        f"({'all compiled: gpuhash_server/miner/client' if args.compiled else 'lib/gpuhash_miner' if args.native else 'bin/miner'}), "
                        f"lspnet drop {args.drop}% on every role, "
                        f"{'per-miner jobs (~0.5 s)' if args.adaptive else f'job 2^{args.job_bits}'}, "
                        f"miner killed at {killed}s",
            "wall_s": round(wall, 3), "system_GHs": round(total / wall / 1e9, 3),
            "jobs_requeued": requeued, "all_results_verified": ok, "outputs": outs[:4],
        }), flush=True)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


if __name__ == "__main__":
    main()
