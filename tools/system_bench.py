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
import hashlib
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bitcoin-miner_amd", "bin")
LIB = os.path.join(ROOT, "bitcoin-miner_amd", "lib")
NATIVE_MINER = os.path.join(LIB, "gpuhash_miner")
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from bitcoin import SEND_COPIES  # noqa: E402


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
    ap.add_argument("--job-bits", type=int, default=0, help="GPUHASH_JOB_SIZE = 2^bits (0: the server's default)")
    ap.add_argument("--kill-after", type=float, default=3.0, help="SIGKILL one miner after s (<0: never)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--adaptive", action="store_true",
                    help="the server sizes jobs per miner (GPUHASH_JOB_SECONDS=0.5) instead of fixed 2^job-bits jobs")
    ap.add_argument("--native", action="store_true",
                    help="miners are the compiled program (lib/gpuhash_miner) instead of bin/miner")
    ap.add_argument("--compiled", action="store_true",
                    help="server, miners and clients all compiled (lib/gpuhash_{server,miner,client})")
    ap.add_argument("--epoch-ms", type=int, default=None,
                    help="LSP_EPOCH_MILLIS for every program (default: none, the reference's 2000)")
    ap.add_argument("--epoch-limit", type=int, default=None,
                    help="LSP_EPOCH_LIMIT for every program (default: none, the reference's 5)")
    ap.add_argument("--send-copies", type=int, default=None,
                    help="LSP_SEND_COPIES for every program (default: none, bitcoin.SEND_COPIES; 1 = as specified)")
    ap.add_argument("--depth", type=int, default=None, help="GPUHASH_MINER_DEPTH (default: the server's)")
    ap.add_argument("--no-backup", action="store_true", help="GPUHASH_BACKUP=0: no speculative copies")
    ap.add_argument("--copies", type=int, default=None, help="GPUHASH_COPIES (default: the server's)")
    ap.add_argument("--label", default="", help="free text copied to the output line")
    ap.add_argument("--server-log", default=None, help="write the server's stderr here, each line with its time")
    ap.add_argument("--compiled-server", action="store_true",
                    help="the server is lib/gpuhash_server (miners and clients as chosen otherwise)")
    ap.add_argument("--emulate", type=float, default=0.0,
                    help="miners are tools/emu_miner.py sleeping n/RATE per job (CPU-only; no verification)")
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs the miners share, for the busy fraction (default: miners, or SYSTEM_BENCH_GPUS)")
    args = ap.parse_args()
    if args.emulate:
        args.no_verify = True

    env = dict(os.environ, LSPNET_CLIENT_READ_DROP=str(args.drop), LSPNET_CLIENT_WRITE_DROP=str(args.drop),
               LSPNET_SERVER_READ_DROP=str(args.drop), LSPNET_SERVER_WRITE_DROP=str(args.drop))
    if args.epoch_ms is not None:
        env["LSP_EPOCH_MILLIS"] = str(args.epoch_ms)
    if args.epoch_limit is not None:
        env["LSP_EPOCH_LIMIT"] = str(args.epoch_limit)
    if args.send_copies is not None:
        env["LSP_SEND_COPIES"] = str(args.send_copies)
    port = free_port()
    procs = []

    lines: dict[int, list] = {}  # pid -> [(wall time, stream, line)], drained by threads

    def drain(p, stream, name):
        for line in stream:
            lines[p.pid].append((time.time(), name, line.rstrip("\n")))

    def start(argv, native=False, **kw):
        p = subprocess.Popen(argv if native else [sys.executable] + argv, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, text=True, **kw)
        procs.append(p)
        lines[p.pid] = []
        for stream, name in ((p.stdout, "out"), (p.stderr, "err")):
            threading.Thread(target=drain, args=(p, stream, name), daemon=True).start()
        return p

    try:
        senv = dict(env, GPUHASH_SERVER_LOG="1")
        if args.depth is not None:
            senv["GPUHASH_MINER_DEPTH"] = str(args.depth)
        if args.no_backup:
            senv["GPUHASH_BACKUP"] = "0"
        if args.copies is not None:
            senv["GPUHASH_COPIES"] = str(args.copies)
        if args.adaptive:
            senv["GPUHASH_JOB_SECONDS"] = "0.5"
        elif args.job_bits:
            senv["GPUHASH_JOB_SIZE"] = str(1 << args.job_bits)
        if args.compiled or args.compiled_server:
            args.native = args.native or args.compiled
            server = start([os.path.join(LIB, "gpuhash_server"), str(port)], native=True, env=senv)
        else:
            server = start([os.path.join(BIN, "server"), str(port)], env=senv)
        time.sleep(0.5)
        ngpu = int(os.environ.get("SYSTEM_BENCH_GPUS", "0"))
        miners = []
        for i in range(args.miners):
            e = dict(env, GPUHASH_MINER_JOBLOG="1")
            if ngpu:
                e["GPUHASH_DEVICES"] = str(i % ngpu)
            if args.emulate:
                miners.append(start([os.path.join(ROOT, "tools", "emu_miner.py"), f"127.0.0.1:{port}",
                                     str(args.emulate)], env=e))
            elif args.native:
                miners.append(start([NATIVE_MINER, f"127.0.0.1:{port}"], native=True, env=e))
            else:
                miners.append(start([os.path.join(BIN, "miner"), f"127.0.0.1:{port}"], env=e))
        time.sleep(1.5 if args.emulate else 5.0)  # miners open their GPU and join
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
        outs, done_at = [], []
        for c in clients:
            c.wait(timeout=1800)
            time.sleep(0.05)
            got = [(t, ln) for t, name, ln in lines[c.pid] if name == "out" and ln.strip()]
            outs.append(got[-1][1].strip() if got else "")
            done_at.append(got[-1][0] if got else time.time())
            print(f"client done: {outs[-1]}", file=sys.stderr, flush=True)
        t0_wall = time.time() - (time.perf_counter() - t0)
        wall = max(done_at) - t0_wall
        server.send_signal(signal.SIGTERM)
        server.wait(timeout=30)
        for m in miners:
            if m.poll() is None:
                m.send_signal(signal.SIGTERM)
        for m in miners:
            try:
                m.wait(timeout=30)
            except subprocess.TimeoutExpired:
                m.kill()
        time.sleep(0.2)
        log = "\n".join(ln for _, name, ln in lines[server.pid] if name == "err")
        if args.server_log:
            with open(args.server_log, "w") as f:
                f.writelines(f"{t - t0_wall:8.3f} {ln}\n" for t, name, ln in lines[server.pid] if name == "err")
        requeued = log.count("requeued")
        jobs = []  # (miner index, lo, hi, recv, start, end, kernel_s)
        for i, m in enumerate(miners):
            for _, name, ln in lines[m.pid]:
                if name == "err" and " job data=" in ln:
                    kv = dict(tok.split("=", 1) for tok in ln.split() if "=" in tok)
                    jobs.append((kv["data"], int(kv["lo"]), int(kv["hi"]), float(kv["recv"]), float(kv["start"]),
                                 float(kv["end"]), float(kv["kernel_ms"]) / 1000.0))
        ngpus = args.gpus or ngpu or args.miners
        busy = sum(j[6] for j in jobs)
        first = {}  # distinct (data, lo, hi) -> its earliest-finishing copy
        for j in jobs:
            if (j[0], j[1], j[2]) not in first or j[5] < first[(j[0], j[1], j[2])][5]:
                first[(j[0], j[1], j[2])] = j
        useful = sum(j[6] for j in first.values())
        window = (max(j[5] for j in jobs) - min(j[3] for j in jobs)) if jobs else 0.0
        # GPU busy while work was available: from each request's arrival at the server (its
        # log line) until its last nonce was computed (tests/lsp_des.py busy_while_available)
        arrive = {}
        for t, name, ln in lines[server.pid]:
            if name == "err" and ": [Request client-" in ln:
                d = ln.split("[Request ", 1)[1].split()[0]
                arrive.setdefault(hashlib.sha1(d.encode()).hexdigest()[:12], t)
        computed = {}
        for (d, lo, hi), j in first.items():
            computed[d] = max(computed.get(d, 0.0), j[5])
        spans = sorted((arrive[d], computed[d]) for d in arrive if d in computed)
        merged = []
        for a, b in spans:
            if merged and a <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], b)
            else:
                merged.append([a, b])
        avail = sum(b - a for a, b in merged)
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
                        f"{'per-miner jobs (~0.5 s)' if args.adaptive else f'job 2^{args.job_bits}' if args.job_bits else 'default jobs'}, "
                        f"miner killed at {killed}s",
            "label": args.label, "lsp": {"epoch_ms": args.epoch_ms or 2000, "epoch_limit": args.epoch_limit or 5,
                                          "send_copies": args.send_copies or SEND_COPIES},
            "depth": args.depth, "backup": not args.no_backup, "emulated_rate": args.emulate or None,
            "wall_s": round(wall, 3), "system_GHs": round(total / wall / 1e9, 3),
            "gpus": ngpus, "jobs": len(jobs), 
            "gpu_busy_s": round(busy, 3), "useful_busy_s": round(useful, 3),
            "busy_frac_wall": round(useful / (ngpus * wall), 4) if wall else None,
            "miner_window_s": round(window, 3),
            "busy_frac_window": round(useful / (ngpus * window), 4) if window else None,
            "available_s": round(avail, 3),
            "busy_frac_avail": round(useful / (ngpus * avail), 4) if avail else None,
            "copies": len(jobs) - len(first),
            "client_done_s": sorted(round(t - t0_wall, 3) for t in done_at),
            "jobs_requeued": requeued, "all_results_verified": ok, "outputs": outs[:4],
            # a client without a Result says why on stderr (its LSP's account)
            "client_errors": {i: [ln for _, name, ln in lines[c.pid] if name == "err"][-4:]
                              for i, (c, o) in enumerate(zip(clients, outs)) if not o.startswith("Result")},
            "server_log_tail": log.splitlines()[-12:] if any(not o.startswith("Result") for o in outs) else [],
        }), flush=True)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


if __name__ == "__main__":
    main()
