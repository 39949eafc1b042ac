"""Miner -- bitcoin/miner/miner.go of the reference (stub; "TODO: implement this!" at :15),
written to p1.pdf pp.13-15 with the min-hash loop replaced by ONE call into the gfx950
engine (gpuhash_min through the C ABI):

    Join -> loop { Read Request -> gpuhash_min(Data, Lower, Upper) -> Write Result }
    and shut down when the server is lost (p1.pdf p.15).

    python bitcoin-miner_amd/bin/miner host:port      (GPUHASH_DEVICES=0,1 narrows devices)
"""
from __future__ import annotations

import hashlib
import os
import sys
import time

import lsp

from . import EMPTY_RESULT, MsgType, NewJoin, NewResult, marshal, params_from_env, unmarshal


def _log(line: str) -> None:  # stderr only: the programs' stdout is graded (p1.pdf p.15)
    print(f"miner: {line}", file=sys.stderr, flush=True)


def open_engine():
    import gpuhash
    devs = os.environ.get("GPUHASH_DEVICES")
    return gpuhash.Engine([int(x) for x in devs.split(",")] if devs else None)


def run(hostport: str, engine=None, params=None, on_client=None) -> int:
    """Serves jobs until the server is lost.  `engine` is anything with
    .min(msg, lower, upper) -> (hash, nonce); by default the gpuhash Engine.
    `on_client` (tests) receives the LSP client once connected."""
    try:
        c = lsp.NewClient(hostport, params or params_from_env())
    except lsp.LSPError as e:
        _log(str(e))
        return 1
    if on_client is not None:
        on_client(c)
    engine = engine or open_engine()
    jobs = 0
    # GPUHASH_MINER_JOBLOG=1: one stderr line per job (wall-clock receive/start/end and the
    # engine's kernel ms), from which tools/system_bench.py measures how busy the GPU was
    joblog = os.environ.get("GPUHASH_MINER_JOBLOG", "") not in ("", "0")
    _log(f"joined as connection {c.ConnID()} (pid {os.getpid()})")
    try:
        c.Write(marshal(NewJoin()))
        while True:
            try:
                raw = c.Read()
                t_recv = time.time()
                m = unmarshal(raw)
            except (ValueError, KeyError):
                continue  # not a Message: ignore, like the server does
            if m.Type != MsgType.Request:
                continue
            if m.Lower > m.Upper:
                # the spec'd loop runs zero times; answer with the min over the empty set
                # (the top of the key order, a no-op in the server's merge) so the job
                # does not stay in flight
                c.Write(marshal(NewResult(*EMPTY_RESULT)))
                continue
            # was: for n := m.Lower; n <= m.Upper; n++ { h := bitcoin.Hash(m.Data, n) ... }
            t_start = time.time()
            try:
                h, n = engine.min(m.Data, m.Lower, m.Upper)
                t_end = time.time()
            except Exception as e:
                if isinstance(e, (ValueError, TypeError)) or getattr(e, "is_argument_error", False):
                    # deterministic (EINVAL/ETOOLONG): no Result can be sent for this job,
                    # and skipping it would leave it in flight forever (the server pairs
                    # each Result with the miner's OLDEST job, so with two jobs per miner
                    # the next Result would even answer the wrong request).  So the miner
                    # exits like on a device error: the server sees the connection lost,
                    # requeues the job, and its requeue cap (server.MAX_REQUEUES) ends the
                    # request with Disconnected at the client after the job has failed a
                    # few miners.  The in-tree servers validate requests, so their jobs
                    # never get here.
                    _log(f"job {m} failed: {e}; exiting so the server requeues it")
                    return 1
                # a device error (no device, HIP failure) propagates: the miner exits and
                # the server requeues the job on another miner (p1.pdf p.15), at most
                # server.MAX_REQUEUES times
                raise
            c.Write(marshal(NewResult(h, n)))
            jobs += 1
            if joblog:
                st = engine.stats() if hasattr(engine, "stats") else {}
                tag = hashlib.sha1(m.Data.encode("utf-8", "surrogatepass")).hexdigest()[:12]
                _log(f"job data={tag} lo={m.Lower} hi={m.Upper} recv={t_recv:.6f} start={t_start:.6f} "
                     f"end={t_end:.6f} kernel_ms={st.get('kernel_ms', 0.0):.3f}")
    except lsp.LSPError as e:
        _log(f"server lost after {jobs} job(s): {e}")
        return 0  # server lost: shut down (p1.pdf p.15)
    finally:
        c.Close()


def main(argv=None) -> int:
    argv = sys.argv if argv is None else argv
    if len(argv) != 2:  # miner.go:9-13
        print("Usage: ./miner <hostport>")
        return 0
    return run(argv[1])


if __name__ == "__main__":
    sys.exit(main())
