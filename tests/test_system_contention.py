"""CPU: config 5's process topology under CPU pressure, and the LSP diagnostics that name a
lost connection's cause.

One round-4 GPU run of the full-size config-5 test lost a client ("Disconnected") after
2 s (10 epochs x 200 ms) of LSP silence, with no record of why.  Every endpoint now says
why it declares a connection lost (silent epochs, when the peer was last heard) and how
late its own epochs fire (LSP_DIAG=1).  These tests run the programs as separate
processes -- the Python server and clients of the product, and the compiled miner linked
to the CPU oracle's ABI shim (tests/native_programs.py, test infrastructure standing in for
the GPU) -- with config 5's LSP parameters and 10% drops on every role:

* test_config5_shape_under_cpu_pressure: the server pinned to one CPU that eight busy-loop
  processes also run on; every client must get its oracle-exact Result, and the server's
  LSP loop must never fire an epoch a whole epoch late (a CFS-fair share of one CPU keeps
  a mostly-sleeping loop responsive);
* test_stalled_server_is_named: the negative control -- the server process stopped
  (SIGSTOP) for 2.6 s, longer than 10 epochs: the clients print Disconnected, their stderr
  names 10 silent epochs with the server last heard >= 9 epochs (1.8 s) earlier, and the server's own
  loop reports the epoch it fired >= 2 s late.  That is the signature a starved server
  leaves, which the full-size GPU test now records.
"""
from __future__ import annotations

import os
import re
import signal
import socket
import subprocess
import sys
import time

import pytest

import sysdiag
from native_programs import build_miner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bitcoin-miner_amd", "bin")
LSP = {"LSP_EPOCH_MILLIS": "200", "LSP_EPOCH_LIMIT": "10", "LSP_WINDOW_SIZE": "1", "LSP_DIAG": "1"}
DROPS = {f"LSPNET_{r}_{w}_DROP": "10" for r in ("CLIENT", "SERVER") for w in ("READ", "WRITE")}


def free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Procs:
    def __init__(self):
        self.ps = []

    def start(self, argv, cpu=None, **env):
        """`cpu`: pin the process (every thread it will start) to that one CPU from exec on."""
        e = dict(os.environ, **LSP, **{k: str(v) for k, v in env.items()})
        pin = None if cpu is None else (lambda: os.sched_setaffinity(0, {cpu}))
        p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e,
                             preexec_fn=pin)
        self.ps.append(p)
        return p

    def py(self, prog, *args, cpu=None, **env):
        return self.start([sys.executable, os.path.join(BIN, prog), *map(str, args)], cpu=cpu, **env)

    def stop(self, p):
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
        try:
            return p.communicate(timeout=20)[1]
        except subprocess.TimeoutExpired:
            p.kill()
            return p.communicate(timeout=10)[1]

    def kill_all(self):
        for p in self.ps:
            if p.poll() is None:
                p.kill()
        for p in self.ps:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                pass


@pytest.fixture
def procs():
    pr = Procs()
    yield pr
    pr.kill_all()


def _hogs(cpu: int, n: int):
    code = f"import os; os.sched_setaffinity(0, {{{cpu}}})\nwhile True: pass"
    return [subprocess.Popen([sys.executable, "-c", code]) for _ in range(n)]


@pytest.mark.timeout(300)
def test_config5_shape_under_cpu_pressure(procs, tmp_path, oracle):
    miner = build_miner(tmp_path)
    port = free_port()
    cpu = sorted(os.sched_getaffinity(0))[-1]
    server = procs.py("server", port, cpu=cpu, GPUHASH_SERVER_LOG=1, GPUHASH_JOB_SIZE=1 << 21, **DROPS)
    hogs = _hogs(cpu, 8)
    try:
        time.sleep(0.5)
        miners = [procs.start([miner, f"127.0.0.1:{port}"], **DROPS) for _ in range(4)]
        time.sleep(1.0)
        # every thread of the server (its LSP loop included) runs on the contended CPU
        for tid in os.listdir(f"/proc/{server.pid}/task"):
            with open(f"/proc/{server.pid}/task/{tid}/status") as f:
                allowed = [ln.split()[1] for ln in f if ln.startswith("Cpus_allowed_list")]
            assert allowed == [str(cpu)], (tid, allowed)
        sampler = sysdiag.CgroupSampler()
        sampler.start()
        n = 1 << 22
        clients = [procs.py("client", f"127.0.0.1:{port}", f"client-{i:02d}", n, **DROPS) for i in range(8)]
        res = [c.communicate(timeout=240) for c in clients]
        cg = sampler.stop()
    finally:
        for h in hogs:
            h.kill()
            h.wait()
    log = procs.stop(server)
    merr = [procs.stop(m) for m in miners]
    late = sysdiag.lsp_lateness({"server": log, **{f"client-{i}": e for i, (_, e) in enumerate(res)},
                                 **{f"miner-{k}": e for k, e in enumerate(merr)}})
    diag = {"cgroup": cg, "max_late_ms": {k: v["max_late_ms"] for k, v in late.items()}}
    for i, (out, err) in enumerate(res):
        parts = out.split()
        assert parts and parts[0] == "Result", (i, out, err[-800:], diag)
        assert (int(parts[1]), int(parts[2])) == oracle.min(f"client-{i:02d}".encode(), 0, n, threads=8), i
    # the server's loop shared its CPU with 8 busy loops and still fired every epoch within
    # one epoch of its due time (the periodic LSP_DIAG reports prove the loop was measured)
    assert "window max lateness" in log, log[-1500:]
    assert late["server"]["max_late_ms"] < 200, diag
    assert not late["server"]["late_epochs"], diag


@pytest.mark.timeout(120)
def test_stalled_server_is_named(procs, tmp_path):
    miner = build_miner(tmp_path)
    port = free_port()
    server = procs.py("server", port, GPUHASH_SERVER_LOG=1, GPUHASH_JOB_SIZE=1 << 16)
    time.sleep(0.5)
    procs.start([miner, f"127.0.0.1:{port}"])
    time.sleep(0.5)
    # requests long enough (the oracle miner at a few MH/s) to still be running at the stall
    clients = [procs.py("client", f"127.0.0.1:{port}", f"stall-{i}", 1 << 27) for i in range(2)]
    time.sleep(1.5)
    server.send_signal(signal.SIGSTOP)
    time.sleep(2.6)
    server.send_signal(signal.SIGCONT)
    res = [c.communicate(timeout=60) for c in clients]
    time.sleep(0.5)
    log = procs.stop(server)
    for out, err in res:
        assert out.strip() == "Disconnected", (out, err[-800:])
        m = re.search(r"connection lost \(10 silent epochs, peer last heard (\d+) ms ago", err)
        assert m and int(m.group(1)) >= 1750, err[-800:]  # 10 epochs counted from the next one
    lines = [int(x) for x in re.findall(r"lsp-server\[\d+\]: epoch fired (\d+) ms late", log)]
    assert lines and max(lines) >= 2000, log[-1500:]
