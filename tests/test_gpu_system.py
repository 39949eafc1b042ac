"""GPU: the whole system -- server, GPU-backed miner processes, client processes over
LSP/UDP on localhost (BASELINE configs 1 and 5, reduced in size for a 1-GPU box).

Config 1: `server` + one miner + `client host:port bradfitz 9999` must print exactly
"Result 1419516646206828 9898" (p1.pdf p.15 output format).
Config 5 at full size (test_config5_full_size): 16 clients x [0, 2^36], 8 miners sharing
the GPU, 10% drops on every role, a SIGKILLed miner; all sixteen clients checked against
their CPU goldens (oracle/golden_scan.c) and re-hashed by the oracle, with LSP and cgroup
diagnostics recorded (tests/sysdiag.py).
Config 5 (scaled): 8 clients, 4 miners sharing the GPU, lspnet read and write drops of
10% on every role, and one miner SIGKILLed mid-job.  Every client's printed result must
equal a direct search of its whole range, and the winner must re-hash (oracle) to the
printed hash.
"""
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bitcoin-miner_amd", "bin")


def free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def env(**extra):
    e = dict(os.environ)
    e.update({"LSP_EPOCH_MILLIS": "200", "LSP_EPOCH_LIMIT": "10", "LSP_WINDOW_SIZE": "1"})
    e.update({k: str(v) for k, v in extra.items()})
    return e


class Procs:
    def __init__(self):
        self.ps = []

    def start(self, args, **kw):
        p = subprocess.Popen([sys.executable] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True, **kw)
        self.ps.append(p)
        return p

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


def test_config1_end_to_end(procs):
    port = free_port()
    procs.start([os.path.join(BIN, "server"), str(port)], env=env())
    time.sleep(0.5)
    procs.start([os.path.join(BIN, "miner"), f"127.0.0.1:{port}"], env=env())
    c = procs.start([os.path.join(BIN, "client"), f"127.0.0.1:{port}", "bradfitz", "9999"], env=env())
    out, err = c.communicate(timeout=90)
    assert out.strip() == "Result 1419516646206828 9898", (out, err)


NATIVE_MINER = os.path.join(ROOT, "bitcoin-miner_amd", "lib", "gpuhash_miner")


def start_native(procs, port, **extra):
    p = subprocess.Popen([NATIVE_MINER, f"127.0.0.1:{port}"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, env=env(**extra))
    procs.ps.append(p)
    return p


def test_config1_with_the_compiled_miner(procs):
    """The miner program in C++ (csrc/miner_main.cpp, linked to the product
    libgpuhash.so) between the Python server and client."""
    port = free_port()
    procs.start([os.path.join(BIN, "server"), str(port)], env=env())
    time.sleep(0.5)
    start_native(procs, port)
    c = procs.start([os.path.join(BIN, "client"), f"127.0.0.1:{port}", "bradfitz", "9999"], env=env())
    out, err = c.communicate(timeout=90)
    assert out.strip() == "Result 1419516646206828 9898", (out, err)


def test_compiled_and_python_miners_together_with_drops_and_a_kill(procs, engine, oracle):
    port = free_port()
    drops = dict(LSPNET_CLIENT_READ_DROP=10, LSPNET_CLIENT_WRITE_DROP=10,
                 LSPNET_SERVER_READ_DROP=10, LSPNET_SERVER_WRITE_DROP=10)
    server = procs.start([os.path.join(BIN, "server"), str(port)],
                         env=env(GPUHASH_JOB_SIZE=1 << 32, GPUHASH_SERVER_LOG=1, **drops))
    time.sleep(0.5)
    native = [start_native(procs, port, **drops) for _ in range(2)]
    procs.start([os.path.join(BIN, "miner"), f"127.0.0.1:{port}"], env=env(**drops))
    time.sleep(3.0)
    max_nonce = 1 << 34
    clients = [procs.start([os.path.join(BIN, "client"), f"127.0.0.1:{port}", f"native-{i:02d}",
                            str(max_nonce)], env=env(**drops)) for i in range(6)]
    time.sleep(1.5)
    native[0].send_signal(signal.SIGKILL)  # mid-job: its job must be re-run elsewhere
    for i, c in enumerate(clients):
        parts = c.communicate(timeout=240)[0].split()
        assert parts[0] == "Result", parts
        h, n = int(parts[1]), int(parts[2])
        msg = f"native-{i:02d}".encode()
        assert (h, n) == engine.min(msg, 0, max_nonce), i
        assert oracle.hash(msg, n) == h
    server.send_signal(signal.SIGTERM)
    log = server.communicate(timeout=30)[1]
    assert "requeued" in log, log[-2000:]


LIB = os.path.join(ROOT, "bitcoin-miner_amd", "lib")


def start_bin(procs, argv, **extra):
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env(**extra))
    procs.ps.append(p)
    return p


def test_all_compiled_config1_and_scaled_config5(procs, engine, oracle):
    """gpuhash_server + gpuhash_miner (on the GPU) + gpuhash_client, no Python in the
    data path: config 1's exact output, then 4 clients x 2^34 with 10% drops on every
    role and a SIGKILLed miner."""
    port = free_port()
    drops = dict(LSPNET_CLIENT_READ_DROP=10, LSPNET_CLIENT_WRITE_DROP=10,
                 LSPNET_SERVER_READ_DROP=10, LSPNET_SERVER_WRITE_DROP=10)
    server = start_bin(procs, [os.path.join(LIB, "gpuhash_server"), str(port)],
                       GPUHASH_JOB_SIZE=1 << 32, GPUHASH_SERVER_LOG=1, **drops)
    time.sleep(0.5)
    miners = [start_bin(procs, [os.path.join(LIB, "gpuhash_miner"), f"127.0.0.1:{port}"], **drops)
              for _ in range(3)]
    time.sleep(3.0)
    c = start_bin(procs, [os.path.join(LIB, "gpuhash_client"), f"127.0.0.1:{port}", "bradfitz", "9999"], **drops)
    assert c.communicate(timeout=90)[0] == "Result 1419516646206828 9898\n"
    max_nonce = 1 << 34
    clients = [start_bin(procs, [os.path.join(LIB, "gpuhash_client"), f"127.0.0.1:{port}", f"compiled-{i}",
                                 str(max_nonce)], **drops) for i in range(4)]
    time.sleep(1.0)
    miners[0].send_signal(signal.SIGKILL)
    for i, cl in enumerate(clients):
        parts = cl.communicate(timeout=240)[0].split()
        assert parts[0] == "Result", parts
        h, n = int(parts[1]), int(parts[2])
        msg = f"compiled-{i}".encode()
        assert (h, n) == engine.min(msg, 0, max_nonce), i
        assert oracle.hash(msg, n) == h
    server.send_signal(signal.SIGTERM)
    assert "requeued" in server.communicate(timeout=30)[1]


def test_client_prints_disconnected_without_server(procs):
    c = procs.start([os.path.join(BIN, "client"), f"127.0.0.1:{free_port()}", "bradfitz", "9999"],
                    env=env(LSP_EPOCH_MILLIS=100, LSP_EPOCH_LIMIT=3))
    out, _ = c.communicate(timeout=30)
    assert out.strip() == "Disconnected"


def test_config5_scaled_drops_and_killed_miner(procs, engine, oracle):
    port = free_port()
    drops = dict(LSPNET_CLIENT_READ_DROP=10, LSPNET_CLIENT_WRITE_DROP=10,
                 LSPNET_SERVER_READ_DROP=10, LSPNET_SERVER_WRITE_DROP=10)
    server = procs.start([os.path.join(BIN, "server"), str(port)],
                         env=env(GPUHASH_JOB_SIZE=1 << 32, GPUHASH_SERVER_LOG=1, **drops))
    time.sleep(0.5)
    miners = [procs.start([os.path.join(BIN, "miner"), f"127.0.0.1:{port}"], env=env(**drops))
              for _ in range(4)]
    time.sleep(3.0)  # let the miners open the GPU and join
    max_nonce = 1 << 34
    clients = [procs.start([os.path.join(BIN, "client"), f"127.0.0.1:{port}", f"client-{i:02d}",
                            str(max_nonce)], env=env(**drops)) for i in range(8)]
    time.sleep(1.5)
    miners[1].send_signal(signal.SIGKILL)  # mid-job: its job must be re-run elsewhere
    outs = [c.communicate(timeout=240)[0].strip() for c in clients]
    for i, out in enumerate(outs):
        parts = out.split()
        assert parts[0] == "Result", out
        h, n = int(parts[1]), int(parts[2])
        msg = f"client-{i:02d}".encode()
        assert (h, n) == engine.min(msg, 0, max_nonce), i
        assert oracle.hash(msg, n) == h
    server.send_signal(signal.SIGTERM)
    log = server.communicate(timeout=30)[1]
    assert "lost; job [" in log and "requeued" in log, log[-2000:]  # the killed miner's job was re-run


@pytest.mark.timeout(600)
def test_config5_full_size(procs, engine, oracle, golden):
    """BASELINE configs[4] at full size on the one GPU (p1.pdf pp.14-15): 16 concurrent
    clients "client-00".."client-15", each Request(msg, 0, 2^36); 8 GPU-backed miners (4
    Python, 4 compiled) sharing the GPU; lspnet read and write drops of 10% on every role;
    one miner SIGKILLed mid-job, whose job must be re-run.  Every client is checked against
    its CPU golden (tests/golden/make_golden.py --huge: the SHA-NI / AVX-512 restatement
    over the whole [0, 2^36], all 16 since round 4), and every printed winner is re-hashed
    by the oracle.

    200 ms epochs, 10 of them before a connection counts as lost (2 s), as in the other
    system tests.  Every program runs with LSP_DIAG=1, so a lost connection says why (its
    silent epochs, when the peer was last heard) and each LSP loop reports how late its
    epochs fired; the cgroup's CPU use and CFS throttling are sampled throughout, and the
    miners' CPU time is read before they are stopped.  All of it goes to
    $GPUHASH_DIAG_DIR/config5_diag.json and into the failure message."""
    import time as _t
    import sysdiag
    gold = {r["name"]: r for r in golden["ranges"]}
    port = free_port()
    drops = dict(LSPNET_CLIENT_READ_DROP=10, LSPNET_CLIENT_WRITE_DROP=10,
                 LSPNET_SERVER_READ_DROP=10, LSPNET_SERVER_WRITE_DROP=10, LSP_DIAG=1)
    server = procs.start([os.path.join(BIN, "server"), str(port)], env=env(GPUHASH_SERVER_LOG=1, **drops))
    time.sleep(0.5)
    miners = [procs.start([os.path.join(BIN, "miner"), f"127.0.0.1:{port}"], env=env(**drops))
              for _ in range(4)]
    miners += [start_native(procs, port, **drops) for _ in range(4)]
    time.sleep(4.0)  # let the miners open the GPU and join
    max_nonce = 1 << 36
    sampler = sysdiag.CgroupSampler()
    sampler.start()
    cpu0 = {m.pid: sysdiag.proc_cpu(m.pid) for m in miners}
    t0 = _t.time()
    clients = [procs.start([os.path.join(BIN, "client"), f"127.0.0.1:{port}", f"client-{i:02d}",
                            str(max_nonce)], env=env(**drops)) for i in range(16)]
    time.sleep(3.0)
    miners[1].send_signal(signal.SIGKILL)  # mid-job (2^34-nonce jobs take ~4 s per miner here)
    res = [c.communicate(timeout=400) for c in clients]
    wall = _t.time() - t0
    cpu1 = {m.pid: sysdiag.proc_cpu(m.pid) for m in miners}
    cgroup = sampler.stop()
    outs = [o.strip() for o, _ in res]
    server.send_signal(signal.SIGTERM)
    log = server.communicate(timeout=30)[1]
    for m in miners:
        if m.poll() is None:
            m.send_signal(signal.SIGTERM)
    merr = [m.communicate(timeout=30)[1] for m in miners]
    miner_cpu = [None if cpu0[m.pid] is None or cpu1[m.pid] is None else round(cpu1[m.pid] - cpu0[m.pid], 2)
                 for m in miners]
    texts = {"server": log, **{f"client-{i:02d}": e for i, (_, e) in enumerate(res)},
             **{f"miner-{k}": e for k, e in enumerate(merr)}}
    late = sysdiag.lsp_lateness(texts)
    failed = [i for i, o in enumerate(outs) if not o.startswith("Result")]
    diag = {"wall_s": round(wall, 2), "failed_clients": failed,
            "failed_client_stderr": {i: res[i][1][-1500:] for i in failed},
            "cgroup": cgroup,
            "miner_cpu_s": miner_cpu, "miner_cpu_per_wall": [None if c is None else round(c / wall, 3)
                                                               for c in miner_cpu],
            "max_late_ms": {k: v["max_late_ms"] for k, v in late.items()},
            "late_epochs": {k: v["late_epochs"] for k, v in late.items() if v["late_epochs"]},
            "server_losses": [ln for ln in log.splitlines() if " lost" in ln or "abandoned" in ln]}
    sysdiag.write_diag("config5_diag.json", diag)
    print("config 5 diagnostics:", diag)
    if failed:  # show the LSP's account of it
        raise AssertionError(f"clients {failed} did not get a Result; diagnostics {diag}; "
                             f"server log tail:\n{log[-4000:]}")
    checked_golden = 0
    for i, out in enumerate(outs):
        parts = out.split()
        assert parts[0] == "Result", (i, out)
        h, n = int(parts[1]), int(parts[2])
        msg = f"client-{i:02d}".encode()
        g = gold[f"cfg5_client-{i:02d}_2p36"]  # a CPU golden for every client
        assert (g["lower"], g["upper"]) == (0, max_nonce) and bytes.fromhex(g["msg_hex"]) == msg
        assert (h, n) == (g["hash"], g["nonce"]), i
        checked_golden += 1
        assert oracle.hash(msg, n) == h
    assert checked_golden == 16
    assert "lost; job [" in log and "requeued" in log, log[-2000:]
    print(f"config 5 full size: 16 x 2^36 nonces in {wall:.1f} s = {16 * (max_nonce + 1) / wall / 1e9:.1f} GH/s")
