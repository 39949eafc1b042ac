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
import re
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
LSP_GAVE_UP = re.compile(r"no connect ack in \d+ epochs|\d+ silent epochs")


def killed_miners_work_rerun(log: str) -> bool:
    """The server log shows a killed miner's unfinished job going out again: requeued when
    its loss was noticed, still held by a speculative copy then, or copied before it
    (bitcoin/server.py and csrc/server_main.cpp log lines)."""
    return bool(re.search(r"job \[\d+, \d+\] of request \d+ (requeued|still held)", log)
                or ("copy of job [" in log and " lost" in log))


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
    assert killed_miners_work_rerun(log), log[-2000:]


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
    log = server.communicate(timeout=30)[1]
    assert killed_miners_work_rerun(log), log[-2000:]


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
    assert killed_miners_work_rerun(log), log[-2000:]


def run_config5_full_size(procs, engine, oracle, golden, envf, kill_after, diag_name):
    """BASELINE configs[4] at full size on the one GPU; `envf` builds each program's
    environment (its LSP parameters).  Returns (outputs, client stderr, server log, diag)."""
    import time as _t
    import sysdiag
    port = free_port()
    drops = dict(LSPNET_CLIENT_READ_DROP=10, LSPNET_CLIENT_WRITE_DROP=10,
                 LSPNET_SERVER_READ_DROP=10, LSPNET_SERVER_WRITE_DROP=10, LSP_DIAG=1)
    server = procs.start([os.path.join(BIN, "server"), str(port)], env=envf(GPUHASH_SERVER_LOG=1, **drops))
    time.sleep(0.5)
    miners = [procs.start([os.path.join(BIN, "miner"), f"127.0.0.1:{port}"], env=envf(**drops))
              for _ in range(4)]
    miners += [subprocess.Popen([NATIVE_MINER, f"127.0.0.1:{port}"], stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE, text=True, env=envf(**drops)) for _ in range(4)]
    procs.ps.extend(miners[4:])
    time.sleep(4.0)  # let the miners open the GPU and join
    max_nonce = 1 << 36
    sampler = sysdiag.CgroupSampler()
    sampler.start()
    cpu0 = {m.pid: sysdiag.proc_cpu(m.pid) for m in miners}
    t0 = _t.time()
    clients = [procs.start([os.path.join(BIN, "client"), f"127.0.0.1:{port}", f"client-{i:02d}",
                            str(max_nonce)], env=envf(**drops)) for i in range(16)]
    time.sleep(kill_after)
    miners[1].send_signal(signal.SIGKILL)  # mid-job
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
    diag = {"wall_s": round(wall, 2), "GHs": round(16 * (max_nonce + 1) / wall / 1e9, 2),
            "failed_clients": failed,
            "failed_client_stderr": {i: res[i][1][-1500:] for i in failed},
            "cgroup": cgroup,
            "miner_cpu_s": miner_cpu, "miner_cpu_per_wall": [None if c is None else round(c / wall, 3)
                                                               for c in miner_cpu],
            "max_late_ms": {k: v["max_late_ms"] for k, v in late.items()},
            "late_epochs": {k: v["late_epochs"] for k, v in late.items() if v["late_epochs"]},
            "server_losses": [ln for ln in log.splitlines() if " lost" in ln or "abandoned" in ln],
            "copies": sum(1 for ln in log.splitlines() if "copy of job" in ln),
            # each miner's exit status and its own account (its connection ID, why it ended)
            "miners": [{"index": k, "returncode": m.returncode,
                        "stderr": [ln for ln in e.splitlines() if "joined as" in ln or " lost" in ln
                                   or "exiting" in ln or "rror" in ln][-6:]} for k, (m, e) in enumerate(zip(miners, merr))]}
    sysdiag.write_diag(diag_name, diag)
    print("config 5 diagnostics:", diag)
    return outs, [e for _, e in res], log, diag


def check_config5(outs, golden, oracle, skip=()):
    gold = {r["name"]: r for r in golden["ranges"]}
    max_nonce = 1 << 36
    checked = 0
    for i, out in enumerate(outs):
        if i in skip:
            continue
        parts = out.split()
        assert parts[0] == "Result", (i, out)
        h, n = int(parts[1]), int(parts[2])
        msg = f"client-{i:02d}".encode()
        g = gold[f"cfg5_client-{i:02d}_2p36"]  # a CPU golden for every client
        assert (g["lower"], g["upper"]) == (0, max_nonce) and bytes.fromhex(g["msg_hex"]) == msg
        assert (h, n) == (g["hash"], g["nonce"]), i
        assert oracle.hash(msg, n) == h
        checked += 1
    return checked


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
    outs, errs, log, diag = run_config5_full_size(procs, engine, oracle, golden, env, 3.0, "config5_diag.json")
    if diag["failed_clients"]:  # show the LSP's account of it
        raise AssertionError(f"clients {diag['failed_clients']} did not get a Result; diagnostics {diag}; "
                             f"server log tail:\n{log[-4000:]}")
    assert check_config5(outs, golden, oracle) == 16
    assert killed_miners_work_rerun(log), log[-2000:]
    print(f"config 5 full size: {diag['GHs']} GH/s")


def env_reference(**extra):
    """No LSP overrides: the reference's lsp/params.go (2 s epochs, EpochLimit 5, window 1)."""
    e = {k: v for k, v in os.environ.items() if not k.startswith("LSP_")}
    e.update({k: str(v) for k, v in extra.items()})
    return e


@pytest.mark.timeout(900)
@pytest.mark.parametrize("send_copies", [None, 1], ids=["send_copies_default", "single_sends"])
def test_config5_full_size_reference_lsp_params(procs, engine, oracle, golden, send_copies):
    """config 5 at full size at the untouched protocol's parameters
    (lsp/params.go:9-11: 2000 ms epochs, EpochLimit 5, window 1), 10% drops on every role,
    a miner SIGKILLed 4 s in (LSP notices it 10 s later; the server copies its overdue
    jobs before then).  Every Result must equal its golden.

    Twice: with the programs' default of sending each datagram three times
    (bitcoin.SEND_COPIES), where every client must get its Result; and with every
    datagram sent once (LSP_SEND_COPIES=1, the protocol exactly as specified), where LSP
    itself gives up on a connection now and then: a client whose Connect or its Ack is
    lost five times running (each gets through with 0.9^2, so (1 - 0.81^2)^5 = 0.5% per
    client, 7.5% that one of 16 does) or that hears nothing for 5 whole epochs prints
    "Disconnected", as the reference's client would (tests/test_scheduler_sim.py measures
    both rates through the protocol model).  One such client is accepted there only with
    LSP's own reason on its stderr; the server must abandon nothing."""
    extra = {} if send_copies is None else {"LSP_SEND_COPIES": send_copies}
    name = "config5_reference_params_diag.json" if send_copies is None else "config5_reference_params_single_diag.json"
    outs, errs, log, diag = run_config5_full_size(procs, engine, oracle, golden,
                                                  lambda **kw: env_reference(**extra, **kw), 4.0, name)
    gave_up = [i for i in diag["failed_clients"] if outs[i] == "Disconnected" and LSP_GAVE_UP.search(errs[i])]
    assert len(gave_up) <= (1 if send_copies == 1 else 0) and set(gave_up) == set(diag["failed_clients"]), diag
    assert "abandoned" not in log, log[-3000:]
    assert check_config5(outs, golden, oracle, skip=set(gave_up)) == 16 - len(gave_up)
    print(f"config 5 full size at the reference's LSP params ({send_copies or 'default'} send copies): "
          f"{diag['GHs']} GH/s, {diag['copies']} speculative copies")
