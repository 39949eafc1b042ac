"""CPU: the compiled server program (bitcoin-miner_amd/csrc/server_main.cpp -- the
reference's server.go, spec'd in p1.pdf pp.13-15, in C++ over lsp_native.h) with
compiled miners (built against the oracle-backed ABI shim, tests/native_programs.py),
Python miners and Python clients over LSP/UDP: chunking and the lexicographic merge,
balancing, a killed miner's job requeued, the requeue cap, a lost client's work dropped,
request validation, two jobs per miner, drops on every role -- and the same runs under
ThreadSanitizer and ASan+UBSan builds of the server.  tests/test_gpu_system.py runs the
all-compiled system (this server, lib/gpuhash_miner on the GPU) end to end.
"""
import os
import signal
import subprocess
import sys
import threading
import time

import pytest

import bitcoin
import lsp
from bitcoin import client as bclient
from bitcoin import miner as bminer
from native_programs import Procs, build_miner, build_server

P = lsp.Params(EpochLimit=20, EpochMillis=40, WindowSize=1)
LSP_ENV = {"LSP_EPOCH_LIMIT": "20", "LSP_EPOCH_MILLIS": "40", "LSP_WINDOW_SIZE": "1"}


def free_port():
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def build_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("native_server")


@pytest.fixture(scope="module")
def miner_bin(build_dir):
    return build_miner(build_dir)


@pytest.fixture
def procs():
    pr = Procs()
    yield pr
    pr.stop_all()
    assert not pr.sanitizer_reports(), pr.sanitizer_reports()[0][-3000:]


class System:
    def __init__(self, procs, server_bin, miner_bin, **server_env):
        self.procs, self.miner_bin = procs, miner_bin
        self.port = free_port()
        self.server = procs.start([server_bin, str(self.port)], dict(LSP_ENV, GPUHASH_SERVER_LOG=1, **server_env))
        time.sleep(0.3)

    def miner(self, **env):
        return self.procs.start([self.miner_bin, f"127.0.0.1:{self.port}"], dict(LSP_ENV, **env))

    def request(self, msg, max_nonce):
        return bclient.request(f"127.0.0.1:{self.port}", msg, max_nonce, P)

    def log(self):
        self.server.terminate()
        self.server.wait(10)
        return self.server.stderr.read()


@pytest.fixture(params=[None, "thread", "address,undefined"], ids=["plain", "tsan", "asan_ubsan"])
def server_bin(request, build_dir):
    return build_server(build_dir, request.param)


@pytest.fixture
def plain_server(build_dir):
    return build_server(build_dir)


def test_usage(plain_server):
    r = subprocess.run([plain_server], capture_output=True, text=True, timeout=10)
    assert (r.returncode, r.stdout) == (0, "Usage: ./server <port>\n")


def test_config1_shape(procs, server_bin, miner_bin):
    s = System(procs, server_bin, miner_bin, GPUHASH_JOB_SIZE=2500)
    s.miner()
    assert s.request("bradfitz", 9999) == (1419516646206828, 9898)
    log = s.log()
    assert "[Request bradfitz 0 9999]" in log


def test_many_clients_compiled_and_python_miners_with_drops(procs, server_bin, miner_bin, oracle):
    """The compiled programs send each datagram in copies (LSP_SEND_COPIES' default, 3),
    the in-process Python miner and clients once (lsp.Params' default)."""
    _many_clients(procs, server_bin, miner_bin, oracle)


def test_many_clients_with_single_sends_from_the_compiled_programs(procs, plain_server, miner_bin, oracle):
    """The other way round: the compiled server and miners send every datagram once (the
    protocol as specified), the Python miner and clients three times."""
    _many_clients(procs, plain_server, miner_bin, oracle, lsp.Params(EpochLimit=20, EpochMillis=40, WindowSize=1,
                                                                     SendCopies=3), LSP_SEND_COPIES=1)


def _many_clients(procs, server_bin, miner_bin, oracle, params=P, **env):
    import lspnet
    drops = dict(LSPNET_SERVER_READ_DROP=10, LSPNET_SERVER_WRITE_DROP=10)
    s = System(procs, server_bin, miner_bin, GPUHASH_JOB_SIZE=3000, **drops, **env)
    for _ in range(2):
        s.miner(LSPNET_CLIENT_READ_DROP=10, LSPNET_CLIENT_WRITE_DROP=10, **env)

    class Eng:
        def min(self, msg, lo, hi):
            return oracle.min(msg.encode(), lo, hi)

    threading.Thread(target=bminer.run, args=(f"127.0.0.1:{s.port}", Eng(), params), daemon=True).start()
    lspnet.SetReadDropPercent(10)
    lspnet.SetWriteDropPercent(10)
    results = {}

    def cl(i):
        results[i] = bclient.request(f"127.0.0.1:{s.port}", f"client-{i:02d}", 20000 + 777 * i, params)

    th = [threading.Thread(target=cl, args=(i,)) for i in range(6)]
    try:
        for t in th:
            t.start()
        for t in th:
            t.join(120)
    finally:
        lspnet.ResetDropPercent()
    for i in range(6):
        assert results[i] == oracle.min(f"client-{i:02d}".encode(), 0, 20000 + 777 * i), i


def test_killed_miner_job_is_requeued(procs, plain_server, miner_bin, oracle):
    s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=10 ** 7)
    doomed = s.miner()
    time.sleep(0.3)
    res = {}
    t = threading.Thread(target=lambda: res.setdefault("r", s.request("killed-miner", 2 * 10 ** 7 - 1)))
    t.start()
    time.sleep(1.0)  # the doomed miner is inside its first ~2 s oracle job
    doomed.send_signal(signal.SIGKILL)
    doomed.wait(10)
    s.miner()
    t.join(120)
    assert res["r"] == oracle.min(b"killed-miner", 0, 2 * 10 ** 7 - 1, threads=8)
    log = s.log()
    assert "lost" in log and "requeued" in log, log


def test_requeue_cap_disconnects_the_client(procs, plain_server, miner_bin):
    s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=1000)
    doomed = [s.miner() for _ in range(4)]
    time.sleep(0.3)
    assert s.request("__gpuhash_test_ehip__", 999) is None  # every miner that takes it exits
    for p in doomed:
        assert p.wait(30) == 1
    s.miner()
    assert s.request("bradfitz", 9999) == (1419516646206828, 9898)  # and the server still serves
    assert "abandoned" in s.log()


def test_rejected_request_and_lost_client(procs, plain_server, miner_bin, oracle):
    s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=1000)
    s.miner()
    c = lsp.NewClient(f"127.0.0.1:{s.port}", P)
    c.Write(bitcoin.marshal(bitcoin.NewRequest("x", 10, 9)))
    with pytest.raises(lsp.LSPError):
        c.Read()  # the server closed the connection: no job is cut
    # a client that vanishes mid-request: its jobs stop being farmed out
    c2 = lsp.NewClient(f"127.0.0.1:{s.port}", P)
    c2.Write(bitcoin.marshal(bitcoin.NewRequest("gone", 0, 10 ** 7)))  # 10^4 jobs
    time.sleep(0.3)
    c2._loop.stop()
    time.sleep(P.EpochLimit * P.EpochMillis / 1000 + 0.5)
    assert s.request("bradfitz", 9999) == (1419516646206828, 9898)
    log = s.log()
    assert "request rejected (empty range" in log and "dropped request" in log, log


def test_two_jobs_per_miner(procs, plain_server, miner_bin, oracle):
    s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=500, GPUHASH_MINER_DEPTH=2)
    for _ in range(2):
        s.miner()
    results = {}
    th = [threading.Thread(target=lambda i=i: results.setdefault(i, s.request(f"d2-{i}", 7000 + 333 * i)))
          for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    for i in range(4):
        assert results[i] == oracle.min(f"d2-{i}".encode(), 0, 7000 + 333 * i), i


def test_requests_are_written_as_go_writes_them(procs, plain_server, miner_bin):
    """The compiled server's Request payloads are byte for byte what Go's json.Marshal
    writes (the same bytes bitcoin.marshal produces), escaped and non-ASCII Data too."""
    s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=10 ** 6)
    m = lsp.NewClient(f"127.0.0.1:{s.port}", P)  # a bare miner: Join, then read the Request
    m.Write(bitcoin.marshal(bitcoin.NewJoin()))
    time.sleep(0.2)
    c = lsp.NewClient(f"127.0.0.1:{s.port}", P)
    data = 'héllo <&> "q" \\ \n\t\x01 ✓ \u2028'
    c.Write(bitcoin.marshal(bitcoin.NewRequest(data, 5, 9)))
    raw = m.Read()
    assert raw == bitcoin.marshal(bitcoin.NewRequest(data, 5, 9)), raw
    m.Write(bitcoin.marshal(bitcoin.NewResult(1, 5)))
    r = bitcoin.unmarshal(c.Read())
    assert (r.Hash, r.Nonce) == (1, 5)
    c.Close()
    m.Close()


# ---- the compiled client (csrc/client_main.cpp) -------------------------------------------

@pytest.fixture(scope="module")
def client_bin(build_dir):
    from native_programs import build_client
    return build_client(build_dir)


def test_client_usage_and_max_nonce_parsing(client_bin):
    r = subprocess.run([client_bin], capture_output=True, text=True, timeout=10)
    assert r.stdout == "Usage: ./client <hostport> <message> <maxNonce>\n"
    for bad in ("-1", "+5", "18446744073709551616", "1e3", ""):
        r = subprocess.run([client_bin, "127.0.0.1:1", "m", bad], capture_output=True, text=True, timeout=10)
        assert r.stdout == f"{bad} is not a number.\n", bad


def test_client_prints_disconnected_without_server(client_bin):
    env = dict(os.environ, LSP_EPOCH_LIMIT="3", LSP_EPOCH_MILLIS="50")
    r = subprocess.run([client_bin, f"127.0.0.1:{free_port()}", "bradfitz", "9999"], capture_output=True,
                       text=True, timeout=20, env=env)
    assert r.stdout == "Disconnected\n"


@pytest.mark.parametrize("san", [None, "thread", "address,undefined"], ids=["plain", "tsan", "asan_ubsan"])
def test_config1_all_compiled(procs, build_dir, miner_bin, san):
    """Server, miner and client all compiled (the miner on the oracle-backed ABI shim
    here; tests/test_gpu_system.py runs it on the GPU): the client prints exactly the
    line p1.pdf p.15 grades."""
    from native_programs import build_client
    s = System(procs, build_server(build_dir, san), miner_bin, GPUHASH_JOB_SIZE=2000)
    s.miner()
    c = procs.start([build_client(build_dir, san), f"127.0.0.1:{s.port}", "bradfitz", "9999"], LSP_ENV)
    out, err = c.communicate(timeout=60)
    assert out == "Result 1419516646206828 9898\n", (out, err)


def test_a_small_request_is_not_starved_by_a_large_one(procs, plain_server, miner_bin, oracle):
    """p1.pdf p.15: the server balances miners across requests.  With one miner busy on a
    10^4-job request, a 5-job request that arrives later is answered within a few job
    round trips (the next job goes to the request with the fewest jobs in flight), long
    before the large one could finish."""
    s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=2000)
    s.miner()
    big = lsp.NewClient(f"127.0.0.1:{s.port}", P)
    big.Write(bitcoin.marshal(bitcoin.NewRequest("large", 0, 2 * 10 ** 7 - 1)))
    time.sleep(0.5)
    t0 = time.time()
    assert s.request("bradfitz", 9999) == (1419516646206828, 9898)
    assert time.time() - t0 < 5.0
    big._loop.stop()  # leave without waiting: the server drops the large request
    time.sleep(P.EpochLimit * P.EpochMillis / 1000 + 0.5)
    assert "dropped request" in s.log()


def _longest_servable_data(upper):
    """Largest ASCII Data whose worst-case job frame (both bounds at `upper`) still fits
    one LSP datagram."""
    import lspnet
    from bitcoin.server import job_frame_worst_case
    n = 1000
    while len(job_frame_worst_case("d" * (n + 1), upper)) <= lspnet.MAX_DATAGRAM:
        n += 1
    return n


def test_jobs_must_fit_one_datagram_python_and_compiled(procs, plain_server, miner_bin, oracle):
    """a request that fits a datagram can yield jobs that do not (20-digit
    job bounds where the client sent Lower = 0); such a job would be truncated and
    resent forever.  Both servers refuse the request at the same length, and serve the
    longest one whose jobs fit, end to end."""
    import lspnet
    from bitcoin.server import request_error
    n = _longest_servable_data(99)
    # jobs are priced at the request's Upper, not at 2^64-1 -- a 2-digit Upper
    # leaves room for 36 more bytes of Data than a 20-digit one
    assert n == _longest_servable_data(bitcoin.UINT64_MAX) + 36
    assert request_error("d" * n, 0, 99) is None and "datagram" in request_error("d" * n, 0, bitcoin.UINT64_MAX)
    client_frame = lsp.message.NewData(1, 1, bitcoin.marshal(bitcoin.NewRequest("d" * (n + 1), 0, 99))).marshal()
    assert len(client_frame) <= lspnet.MAX_DATAGRAM  # the client's own Request fits
    assert request_error("d" * n, 0, 99) is None
    assert "datagram" in request_error("d" * (n + 1), 0, 99)
    s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=40)
    s.miner()
    assert s.request("d" * (n + 1), 99) is None  # Disconnected
    assert s.request("d" * n, 99) == oracle.min(b"d" * n, 0, 99)
    log = s.log()
    assert "would not fit a 2000-byte LSP datagram" in log, log


def test_overdue_copy_under_sanitizers(procs, server_bin, miner_bin, oracle):
    """The compiled server's copy path (Job shared between miners' queues, the timed
    read_until wake-up) under the plain, TSan and ASan + UBSan builds."""
    _overdue_case(procs, server_bin, miner_bin, oracle, "compiled")


@pytest.mark.parametrize("which", ["python", "compiled"])
def test_overdue_job_is_copied_to_an_idle_miner(procs, plain_server, miner_bin, oracle, which):
    _overdue_case(procs, plain_server, miner_bin, oracle, which)


def _overdue_case(procs, plain_server, miner_bin, oracle, which):
    """Speculative copies (bitcoin/server.py Scheduler, csrc/server_main.cpp Scheduler): a
    miner that answered once and then sits on its next job forever -- its LSP connection
    alive, so the server never sees it lost -- does not hold that request up.  Once the
    job is overdue by the miner's learned rate, an idle miner gets a copy and its Result
    answers the client."""
    import queue
    if which == "compiled":
        s = System(procs, plain_server, miner_bin, GPUHASH_JOB_SIZE=10 ** 6)
        port, log = s.port, s.log
    else:
        lines = queue.Queue()
        holder = {}
        threading.Thread(target=bserver_serve, args=(P, 10 ** 6, holder, lines.put), daemon=True).start()
        while "srv" not in holder:
            time.sleep(0.01)
        port = holder["srv"].port

        def log():
            out = []
            while not lines.empty():
                out.append(lines.get())
            return "\n".join(out)

    class Stuck:  # answers its first job, then never returns
        calls = 0

        def min(self, msg, lo, hi):
            Stuck.calls += 1
            if Stuck.calls > 1:
                threading.Event().wait()
            return oracle.min(msg.encode(), lo, hi)

    threading.Thread(target=bminer.run, args=(f"127.0.0.1:{port}", Stuck(), P), daemon=True).start()
    time.sleep(0.3)
    hp = f"127.0.0.1:{port}"
    assert bclient.request(hp, "first", 999, P) == oracle.min(b"first", 0, 999)  # the stuck miner learns a rate
    if which == "compiled":
        s.miner()
    else:
        class Eng:
            def min(self, msg, lo, hi):
                return oracle.min(msg.encode(), lo, hi)
        threading.Thread(target=bminer.run, args=(hp, Eng(), P), daemon=True).start()
    time.sleep(0.3)
    t = time.time()
    assert bclient.request(hp, "second", 999, P) == oracle.min(b"second", 0, 999)
    assert time.time() - t < 5.0
    assert Stuck.calls == 2  # the stuck miner took the job; a copy answered it
    assert "copy of job [0, 999]" in log()


def bserver_serve(params, job_size, holder, log):
    from bitcoin import server as bserver
    bserver.serve(0, params=params, job_size=job_size, ready=lambda srv: holder.setdefault("srv", srv), log=log)


@pytest.mark.parametrize("lsp_env", [{}, {"LSP_SEND_COPIES": "1"}, {"LSP_EPOCH_MILLIS": "200"},
                                     {"LSP_EPOCH_MILLIS": "40", "LSP_EPOCH_LIMIT": "20", "LSP_SEND_COPIES": "2"},
                                     {"GPUHASH_JOB_SIZE": "12345", "GPUHASH_MINER_DEPTH": "2", "GPUHASH_BACKUP": "0"}],
                         ids=["reference_params", "single_sends", "200ms", "40ms_two_copies", "overrides"])
def test_compiled_and_python_servers_choose_the_same_defaults(procs, plain_server, lsp_env):
    """Both servers log their configuration at start; for the same environment the lines
    are identical: job size (server.py default_job_size / server_main.cpp's mirror, from
    the epoch and the send copies), depth, speculative copies and the LSP parameters."""
    server_py = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "bitcoin-miner_amd", "bin", "server")
    base = {k: v for k, v in os.environ.items() if not k.startswith(("LSP_", "GPUHASH_"))}
    lines = []
    for argv in ([plain_server], [sys.executable, server_py]):
        env = dict(base, GPUHASH_SERVER_LOG="1", **lsp_env)
        p = subprocess.Popen(argv + [str(free_port())], env=env, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, text=True)
        procs.ps.append(p)
        line = ""
        deadline = time.monotonic() + 30
        while time.monotonic() < deadline and "config:" not in line:
            line = p.stderr.readline()
        p.terminate()
        p.wait(10)
        assert "config:" in line, (argv, line)
        lines.append(line.strip())
    assert lines[0] == lines[1], lines
    if not lsp_env:
        assert "jobs of 17179869184 nonces, depth 3, 3 live copies" in lines[0] and "send copies 3" in lines[0]
    if lsp_env == {"LSP_SEND_COPIES": "1"}:
        assert "jobs of 68719476736 nonces" in lines[0]
