"""CPU: argument validation along the Request path (client -> server -> miner -> engine).

Go's client would parse maxNonce with strconv.ParseUint and Go's json.Unmarshal refuses a
uint64 field outside [0, 2^64-1]; the server must not cut jobs from a request it cannot
serve, a miner must not exit (and get its job requeued to the next miner) on an error
that every miner would hit, and the ctypes mirror must not let ctypes wrap a bound
silently (2**64+5 -> 5).  The miners here use stand-in engines; no GPU is needed.
"""
import json
import threading
import time

import pytest

import bitcoin
import gpuhash
import lsp
from bitcoin import client as bclient
from bitcoin import miner as bminer
from bitcoin import server as bserver

U64 = (1 << 64) - 1
P = lsp.Params(EpochLimit=10, EpochMillis=40, WindowSize=1)


# ---- client: maxNonce as strconv.ParseUint(s, 10, 64) ------------------------------------

@pytest.mark.parametrize("s,v", [("0", 0), ("9999", 9999), ("007", 7), (str(U64), U64)])
def test_parse_uint_accepts_decimal_u64(s, v):
    assert bitcoin.ParseUint(s) == v


@pytest.mark.parametrize("s", ["", "-1", "+5", " 5", "5 ", "1_000", "0x10", "1e3", "1.0",
                               str(U64 + 1), "١٢٣"])
def test_parse_uint_rejects_what_go_rejects(s):
    with pytest.raises(ValueError):
        bitcoin.ParseUint(s)


@pytest.mark.parametrize("arg", ["-1", str(U64 + 1), "+5"])
def test_client_cli_refuses_bad_max_nonce(arg, capsys):
    assert bclient.main(["client", "127.0.0.1:1", "msg", arg]) == 0
    assert capsys.readouterr().out == f"{arg} is not a number.\n"


@pytest.mark.parametrize("v", [-1, U64 + 1, 1.5, True])
def test_client_request_refuses_out_of_range(v):
    with pytest.raises(ValueError):
        bclient.request("127.0.0.1:1", "msg", v)


# ---- wire format: json.Unmarshal into bitcoin.Message -------------------------------------

def test_unmarshal_round_trips_extremes():
    m = bitcoin.NewRequest("x", 0, U64)
    assert bitcoin.unmarshal(bitcoin.marshal(m)) == m
    r = bitcoin.NewResult(U64, U64)
    assert bitcoin.unmarshal(bitcoin.marshal(r)) == r


@pytest.mark.parametrize("field,value", [("Lower", -1), ("Upper", U64 + 1), ("Upper", 1.0),
                                         ("Hash", 1e30), ("Nonce", True), ("Lower", "5"),
                                         ("Type", "1"), ("Data", 5)])
def test_unmarshal_rejects_what_go_rejects(field, value):
    d = {"Type": 1, "Data": "x", "Lower": 0, "Upper": 9, "Hash": 0, "Nonce": 0}
    d[field] = value
    with pytest.raises(ValueError):
        bitcoin.unmarshal(json.dumps(d).encode())


def test_unmarshal_null_fields_are_zero_values():
    m = bitcoin.unmarshal(b'{"Type":1,"Data":null,"Lower":null,"Upper":3}')
    assert (m.Data, m.Lower, m.Upper) == ("", 0, 3)


# ---- server: request validation and the requeue cap ---------------------------------------

@pytest.mark.parametrize("lo,hi", [(5, 4), (-1, 3), (0, U64 + 1), (0, 1.5)])
def test_scheduler_rejects_unservable_ranges(lo, hi):
    s = bserver.Scheduler(job_size=10)
    with pytest.raises(ValueError):
        s.add_request(client=100, data="a", lower=lo, upper=hi)
    assert s.requests == {}
    s.add_miner(1)
    assert s.next_assignment() is None  # nothing was cut


def test_scheduler_rejects_data_over_engine_cap_and_datagram():
    s = bserver.Scheduler(job_size=10)
    with pytest.raises(ValueError, match="engine"):
        s.add_request(client=100, data="a" * (gpuhash.GPUHASH_MAX_MSG + 1), lower=0, upper=9)
    # the LSP datagram (2000 bytes, lspnet/conn.go:35) is the tighter cap: the job frames
    # must fit it (tests/test_native_server.py finds the exact boundary for both servers)
    with pytest.raises(ValueError, match="datagram"):
        s.add_request(client=100, data="a" * 1400, lower=0, upper=9)
    s.add_request(client=100, data="a" * 1300, lower=0, upper=9)


def test_scheduler_accepts_full_u64_and_single_nonce():
    s = bserver.Scheduler(job_size=10)
    s.add_request(client=100, data="a", lower=0, upper=U64)
    s.add_request(client=101, data="b", lower=U64, upper=U64)


def test_requeue_cap_abandons_a_job_that_kills_every_miner():
    s = bserver.Scheduler(job_size=10, max_requeues=3)
    rid = s.add_request(client=100, data="a", lower=0, upper=9)
    s.add_request(client=200, data="b", lower=0, upper=29)
    miner = 1
    s.add_miner(miner)
    m, job, _ = s.next_assignment()
    first = (job.lower, job.upper)
    for k in range(3):  # three losses: requeued each time, first in line
        assert "requeued" in s.lost(m)
        miner += 1
        s.add_miner(miner)
        m, job, _ = s.next_assignment()
        if job.req_id != rid:  # the other request may take the new miner first
            miner += 1
            s.add_miner(miner)
            m, job, _ = s.next_assignment()
        assert (job.lower, job.upper) == first and job.requeues == k + 1
    note = s.lost(m)  # the fourth loss abandons the request
    assert "abandoned" in note and rid not in s.requests
    assert list(s.abandoned) == [100]
    # the other client's request is untouched
    assert any(r.client == 200 for r in s.requests.values())


def _start_server():
    box, ready = {}, threading.Event()

    def on_ready(srv):
        box["srv"] = srv
        ready.set()

    threading.Thread(target=bserver.serve, args=(0,), kwargs=dict(params=P, job_size=100, ready=on_ready),
                     daemon=True).start()
    ready.wait(5)
    return box["srv"]


def test_server_closes_a_client_with_an_empty_range(oracle):
    srv = _start_server()
    calls = []

    class Eng:
        def min(self, msg, lo, hi):
            calls.append((lo, hi))
            return oracle.min(msg.encode(), lo, hi)

    threading.Thread(target=bminer.run, args=(f"127.0.0.1:{srv.port}", Eng(), P), daemon=True).start()
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", P)
    c.Write(bitcoin.marshal(bitcoin.NewRequest("x", 10, 9)))
    t = time.time()
    with pytest.raises(lsp.LSPError):
        c.Read()  # no Result ever comes: the connection is closed on the client
    assert time.time() - t < 10
    assert calls == []  # no job was cut
    # the server still serves a valid request
    assert bclient.request(f"127.0.0.1:{srv.port}", "bradfitz", 9999, P) == (1419516646206828, 9898)
    try:
        srv.Close()
    except lsp.LSPError:
        pass


# ---- miner: empty ranges, argument errors, device errors ----------------------------------

class _Server:
    """A bare LSP server standing in for the bitcoin server: hands out given jobs."""

    def __init__(self):
        self.srv = lsp.NewServer(0, P)

    def join(self):
        conn, payload = self.srv.Read()
        assert bitcoin.unmarshal(payload).Type == bitcoin.MsgType.Join
        return conn

    def result(self):
        conn, payload = self.srv.Read()
        return bitcoin.unmarshal(payload)


def _argument_error():
    e = gpuhash.GpuHashError.__new__(gpuhash.GpuHashError)
    e.rc = gpuhash.GPUHASH_ETOOLONG
    RuntimeError.__init__(e, "gpuhash_min: message longer than GPUHASH_MAX_MSG (rc=-4)")
    return e


def _device_error():
    e = gpuhash.GpuHashError.__new__(gpuhash.GpuHashError)
    e.rc = gpuhash.GPUHASH_EHIP
    RuntimeError.__init__(e, "gpuhash_min: HIP runtime error (rc=-3)")
    return e


def test_miner_answers_empty_range_and_exits_on_argument_errors(oracle):
    """every Request gets exactly one Result or a lost connection.
    The stub server here does NOT validate, so the argument error reaches the engine; the
    miner must not skip the job (it would stay in flight, and with two jobs per miner the
    next Result would answer the wrong request) but exit, so the job is requeued."""
    s = _Server()

    class Eng:
        def min(self, msg, lo, hi):
            if msg == "bad":
                raise _argument_error()
            return oracle.min(msg.encode(), lo, hi)

    rc = {}
    th = threading.Thread(target=lambda: rc.setdefault("rc", bminer.run(f"127.0.0.1:{s.srv.port}", Eng(), P)),
                          daemon=True)
    th.start()
    conn = s.join()
    s.srv.Write(conn, bitcoin.marshal(bitcoin.NewRequest("msg", 5, 4)))
    r = s.result()
    assert (r.Type, r.Hash, r.Nonce) == (bitcoin.MsgType.Result, U64, U64)
    s.srv.Write(conn, bitcoin.marshal(bitcoin.NewRequest("msg", 0, 2)))
    r = s.result()
    assert (r.Hash, r.Nonce) == (4754799531757243342, 1)  # p1.pdf p.12
    s.srv.Write(conn, bitcoin.marshal(bitcoin.NewRequest("bad", 0, 9)))  # -> exit, no Result
    s.srv.Write(conn, bitcoin.marshal(bitcoin.NewRequest("msg", 0, 2)))  # queued, never served
    th.join(10)
    assert not th.is_alive() and rc.get("rc") == 1
    # the server side sees the connection lost, never a Result for the failed job
    with pytest.raises(lsp.LSPError):
        s.result()
    try:
        s.srv.Close()
    except lsp.LSPError:
        pass


def test_argument_error_on_every_miner_hits_the_requeue_cap(oracle):
    """The real server with its request validation bypassed (so a job the engine refuses
    reaches the miners): each miner exits on it, the job is requeued, and after
    MAX_REQUEUES the client sees Disconnected instead of hanging; the server goes on."""
    from bitcoin import client as bclient
    from bitcoin import server as bserver
    box, ready, lines = {}, threading.Event(), []
    orig = bserver.request_error
    bserver.request_error = lambda *a, **k: None  # a server that does not validate
    try:
        def on_ready(srv):
            box["srv"] = srv
            ready.set()
        threading.Thread(target=bserver.serve, args=(0,),
                         kwargs=dict(params=P, job_size=1000, ready=on_ready, log=lines.append),
                         daemon=True).start()
        ready.wait(5)
        port = box["srv"].port

        class Eng:
            def min(self, msg, lo, hi):
                if msg == "bad":
                    raise _argument_error()
                return oracle.min(msg.encode(), lo, hi)

        rcs = []
        ths = [threading.Thread(target=lambda: rcs.append(bminer.run(f"127.0.0.1:{port}", Eng(), P)), daemon=True)
               for _ in range(bserver.MAX_REQUEUES + 1)]
        for t in ths:
            t.start()
        time.sleep(0.3)
        assert bclient.request(f"127.0.0.1:{port}", "bad", 99, P) is None  # Disconnected
        for t in ths:
            t.join(30)
        assert rcs == [1] * (bserver.MAX_REQUEUES + 1)
        assert any("abandoned" in ln for ln in lines), lines
        # the server still serves a good request with a healthy miner
        threading.Thread(target=lambda: bminer.run(f"127.0.0.1:{port}", Eng(), P), daemon=True).start()
        assert bclient.request(f"127.0.0.1:{port}", "bradfitz", 9999, P) == (1419516646206828, 9898)
    finally:
        bserver.request_error = orig
        try:
            box["srv"].Close()
        except (lsp.LSPError, KeyError):
            pass


def test_miner_exits_on_device_error():
    s = _Server()

    class Eng:
        def min(self, msg, lo, hi):
            raise _device_error()

    err = {}

    def run():
        try:
            bminer.run(f"127.0.0.1:{s.srv.port}", Eng(), P)
        except gpuhash.GpuHashError as e:
            err["e"] = e

    th = threading.Thread(target=run, daemon=True)
    th.start()
    conn = s.join()
    s.srv.Write(conn, bitcoin.marshal(bitcoin.NewRequest("msg", 0, 9)))
    th.join(10)
    assert not th.is_alive() and err["e"].rc == gpuhash.GPUHASH_EHIP
    try:
        s.srv.Close()
    except lsp.LSPError:
        pass


# ---- engine mirror: bounds never reach ctypes out of range --------------------------------

class _NoCallLib:
    def __getattr__(self, name):
        raise AssertionError(f"{name} reached the C ABI")


def _engine_without_device():
    eng = gpuhash.Engine.__new__(gpuhash.Engine)
    eng._lib = _NoCallLib()
    eng._ctx = None
    return eng


@pytest.mark.parametrize("lo,hi", [(-1, 5), (0, U64 + 1), (U64 + 5, U64 + 6), (0, 2.0), (True, 3)])
def test_engine_min_refuses_bounds_outside_u64(lo, hi):
    eng = _engine_without_device()
    with pytest.raises((ValueError, TypeError)):
        eng.min("msg", lo, hi)


def test_engine_hash_range_and_hash_refuse_bad_bounds():
    eng = _engine_without_device()
    with pytest.raises(ValueError):
        eng.hash_range("msg", -1, 4)
    with pytest.raises(ValueError):
        eng.hash_range("msg", 0, U64 + 1)
    with pytest.raises(ValueError):
        gpuhash.Hash("msg", U64 + 1)


def test_argument_error_classification():
    assert _argument_error().is_argument_error
    assert not _device_error().is_argument_error


# ---- wire format: json.Marshal(bitcoin.Message) byte for byte ----------------------------

@pytest.mark.parametrize("msg,raw", [
    (bitcoin.NewJoin(), b'{"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}'),
    (bitcoin.NewResult(U64, 7), b'{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":18446744073709551615,"Nonce":7}'),
    # Go: HTML-safe escapes for < > &, raw UTF-8, \n \r \t short forms, other controls \u00XX
    (bitcoin.NewRequest('a<b>&"c"\\é\n\r\t\x01\x08\x0c\x7f ', 0, 9),
     b'{"Type":1,"Data":"a\\u003cb\\u003e\\u0026\\"c\\"\\\\\xc3\xa9\\n\\r\\t\\u0001\\u0008\\u000c\x7f\\u2028",'
     b'"Lower":0,"Upper":9,"Hash":0,"Nonce":0}'),
])
def test_marshal_is_byte_exact_with_go(msg, raw):
    assert bitcoin.marshal(msg) == raw
    assert bitcoin.unmarshal(raw) == msg


def test_marshal_replaces_invalid_utf8_like_go():
    assert bitcoin.marshal(bitcoin.NewRequest("x\ud800y", 1, 2)).startswith(b'{"Type":1,"Data":"x\xef\xbf\xbdy"')


def test_unmarshal_replaces_lone_surrogates_and_bad_utf8_like_go():
    """Go's json.Unmarshal decodes a lone surrogate escape and invalid UTF-8
    to U+FFFD (so the message is served, and hashed as EF BF BD), as lsp_native.h does;
    the Python side used to keep the lone surrogate and then fail the request."""
    m = bitcoin.unmarshal(b'{"Type":1,"Data":"a\\ud800b\\udc00c","Lower":0,"Upper":5}')
    assert m.Data == "a�b�c"
    assert bitcoin.unmarshal(b'{"Type":1,"Data":"\\ud83d\\ude00","Lower":0,"Upper":5}').Data == "\U0001F600"
    assert bitcoin.unmarshal(b'{"Type":1,"Data":"x\xff\xfey","Lower":0,"Upper":5}').Data == "x��y"
    assert bserver.request_error(m.Data, 0, 5) is None
    assert m.Data.encode() == b"a\xef\xbf\xbdb\xef\xbf\xbdc"


def test_unmarshal_field_matching_like_go():
    """encoding/json matches keys to fields ignoring case (the last
    matching key wins) and skips unknown fields of any shape; both the Python reader and
    csrc/lsp_native.h now do (tests/test_native_miner.py drives the compiled one)."""
    m = bitcoin.unmarshal(b'{"type":1,"DATA":"x","lower":3,"Upper":9,"extra":{"a":[1,{"b":"}"}]},"z":[]}')
    assert (m.Type, m.Data, m.Lower, m.Upper) == (bitcoin.MsgType.Request, "x", 3, 9)
    m = bitcoin.unmarshal(b'{"Type":1,"Upper":5,"upper":7}')
    assert m.Upper == 7
    with pytest.raises((ValueError, TypeError)):
        bitcoin.unmarshal(b'{"Type":1,"Lower":{"x":1}}')  # a known field of the wrong shape
    import lsp.message as lm
    x = lm.Message.unmarshal(b'{"type":1,"connid":4,"SEQNUM":2,"payload":"eA==","n":{"q":[1]}}')
    assert (x.Type, x.ConnID, x.SeqNum, x.Payload) == (lm.MsgType.MsgData, 4, 2, b"x")
