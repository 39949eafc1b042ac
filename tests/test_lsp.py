"""CPU: the LSP transport (bitcoin-miner_amd/lsp) that carries Request/Result messages.

Modelled on the reference's own LSP suite (src/github.com/cmu440/lsp/lsp{1,2,3,4}_test.go):
an echo server with several clients (lsp1 TestBasic*), write drops (TestRobust*), window
sizes with scattered/in-order delivery (lsp2 TestWindow*), explicit closes and lost
connections (lsp3/lsp4).  Epochs are shortened so the suite runs in seconds.
"""
import random
import threading
import time

import pytest

import lsp
import lspnet

FAST = dict(EpochLimit=5, EpochMillis=50)


@pytest.fixture(autouse=True)
def no_drops():
    lspnet.SetReadDropPercent(0)
    lspnet.SetWriteDropPercent(0)
    yield
    lspnet.SetReadDropPercent(0)
    lspnet.SetWriteDropPercent(0)


def echo_server(params):
    srv = lsp.NewServer(0, params)
    stop = threading.Event()

    def loop():
        while not stop.is_set():
            try:
                cid, payload = srv.Read()
            except lsp.LSPError as e:
                if e.conn_id == 0:
                    return
                continue
            try:
                srv.Write(cid, payload)
            except lsp.LSPError:
                pass

    t = threading.Thread(target=loop, daemon=True)
    t.start()
    return srv, stop, t


def run_echo(nclients, nmsgs, params, drop=0, client_params=None):
    srv, stop, t = echo_server(params)
    clients = [lsp.NewClient(f"127.0.0.1:{srv.port}", client_params or params) for _ in range(nclients)]
    assert len({c.ConnID() for c in clients}) == nclients
    lspnet.SetWriteDropPercent(drop)
    errors = []

    def client_loop(c, seed):
        rng = random.Random(seed)
        msgs = [str(rng.randrange(10 ** 9)).encode() for _ in range(nmsgs)]
        for m in msgs:
            c.Write(m)
        got = [c.Read() for _ in msgs]
        if got != msgs:
            errors.append((c.ConnID(), got[:3], msgs[:3]))

    ts = [threading.Thread(target=client_loop, args=(c, i)) for i, c in enumerate(clients)]
    for x in ts:
        x.start()
    for x in ts:
        x.join(60)
    lspnet.SetWriteDropPercent(0)
    for c in clients:
        c.Close()
    stop.set()
    try:
        srv.Close()
    except lsp.LSPError:
        # a closed client may never ack the server's last retransmission when its ack
        # was dropped; Close then reports the lost client (server_api.go:33-38)
        pass
    assert not errors, errors


@pytest.mark.parametrize("nclients,nmsgs", [(1, 1), (1, 50), (3, 30), (10, 20)])
def test_basic_echo(nclients, nmsgs):
    run_echo(nclients, nmsgs, lsp.Params(WindowSize=1, **FAST))


@pytest.mark.parametrize("window", [1, 2, 5, 10])
def test_window_sizes(window):
    run_echo(3, 40, lsp.Params(WindowSize=window, **FAST))


@pytest.mark.parametrize("drop", [10, 20])
def test_robust_with_write_drops(drop):
    run_echo(4, 25, lsp.Params(EpochLimit=20, EpochMillis=20, WindowSize=4), drop=drop)


@pytest.mark.parametrize("copies,window", [(2, 1), (3, 1), (3, 4)])
def test_send_copies_deliver_once_in_order(copies, window):
    """SendCopies (lsp/endpoint.py): every originated datagram goes out `copies` times; the
    receiver must still deliver each message exactly once, in order, under drops."""
    p = lsp.Params(EpochLimit=20, EpochMillis=20, WindowSize=window, SendCopies=copies)
    run_echo(4, 25, p, drop=20)


@pytest.mark.parametrize("server_copies,client_copies", [(1, 3), (3, 1)])
def test_send_copies_interoperate_with_single_sends(server_copies, client_copies):
    """A peer that sends copies talks to one that sends each datagram once (the protocol
    as specified, e.g. the reference's own endpoints): the copies are duplicates it
    already handles."""
    p = dict(EpochLimit=20, EpochMillis=20, WindowSize=1)
    run_echo(3, 20, lsp.Params(SendCopies=server_copies, **p), drop=15,
             client_params=lsp.Params(SendCopies=client_copies, **p))


def test_send_copies_count():
    """What goes out: a Data message `copies` times; its ack `copies` times the first time
    it arrives and once per later duplicate; each epoch's resends, re-acks and heartbeats
    `copies` times."""
    from lsp.endpoint import ConnState
    sent = []
    a = ConnState(1, 1, 5, sent.append, copies=3)
    a.write(b"x")
    assert [(m.Type, m.SeqNum) for m in sent] == [(lsp.MsgType.MsgData, 1)] * 3
    sent.clear()
    b_sent = []
    b = ConnState(1, 1, 5, b_sent.append, copies=3)
    assert b.on_message(lsp.NewData(1, 1, b"x")) == [b"x"]
    assert b.on_message(lsp.NewData(1, 1, b"x")) == []  # a copy: acked again, not delivered
    assert [(m.Type, m.SeqNum) for m in b_sent] == [(lsp.MsgType.MsgAck, 1)] * 4
    b_sent.clear()
    b.on_epoch()  # re-ack the last received message, three times
    assert [(m.Type, m.SeqNum) for m in b_sent] == [(lsp.MsgType.MsgAck, 1)] * 3
    a.on_epoch()  # unacked: resent three times; no data received yet: heartbeat too
    assert [(m.Type, m.SeqNum) for m in sent].count((lsp.MsgType.MsgData, 1)) == 3
    assert [(m.Type, m.SeqNum) for m in sent].count((lsp.MsgType.MsgAck, 0)) == 3
    assert lsp.Params().SendCopies == 1  # the library's default: the protocol as specified


def test_in_order_delivery_under_reordering_window():
    # a window of 8 lets up to 8 messages be in flight; the receiver must still deliver
    # in sequence-number order (lsp2 "scattered" mode)
    params = lsp.Params(EpochLimit=20, EpochMillis=20, WindowSize=8)
    run_echo(2, 100, params, drop=15)


def test_json_wire_format_matches_go():
    m = lsp.NewData(3, 7, b"hello")
    assert m.marshal() == b'{"Type":1,"ConnID":3,"SeqNum":7,"Payload":"aGVsbG8="}'
    assert lsp.Message.unmarshal(m.marshal()) == m
    assert lsp.NewAck(3, 0).marshal() == b'{"Type":2,"ConnID":3,"SeqNum":0,"Payload":null}'
    assert str(m) == "[Data 3 7 hello]"
    assert str(lsp.NewParams()) == "[EpochLimit: 5, EpochMillis: 2000, WindowSize: 1]"


def test_connect_fails_without_server():
    t = time.time()
    with pytest.raises(lsp.LSPError):
        lsp.NewClient("127.0.0.1:9", lsp.Params(EpochLimit=3, EpochMillis=30))
    assert time.time() - t < 5


def test_client_detects_lost_server():
    params = lsp.Params(**FAST)
    srv = lsp.NewServer(0, params)
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", params)
    srv.Close()  # no clients pending -> returns; the client now hears nothing
    t = time.time()
    with pytest.raises(lsp.LSPError):
        c.Read()
    assert time.time() - t < 2
    with pytest.raises(lsp.LSPError):
        c.Write(b"x")
    c.Close()


def test_server_detects_lost_client_and_reports_conn_id():
    params = lsp.Params(**FAST)
    srv = lsp.NewServer(0, params)
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", params)
    c.Write(b"hi")
    assert srv.Read() == (c.ConnID(), b"hi")
    c._loop.stop()  # kill the client without a Close: it goes silent
    with pytest.raises(lsp.LSPError) as e:
        srv.Read()
    assert e.value.conn_id == c.ConnID()
    with pytest.raises(lsp.LSPError):
        srv.Write(c.ConnID(), b"late")
    srv.Close()


def test_close_conn_flushes_pending_then_reports():
    params = lsp.Params(WindowSize=2, **FAST)
    srv = lsp.NewServer(0, params)
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", params)
    c.Write(b"hello")
    cid, _ = srv.Read()
    for i in range(5):
        srv.Write(cid, b"m%d" % i)
    srv.CloseConn(cid)
    assert [c.Read() for _ in range(5)] == [b"m%d" % i for i in range(5)]
    with pytest.raises(lsp.LSPError) as e:
        srv.Read()
    assert e.value.conn_id == cid
    c.Close()
    srv.Close()


def test_client_close_waits_for_acks():
    params = lsp.Params(EpochLimit=20, EpochMillis=20, WindowSize=1)
    srv = lsp.NewServer(0, params)
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", params)
    lspnet.SetClientWriteDropPercent(30)
    for i in range(20):
        c.Write(b"%d" % i)
    c.Close()  # returns only when all 20 are acknowledged
    lspnet.SetClientWriteDropPercent(0)
    got = [srv.Read()[1] for _ in range(20)]
    assert got == [b"%d" % i for i in range(20)]
    srv.Close()


def test_duplicate_connect_same_address_keeps_one_connection():
    params = lsp.Params(**FAST)
    srv = lsp.NewServer(0, params)
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", params)
    for _ in range(3):
        c._conn.write_to(lsp.NewConnect().marshal())
    time.sleep(0.1)
    assert len(srv._conns) == 1
    c.Close()
    srv.Close()


def test_client_hears_only_its_server():
    """The reference's lspnet.DialUDP is a connected UDP socket, so a client reads only its
    server's datagrams; a frame from any other address (here a Data frame carrying the
    client's own conn ID and the next sequence number) is ignored, as csrc/lsp_native.h
    does."""
    import socket
    from lsp.message import NewData
    params = lsp.Params(**FAST)
    srv = lsp.NewServer(0, params)
    c = lsp.NewClient(f"127.0.0.1:{srv.port}", params)
    rogue = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rogue.bind(("127.0.0.1", 0))
    for _ in range(3):
        rogue.sendto(NewData(c.ConnID(), 1, b"forged").marshal(), ("127.0.0.1", c._conn.local_addr()[1]))
    time.sleep(0.2)
    srv.Write(c.ConnID(), b"real")
    assert c.Read() == b"real"
    rogue.close()
    c.Close()
    try:
        srv.Close()
    except lsp.LSPError:
        pass


def test_copy_filter():
    """lsp.endpoint.CopyFilter: the same bytes from the same address within min(10 ms,
    epoch / 20) are a copy, answered with the reply its first instance got; a resend an
    epoch later, or the same bytes from another address, are handled in full."""
    from lsp.endpoint import CopyFilter
    f = CopyFilter(2.0)
    a, b = ("127.0.0.1", 1), ("127.0.0.1", 2)
    assert f.copy_of(a, b"d1", 100.0) is None
    f.reply(a, b"d1", b"ack1")
    assert f.copy_of(a, b"d1", 100.001) == b"ack1"
    assert f.copy_of(b, b"d1", 100.001) is None          # another peer
    assert f.copy_of(a, b"d1", 102.0) is None            # an epoch resend
    assert f.copy_of(a, b"h0", 102.0) is None and f.copy_of(a, b"h0", 102.0) == b""  # no reply
    f.forget(a)
    assert f.copy_of(a, b"h0", 102.0) is None
    assert CopyFilter(0.04).window == pytest.approx(0.002)
