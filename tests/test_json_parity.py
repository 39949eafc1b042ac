"""CPU: the two Go-compatible JSON readers -- bitcoin.unmarshal (Python server/miner) and
csrc/lsp_native.h btc_unmarshal (compiled server/miner) -- decode every document of a
corpus the way Go's json.Unmarshal into bitcoin.Message (message.go:16-21) does, and so
agree with each other byte for byte (invalid UTF-8 one U+FFFD per byte,
malformed nested values rejected, duplicate keys with null / wrong-type members).  The
same for the LSP frame readers, lsp.Message.unmarshal and lsp_native.h lsp_unmarshal, on
lsp.Message (lsp/message.go:17-22): []byte Payload null resets it to nil, int fields take
integer literals only."""
import os
import subprocess

import pytest

import bitcoin

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
U64 = (1 << 64) - 1
F = "�".encode()

# (document, expected) -- expected None: Go's Unmarshal returns an error (message dropped);
# else (Type, Data bytes, Lower, Upper)
CASES = [
    (b'{"Type":1,"Data":"x","Lower":1,"Upper":2}', (1, b"x", 1, 2)),
    # invalid UTF-8 inside the string: one U+FFFD per invalid byte (utf8.DecodeRune size 1)
    (b'{"Type":1,"Data":"\xe2\x82A","Upper":2}', (1, F + F + b"A", 0, 2)),
    (b'{"Type":1,"Data":"\xf0\x9f\x98","Upper":2}', (1, F * 3, 0, 2)),
    (b'{"Type":1,"Data":"\xf0\x9f\x98\x80","Upper":2}', (1, b"\xf0\x9f\x98\x80", 0, 2)),
    (b'{"Type":1,"Data":"\xed\xa0\x80","Upper":2}', (1, F * 3, 0, 2)),   # encoded surrogate
    (b'{"Type":1,"Data":"\xc0\x80z","Upper":2}', (1, F * 2 + b"z", 0, 2)),  # overlong NUL
    (b'{"Type":1,"Data":"\xff\xfe","Upper":2}', (1, F * 2, 0, 2)),
    (b'{"Type":1,"Data":"\x80\xbf","Upper":2}', (1, F * 2, 0, 2)),  # stray continuations
    (b'{"Type":1,"Data":"\xf4\x90\x80\x80","Upper":2}', (1, F * 4, 0, 2)),  # > U+10FFFF
    # malformed nested values in an unknown field: the whole document is a syntax error
    (b'{"Type":1,"X":[1 2],"Upper":2}', None),
    (b'{"Type":1,"X":{1:2},"Upper":2}', None),
    (b'{"Type":1,"X":{"a"},"Upper":2}', None),
    (b'{"Type":1,"X":[,,],"Upper":2}', None),
    (b'{"Type":1,"X":[1,],"Upper":2}', None),
    (b'{"Type":1,"X":{"a":1,},"Upper":2}', None),
    (b'{"Type":1,"X":[1]],"Upper":2}', None),
    (b'{"Type":1,"X":{"a":[1,{"b":"}]"}],"c":null},"Upper":2}', (1, b"", 0, 2)),
    (b'{"Type":1,"X":[],"Y":{},"Upper":2}', (1, b"", 0, 2)),
    # numbers: RFC 8259 grammar (Go's scanner), uint64 fields ParseUint
    (b'{"Type":1,"X":1-2,"Upper":2}', None),
    (b'{"Type":1,"X":01,"Upper":2}', None),
    (b'{"Type":1,"X":-,"Upper":2}', None),
    (b'{"Type":1,"X":1.,"Upper":2}', None),
    (b'{"Type":1,"X":1e,"Upper":2}', None),
    (b'{"Type":1,"X":-0.5e+7,"Upper":2}', (1, b"", 0, 2)),
    (b'{"Type":1,"X":NaN,"Upper":2}', None),
    (b'{"Type":1,"X":-Infinity,"Upper":2}', None),
    (b'{"Type":1,"Upper":1e3}', None),
    (b'{"Type":1,"Upper":-0}', None),
    (b'{"Type":1,"Upper":18446744073709551615}', (1, b"", 0, U64)),
    (b'{"Type":1,"Upper":18446744073709551616}', None),
    (b'{"Type":-0,"Upper":3}', (0, b"", 0, 3)),
    # duplicate keys (any ASCII case): every member decodes in order; null leaves the
    # field as it was; one member of the wrong type fails the message
    (b'{"Type":1,"Lower":5,"lower":null,"Upper":9}', (1, b"", 5, 9)),
    (b'{"Type":1,"Lower":"x","Lower":1,"Upper":9}', None),
    (b'{"Type":1,"Lower":1,"LOWER":true,"Upper":9}', None),
    (b'{"Type":1,"Data":"a","data":null,"Upper":9}', (1, b"a", 0, 9)),
    (b'{"Type":1,"Data":"a","DATA":"b","Upper":9}', (1, b"b", 0, 9)),
    (b'{"Type":1,"Data":5,"data":"b","Upper":9}', None),
    (b'{"Type":null,"type":1,"Upper":9,"upper":null}', (1, b"", 0, 9)),
    (b'{"Type":1,"Upper":9,"upper":7}', (1, b"", 0, 7)),
]


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("json") / "json_probe")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I",
                           os.path.join(ROOT, "bitcoin-miner_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "json_probe.cpp"), "-lpthread", "-o", exe])
    return exe


def _native(exe, docs):
    out = subprocess.run([exe], input="\n".join(d.hex() for d in docs) + "\n", capture_output=True,
                         text=True, timeout=30, check=True).stdout.splitlines()
    res = []
    for ln in out:
        if ln == "ERR":
            res.append(None)
        else:
            _, t, lo, up, _h, _n, *data = ln.split(" ")
            res.append((int(t), bytes.fromhex(data[0] if data else ""), int(lo), int(up)))
    return res


def _python(doc):
    try:
        m = bitcoin.unmarshal(doc)
    except (ValueError, TypeError):
        return None
    return (int(m.Type), m.Data.encode(), m.Lower, m.Upper)


def test_unicode_key_folding_reaches_bitcoin_fields(probe):
    """'Haſh' (U+017F) sets Hash in Go; the Kelvin sign folds to 'k' (no field has one)."""
    doc = '{"Type":2,"Haſh":77,"Nonce":5}'.encode()
    assert (bitcoin.unmarshal(doc).Hash, bitcoin.unmarshal(doc).Nonce) == (77, 5)
    out = subprocess.run([probe], input=doc.hex() + "\n", capture_output=True, text=True, timeout=30,
                         check=True).stdout.split()
    assert (int(out[4]), int(out[5])) == (77, 5)
    import gojson
    assert "\u212aind".translate(gojson._FOLD) == "kind" and "\u017f".translate(gojson._FOLD) == "s"


def test_python_reader_decodes_like_go():
    for doc, want in CASES:
        assert _python(doc) == want, doc


def test_native_reader_decodes_like_go(probe):
    got = _native(probe, [d for d, _ in CASES])
    for (doc, want), g in zip(CASES, got):
        assert g == want, doc


def test_readers_agree_on_random_byte_strings(probe):
    """Random Data payloads of raw bytes (any UTF-8 validity) inside a Request: the two
    readers produce the same Data bytes, hence hash the same message."""
    import random
    rng = random.Random(7)
    docs = []
    for _ in range(400):
        n = rng.randrange(0, 24)
        raw = bytes(rng.choice([rng.randrange(0x80, 0x100), rng.randrange(0x20, 0x7F)]) for _ in range(n))
        raw = raw.replace(b'"', b"'").replace(b"\\", b"/")
        docs.append(b'{"Type":1,"Data":"' + raw + b'","Lower":0,"Upper":7}')
    assert _native(probe, docs) == [_python(d) for d in docs]


# (frame, expected) for lsp.Message -- None: Go's Unmarshal errors; else
# (Type, ConnID, SeqNum, Payload bytes or None for nil)
LSP_CASES = [
    (b'{"Type":1,"ConnID":3,"SeqNum":4,"Payload":"aGk="}', (1, 3, 4, b"hi")),
    (b'{"Type":2,"ConnID":3,"SeqNum":4,"Payload":null}', (2, 3, 4, None)),
    (b'{"Type":1,"ConnID":3,"SeqNum":4}', (1, 3, 4, None)),
    # []byte: a later null resets the slice to nil (ADVICE r04 on lsp_native.h)
    (b'{"Type":1,"ConnID":3,"SeqNum":4,"Payload":"aGk=","payload":null}', (1, 3, 4, None)),
    (b'{"Type":1,"ConnID":3,"SeqNum":4,"payload":null,"PAYLOAD":"aGk="}', (1, 3, 4, b"hi")),
    (b'{"Type":1,"Payload":"aGk=","payload":"eW8="}', (1, 0, 0, b"yo")),
    # base64: StdEncoding, padded; CR/LF ignored; other junk fails the frame
    (b'{"Type":1,"Payload":"aG\\r\\nk="}', (1, 0, 0, b"hi")),
    (b'{"Type":1,"Payload":"aGk"}', None),
    (b'{"Type":1,"Payload":"a$Gk="}', None),
    (b'{"Type":1,"Payload":5}', None),
    (b'{"Type":1,"Payload":"!!!!","payload":"aGk="}', None),
    # ints: integer literals only; a wrong-typed member fails even before a good one
    (b'{"Type":1.0,"ConnID":1}', None),
    (b'{"Type":"1","ConnID":1}', None),
    (b'{"Type":true}', None),
    (b'{"Type":1,"ConnID":1e2}', None),
    (b'{"ConnID":"x","connid":2,"Type":2}', None),
    (b'{"Type":null,"type":2,"ConnID":7,"connid":null}', (2, 7, 0, None)),
    (b'{"Type":2,"SeqNum":9223372036854775807}', (2, 0, 9223372036854775807, None)),
    (b'{"Type":2,"SeqNum":9223372036854775808}', None),
    (b'{"Type":2,"SeqNum":-3}', (2, 0, -3, None)),
    # absent Type is MsgConnect (0); unknown types decode (the endpoints ignore them)
    (b'{"ConnID":0,"SeqNum":0}', (0, 0, 0, None)),
    (b'{"Type":7,"ConnID":1}', (7, 1, 0, None)),
    (b'{"tYpE":2,"cOnNiD":5,"seqnum":6,"X":[1,{"y":null}]}', (2, 5, 6, None)),
    (b'[1,2]', None),
    (b'{"Type":1,"X":NaN}', None),
    # []byte from an array: encoding/json decodes a JSON array into any slice,
    # each element a uint8 (ParseUint, <= 255), null leaving its element 0
    (b'{"Type":1,"Payload":[104,105]}', (1, 0, 0, b"hi")),
    (b'{"Type":1,"Payload":[]}', (1, 0, 0, b"")),
    (b'{"Type":1,"Payload":[104,null,105]}', (1, 0, 0, b"h\x00i")),
    (b'{"Type":1,"Payload":[0,255]}', (1, 0, 0, b"\x00\xff")),
    (b'{"Type":1,"Payload":[256]}', None),
    (b'{"Type":1,"Payload":[-1]}', None),
    (b'{"Type":1,"Payload":[1.0]}', None),
    (b'{"Type":1,"Payload":[1e1]}', None),
    (b'{"Type":1,"Payload":["a"]}', None),
    (b'{"Type":1,"Payload":[[1]]}', None),
    (b'{"Type":1,"Payload":[true]}', None),
    (b'{"Type":1,"Payload":{"a":1}}', None),
    (b'{"Type":1,"Payload":[104],"payload":"eW8="}', (1, 0, 0, b"yo")),
    (b'{"Type":1,"Payload":"eW8=","payload":[104]}', (1, 0, 0, b"h")),
    (b'{"Type":1,"Payload":[104],"payload":null}', (1, 0, 0, None)),
    # key folding beyond ASCII: the long s U+017F matches 's' (ADVICE r05); other
    # non-ASCII letters match nothing
    (b'{"Type":2,"\xc5\xbfeqNum":6}', (2, 0, 6, None)),
    (b'{"Type":2,"SEQNUM":5,"\xc5\xbfeqnum":6}', (2, 0, 6, None)),
    (b'{"Type":2,"\xc5\xbfeqNum":"x"}', None),
    (b'{"Type":2,"\xc4\xb1d":1,"Conn\xc4\xb0D":3}', (2, 0, 0, None)),
]


def _lsp_python(doc):
    from lsp.message import Message
    try:
        m = Message.unmarshal(doc)
    except (ValueError, TypeError):
        return None
    return (int(m.Type), m.ConnID, m.SeqNum, m.Payload)


def _lsp_native(exe, docs):
    out = subprocess.run([exe, "lsp"], input="\n".join(d.hex() for d in docs) + "\n", capture_output=True,
                         text=True, timeout=30, check=True).stdout.splitlines()
    res = []
    for ln in out:
        if ln == "ERR":
            res.append(None)
        else:
            _, t, c, q, p = ln.split(" ")
            res.append((int(t), int(c), int(q), None if p == "-" else bytes.fromhex(p)))
    return res


def test_python_lsp_reader_decodes_like_go():
    for doc, want in LSP_CASES:
        assert _lsp_python(doc) == want, doc


def test_native_lsp_reader_decodes_like_go(probe):
    got = _lsp_native(probe, [d for d, _ in LSP_CASES])
    for (doc, want), g in zip(LSP_CASES, got):
        assert g == want, doc


def test_lsp_readers_round_trip_and_agree_on_random_frames(probe):
    """Frames the writers produce read back exactly, and random mutations of them (case
    changes, duplicated keys, nulls, junk base64) decode the same in both readers."""
    import random
    from lsp.message import Message, MsgType
    rng = random.Random(11)
    docs = []
    for _ in range(300):
        m = Message(rng.choice(list(MsgType)), rng.randrange(0, 1 << 31), rng.randrange(0, 1 << 31),
                    None if rng.random() < 0.3 else bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))))
        raw = m.marshal()
        assert Message.unmarshal(raw) == m
        s = raw.decode()
        k = rng.randrange(5)
        if k == 0:
            s = s.replace('"Payload"', '"payload"')
        elif k == 1:
            s = s[:-1] + ',"PAYLOAD":null}'
        elif k == 2:
            s = s[:-1] + ',"payload":"' + rng.choice(["aGk=", "aG", "a=Gk", "@@@@", ""]) + '"}'
        elif k == 3:
            s = s[:-1] + ',"seqnum":' + rng.choice(["1", "-1", "1.5", '"1"', "null"]) + "}"
        docs.append(s.encode())
    assert _lsp_native(probe, docs) == [_lsp_python(d) for d in docs]
