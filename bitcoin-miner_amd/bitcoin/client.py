"""Request client -- bitcoin/client/client.go of the reference (stub at :15), written to
p1.pdf p.14: send [Request message 0 maxNonce], print "Result minHash nonce", or
"Disconnected" if the server is lost (printResult / printDisconnected, client.go:19-26).

    python bitcoin-miner_amd/bin/client host:port message maxNonce
"""
from __future__ import annotations

import sys

import lsp

from . import UINT64_MAX, NewRequest, MsgType, ParseUint, marshal, params_from_env, unmarshal


def printResult(hash_: str, nonce: str) -> None:  # client.go:19-21
    print("Result", hash_, nonce, flush=True)


def printDisconnected() -> None:  # client.go:24-26
    print("Disconnected", flush=True)


def request(hostport: str, message: str, max_nonce: int, params=None):
    """Returns (hash, nonce), or None when the connection to the server is lost."""
    if isinstance(max_nonce, bool) or not isinstance(max_nonce, int) or not 0 <= max_nonce <= UINT64_MAX:
        raise ValueError(f"maxNonce {max_nonce!r} outside [0, 2^64-1]")
    try:
        c = lsp.NewClient(hostport, params or params_from_env())
    except lsp.LSPError as e:
        print(f"client: {e}", file=sys.stderr, flush=True)  # stderr: stdout is graded
        return None
    try:
        c.Write(marshal(NewRequest(message, 0, max_nonce)))
        while True:
            try:
                m = unmarshal(c.Read())
            except (ValueError, KeyError):
                continue  # not a Message: ignored, as json.Unmarshal's error would be
            if m.Type == MsgType.Result:
                return m.Hash, m.Nonce
    except lsp.LSPError as e:
        print(f"client: {e}", file=sys.stderr, flush=True)
        return None
    finally:
        c.Close()


def main(argv=None) -> int:
    argv = sys.argv if argv is None else argv
    if len(argv) != 4:  # client.go:9-13
        print("Usage: ./client <hostport> <message> <maxNonce>")
        return 0
    try:
        max_nonce = ParseUint(argv[3])  # a uint64, as strconv.ParseUint would have it
    except ValueError:
        print(f"{argv[3]} is not a number.")
        return 0
    res = request(argv[1], argv[2], max_nonce)
    if res is None:
        printDisconnected()
    else:
        printResult(str(res[0]), str(res[1]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
