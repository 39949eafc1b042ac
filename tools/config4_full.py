#!/usr/bin/env python3
"""Config 4 at full size on one MI355X: argmin over [0, 2^40) of "bradfitz", three ways.

The CPU oracle cannot scan 2^40 nonces (about 60 h on 16 cores), so parity at this size
rests on size-independent properties:

  1. one gpuhash_min call over the whole range on one device;
  2. the same range as 8 contiguous cost-balanced shards (the in-process multi-device
     path, here 8 shards on the same GPU) with the 16-byte host argmin;
  3. the 8 per-rank windows of bench.py --config 4 (rank r: [r*2^37, (r+1)*2^37)),
     searched one call each and merged with gpuhash.dist.merge_min.

All three must return the same (hash, nonce), the returned hash must equal the oracle's
bitcoin.Hash of the returned nonce, and every nonce of a window around the winner must
hash no lower (oracle scan, lowest nonce on ties).  Prints one JSON line per step.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gpuhash  # noqa: E402
from gpuhash.dist import merge_min  # noqa: E402
import hash_oracle  # noqa: E402

MSG = b"bradfitz"
LO, HI = 0, (1 << 40) - 1


def emit(**kv):
    print(json.dumps(kv), flush=True)


def main() -> None:
    oracle = hash_oracle.load_c_oracle()
    out = {}
    with gpuhash.Engine([0]) as eng:
        t = time.perf_counter()
        out["one_call"] = eng.min(MSG, LO, HI)
        dt = time.perf_counter() - t
        emit(step="one_call", result=list(out["one_call"]), s=round(dt, 3),
             GHs=round((HI - LO + 1) / dt / 1e9, 3))

        parts = []
        t = time.perf_counter()
        for r in range(8):
            parts.append(eng.min(MSG, r << 37, ((r + 1) << 37) - 1))
            emit(step="rank_window", rank=r, result=list(parts[-1]))
        out["rank_windows"] = merge_min(parts)
        dt = time.perf_counter() - t
        emit(step="rank_windows", result=list(out["rank_windows"]), s=round(dt, 3))

    with gpuhash.Engine([0] * 8) as eng8:
        t = time.perf_counter()
        out["shards8"] = eng8.min(MSG, LO, HI)
        dt = time.perf_counter() - t
        emit(step="shards8", result=list(out["shards8"]), s=round(dt, 3))

    h, n = out["one_call"]
    agree = len({tuple(v) for v in out.values()}) == 1
    hash_ok = oracle.hash(MSG, n) == h
    # oracle scan of a window around the winner: nothing in it beats (h, n)
    wlo, whi = max(LO, n - (1 << 25)), min(HI, n + (1 << 25))
    wmin = oracle.min(MSG, wlo, whi, threads=min(16, os.cpu_count() or 1))
    window_ok = tuple(wmin) == (h, n)
    emit(step="verdict", result=[h, n], all_three_agree=agree, oracle_hash_of_nonce_ok=hash_ok,
         oracle_window=[wlo, whi], oracle_window_min=list(wmin), window_ok=window_ok)
    sys.exit(0 if agree and hash_ok and window_ok else 1)


if __name__ == "__main__":
    main()
