"""gpuhash.dist -- one process per GPU over torch.distributed, gloo by default (a host-side
TCP merge of 24-byte results; no RCCL on the data path -- bench.py's GPUHASH_DIST_BACKEND=nccl
moves only the barrier and merge onto RCCL).

The nonce search partitions perfectly: nonces are independent and the reduction is one
associative argmin over the lexicographic (hash, nonce) key.  So ranks
search contiguous shards with NO data-path collective; the only communication is the
final 16-byte result per rank, gathered once (the host-argmin step of the north_star,
done across processes instead of across threads).

  split_range   strong scaling: [lower, upper] cut into `world` contiguous shards; given
                the message length, by the ENGINE's cost model (gpuhash_shard_range, the
                same cut points gpuhash_min uses over devices), else by count
  weak_range    weak scaling: rank r searches [base + r*per_rank, base + (r+1)*per_rank)
  merge_min     lexicographic (hash, nonce) argmin -- lowest nonce on equal hashes
  distributed_min   shard -> local search -> all_gather(16 B) -> merge
"""
from __future__ import annotations

from typing import Callable, Iterable

U64_MAX = (1 << 64) - 1


def split_range(lower: int, upper: int, world: int, msg_len: int | None = None,
                policy: int | None = None) -> list[tuple[int, int] | None]:
    """Contiguous shards of the inclusive range, in rank order; None for an empty shard.

    With msg_len, the shards are of equal estimated COST (for message
    lengths 45-54 the digit groups differ in SHA blocks per nonce, so equal counts would
    leave the 2-block ranks last): the cut points come from the C ABI,
    gpuhash_shard_range, so in-process devices and processes shard identically.  Without
    it, equal counts (a search function that is not the engine, e.g. the oracle).  `policy`:
    the layout policy the ranks' engines run (gpuhash_shard_range_policy; default AUTO),
    since the cost of a digit group depends on its layout."""
    if lower > upper:
        raise ValueError("lower > upper")
    if msg_len is not None:
        from gpuhash import shard_range
        return shard_range(msg_len, lower, upper, world, policy)
    count = upper - lower + 1
    out: list[tuple[int, int] | None] = []
    start = lower
    for r in range(world):
        n = count // world + (1 if r < count % world else 0)
        out.append((start, start + n - 1) if n else None)
        start += n
    return out


def weak_range(base: int, per_rank: int, rank: int) -> tuple[int, int]:
    lo = base + rank * per_rank
    hi = lo + per_rank - 1
    if hi > U64_MAX:
        raise ValueError("weak-scaling range past 2^64-1")
    return lo, hi


def merge_min(results: Iterable[tuple[int, int] | None]) -> tuple[int, int]:
    best = None
    for r in results:
        if r is None:
            continue
        if best is None or r < best:  # tuple order == (hash, nonce) lexicographic
            best = r
    if best is None:
        raise ValueError("no results to merge")
    return best


def _pack(res: tuple[int, int] | None):
    import numpy as np
    import torch
    if res is None:
        arr = np.array([U64_MAX, U64_MAX, 0], dtype=np.uint64)
    else:
        arr = np.array([res[0], res[1], 1], dtype=np.uint64)
    return torch.from_numpy(arr.view(np.int64).copy())


def gather_results(res: tuple[int, int] | None, device=None) -> list[tuple[int, int] | None]:
    """all_gather of each rank's (hash, nonce) -- 24 bytes per rank, one collective into
    one tensor and one copy back to the host."""
    import numpy as np
    import torch
    import torch.distributed as dist
    t = _pack(res)
    if device is not None:
        t = t.to(device)
    world = dist.get_world_size()
    out = torch.empty(3 * world, dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t)
    a = out.cpu().numpy().view(np.uint64).reshape(world, 3)
    return [(int(h), int(n)) if int(v) else None for h, n, v in a]


def distributed_min(search: Callable[[int, int], tuple[int, int]], lower: int, upper: int,
                    device=None, msg_len: int | None = None) -> tuple[int, int]:
    """Every rank searches its shard of [lower, upper] with `search(lo, hi)`; returns the
    global argmin on every rank.  msg_len selects the engine's cost-balanced split."""
    import torch.distributed as dist
    shard = split_range(lower, upper, dist.get_world_size(), msg_len)[dist.get_rank()]
    local = search(*shard) if shard is not None else None
    return merge_min(gather_results(local, device))
