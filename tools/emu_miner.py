#!/usr/bin/env python3
"""A miner whose engine only takes the time a GPU would: the real bitcoin/miner.py loop
and LSP client, with gpuhash_min replaced by a sleep of (Upper - Lower + 1) / rate.  It
lets the scheduler and the LSP be measured on the CPU at node scale (8 "GPUs" at the
measured 34.6 GH/s each) with real sockets, drops and epochs, to check the discrete-event
model in tests/lsp_des.py against them.  Test/measurement infrastructure only: its
results are not hashes.

    python tools/emu_miner.py host:port rate_nonces_per_s
"""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))


class EmuEngine:
    def __init__(self, rate: float, overhead_s: float = 0.001):
        self.rate = rate
        self.overhead_s = overhead_s
        self._ms = 0.0

    def min(self, msg, lower: int, upper: int):
        dt = (upper - lower + 1) / self.rate
        time.sleep(dt + self.overhead_s)
        self._ms = 1000.0 * dt
        # a fixed function of the range: merging is exercised elsewhere, timing here
        return (lower * 2654435761) % (1 << 64), lower

    def stats(self) -> dict:
        return {"kernel_ms": self._ms}


def main() -> int:
    from bitcoin import miner
    return miner.run(sys.argv[1], engine=EmuEngine(float(sys.argv[2])))


if __name__ == "__main__":
    sys.exit(main())
