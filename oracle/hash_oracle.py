"""oracle/hash_oracle.py -- hashlib restatement of the reference hot path + C-oracle loader.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / the timed CPU
baseline.  Nothing in bitcoin-miner_amd/ imports it.

Two independent CPU restatements live in oracle/:
  * this file: Python + hashlib (OpenSSL's SHA-256), a line-for-line restatement of
    bitcoin.Hash, src/github.com/cmu440/bitcoin/hash.go:11-15:
        hasher.Write([]byte(fmt.Sprintf("%s %d", msg, nonce)))   # hash.go:13
        return binary.BigEndian.Uint64(hasher.Sum(nil))           # hash.go:14
    and of the spec'd miner loop (p1.pdf pp.12-14; stub at bitcoin/miner/miner.go:15):
    ascending scan of the inclusive [Lower, Upper], strict '<' (lowest nonce wins ties).
  * hash_oracle.c: a from-FIPS-180-4 C restatement of the same, fast enough for the
    2^32-nonce golden and for the CPU baseline.  `load_c_oracle()` builds/loads it.
  * golden_scan.c: a third restatement on the x86 SHA extensions and AVX-512, only to
    compute the goldens of searches of 2^36-2^40 nonces (`GoldenScan`).

Both are pinned to the handout's known-answer values (p1.pdf p.12), see
tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

# p1.pdf p.12 known-answer values (the only reference-provided pins).
SPEC_KATS = [
    (b"msg", 0, 13781283048668101583),
    (b"msg", 1, 4754799531757243342),
    (b"msg", 2, 5611725180048225792),
]


def hash_py(msg: bytes, nonce: int) -> int:
    """bitcoin.Hash(msg, nonce) -- hash.go:11-15."""
    data = msg + b" " + str(int(nonce)).encode()
    return int.from_bytes(hashlib.sha256(data).digest()[:8], "big")


def min_py(msg: bytes, lower: int, upper: int) -> tuple[int, int]:
    """Spec'd miner loop: argmin over inclusive [lower, upper], lowest nonce on ties."""
    if lower > upper:
        raise ValueError("lower > upper")
    best_h, best_n = hash_py(msg, lower), lower
    for n in range(lower + 1, upper + 1):
        h = hash_py(msg, n)
        if h < best_h:
            best_h, best_n = h, n
    return best_h, best_n


def build_c_oracle(force: bool = False) -> str:
    """Compile hash_oracle.c (and the bench's cpu_baseline.c) with gcc (no GPU, no ROCm
    needed)."""
    src = os.path.join(HERE, "hash_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-pthread", "-o", LIB_PATH, src])
    build_cpu_baseline(force)
    build_golden_scan(force)
    return LIB_PATH


BASELINE_PATH = os.path.join(HERE, "build", "libcpubaseline.so")


def build_cpu_baseline(force: bool = False) -> str:
    """oracle/cpu_baseline.c: the reference loop with OpenSSL's SHA-256 (bench only)."""
    src = os.path.join(HERE, "cpu_baseline.c")
    if force or not os.path.exists(BASELINE_PATH) or os.path.getmtime(BASELINE_PATH) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(BASELINE_PATH), exist_ok=True)
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-pthread", "-o", BASELINE_PATH, src, "-ldl"])
    return BASELINE_PATH


class CpuBaseline:
    """ctypes view of oracle/build/libcpubaseline.so (bench.py's cpu_baseline leg)."""

    def __init__(self):
        if not os.path.exists(BASELINE_PATH):
            build_cpu_baseline()
        self.lib = ctypes.CDLL(BASELINE_PATH)
        u64, sz, p = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_char_p
        self.lib.baseline_available.restype = ctypes.c_int
        self.lib.baseline_hash.restype = u64
        self.lib.baseline_hash.argtypes = [p, sz, u64]
        self.lib.baseline_min.restype = ctypes.c_int
        self.lib.baseline_min.argtypes = [p, sz, u64, u64, ctypes.c_int, ctypes.POINTER(u64), ctypes.POINTER(u64)]

    def available(self) -> bool:
        return bool(self.lib.baseline_available())

    def hash(self, msg: bytes, nonce: int) -> int:
        return int(self.lib.baseline_hash(msg, len(msg), nonce))

    def min(self, msg: bytes, lower: int, upper: int, threads: int = 1) -> tuple[int, int]:
        h, n = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self.lib.baseline_min(msg, len(msg), lower, upper, threads, ctypes.byref(h), ctypes.byref(n))
        if rc != 0:
            raise ValueError(f"baseline_min rc={rc}")
        return int(h.value), int(n.value)


def load_cpu_baseline() -> CpuBaseline:
    build_cpu_baseline()
    return CpuBaseline()


class COracle:
    """ctypes view of oracle/build/liboracle.so."""

    def __init__(self, path: str | None = None):
        path = path or LIB_PATH
        if not os.path.exists(path):
            build_c_oracle()
        self.lib = ctypes.CDLL(path)
        u64, sz, p = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_char_p
        self.lib.oracle_hash.restype = u64
        self.lib.oracle_hash.argtypes = [p, sz, u64]
        self.lib.oracle_min.restype = ctypes.c_int
        self.lib.oracle_min.argtypes = [p, sz, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        self.lib.oracle_min_mt.restype = ctypes.c_int
        self.lib.oracle_min_mt.argtypes = [p, sz, u64, u64, ctypes.c_int,
                                           ctypes.POINTER(u64), ctypes.POINTER(u64)]
        self.lib.oracle_hash_range.restype = None
        self.lib.oracle_hash_range.argtypes = [p, sz, u64, u64, ctypes.c_void_p]

    def hash(self, msg: bytes, nonce: int) -> int:
        return int(self.lib.oracle_hash(msg, len(msg), nonce))

    def min(self, msg: bytes, lower: int, upper: int, threads: int = 1) -> tuple[int, int]:
        h, n = ctypes.c_uint64(), ctypes.c_uint64()
        if threads > 1:
            rc = self.lib.oracle_min_mt(msg, len(msg), lower, upper, threads,
                                        ctypes.byref(h), ctypes.byref(n))
        else:
            rc = self.lib.oracle_min(msg, len(msg), lower, upper, ctypes.byref(h), ctypes.byref(n))
        if rc != 0:
            raise ValueError("lower > upper")
        return int(h.value), int(n.value)

    def hash_range(self, msg: bytes, lower: int, count: int):
        import numpy as np
        out = np.empty(count, dtype=np.uint64)
        self.lib.oracle_hash_range(msg, len(msg), lower, count, out.ctypes.data)
        return out


GOLDEN_PATH = os.path.join(HERE, "build", "libgoldenscan.so")


def build_golden_scan(force: bool = False) -> str:
    """oracle/golden_scan.c: the SHA-NI / AVX-512 scanner for the large fixtures."""
    src = os.path.join(HERE, "golden_scan.c")
    if force or not os.path.exists(GOLDEN_PATH) or os.path.getmtime(GOLDEN_PATH) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(GOLDEN_PATH), exist_ok=True)
        subprocess.check_call(["gcc", "-O3", "-msha", "-msse4.1", "-fPIC", "-shared", "-pthread",
                               "-o", GOLDEN_PATH, src])
    return GOLDEN_PATH


class GoldenScan:
    """ctypes view of oracle/build/libgoldenscan.so (large goldens only)."""

    def __init__(self):
        self.lib = ctypes.CDLL(build_golden_scan())
        u64, sz, p = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_char_p
        self.lib.golden_available.restype = ctypes.c_int
        self.lib.golden_hash.restype = u64
        self.lib.golden_hash.argtypes = [p, sz, u64]
        self.lib.golden_min.restype = ctypes.c_int
        self.lib.golden_min.argtypes = [p, sz, u64, u64, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(u64), ctypes.POINTER(u64)]

    def available(self) -> bool:
        return bool(self.lib.golden_available())

    def hash(self, msg: bytes, nonce: int) -> int:
        return int(self.lib.golden_hash(msg, len(msg), nonce))

    def min(self, msg: bytes, lower: int, upper: int, threads: int = 1,
            progress: bool = False) -> tuple[int, int]:
        h, n = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self.lib.golden_min(msg, len(msg), lower, upper, threads, int(progress),
                                 ctypes.byref(h), ctypes.byref(n))
        if rc != 0:
            raise ValueError(f"golden_min rc={rc}")
        return int(h.value), int(n.value)


def load_c_oracle() -> COracle:
    build_c_oracle()
    return COracle()
