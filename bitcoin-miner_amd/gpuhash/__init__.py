"""gpuhash -- Python host-side mirror of the reference's hot-path interface.

The product is the C-ABI library ``lib/libgpuhash.so`` (include/gpuhash.h) with the
gfx950 HIP kernels.  This module is a thin ctypes binding over it that mirrors the Go
names of the reference so tests and bench read like the reference's own code:

  reference (mohitreddy1996/BitCoin-Miner)                 here
  bitcoin.Hash(msg, nonce)       bitcoin/hash.go:11-15      Hash(msg, nonce)
  bitcoin.Message/MsgType        bitcoin/message.go:8-21    Message, MsgType
  bitcoin.NewRequest/NewResult   bitcoin/message.go:25-42   NewRequest, NewResult
  bitcoin.NewJoin                bitcoin/message.go:45-47   NewJoin
  miner loop (spec'd, stubbed)   bitcoin/miner/miner.go:15  Miner.handle(request)
                                 p1.pdf pp.12-14

There is no CPU fallback: if the shared library or a gfx950 device is missing, the
constructors raise.  (``Hash`` for a single nonce is the host convenience
gpuhash_hash_cpu, the Go miner's optional self-check -- never used for a search.)
"""
from __future__ import annotations

import ctypes
import enum
import os
from dataclasses import dataclass

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libgpuhash.so")
# test-only build of the same sources with the hash truncated to 4 bits (ties everywhere)
TIETEST_LIB_PATH = os.path.join(PKG_DIR, "lib", "libgpuhash_tietest.so")

GPUHASH_OK = 0
GPUHASH_EINVAL = -1
GPUHASH_ENODEV = -2
GPUHASH_EHIP = -3
GPUHASH_ETOOLONG = -4
GPUHASH_ENOMEM = -5
GPUHASH_MAX_MSG = 1 << 20
LAYOUT_AUTO, LAYOUT_UNIFORM, LAYOUT_CLASSIC, LAYOUT_LANETABLE = 0, 1, 2, 3
# OR-able flags: tail-digit launches always / never (include/gpuhash.h)
LAYOUT_TAIL_ALWAYS, LAYOUT_TAIL_NEVER = 16, 32
TAIL_MIN_SPAN = 1 << 33

# Every symbol include/gpuhash.h declares (tests check the .so exports all of them).
EXPORTED = [
    "gpuhash_open", "gpuhash_ndevices", "gpuhash_device_count", "gpuhash_shard_range",
    "gpuhash_shard_range_policy",
    "gpuhash_set_layout_policy", "gpuhash_min", "gpuhash_min_ex",
    "gpuhash_hash_range", "gpuhash_hash_cpu", "gpuhash_last_stats", "gpuhash_last_launches",
    "gpuhash_close",
    "gpuhash_strerror", "gpuhash_version",
]


UINT64_MAX = (1 << 64) - 1
# deterministic argument errors: the same call fails the same way on any device/miner
ARGUMENT_ERRORS = (GPUHASH_EINVAL, GPUHASH_ETOOLONG)


class GpuHashError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        super().__init__(f"{what}: {_lib().gpuhash_strerror(rc).decode()} (rc={rc})")

    @property
    def is_argument_error(self) -> bool:
        """True for EINVAL/ETOOLONG: retrying the job on another miner cannot succeed.
        False for device/resource errors (ENODEV/EHIP/ENOMEM)."""
        return self.rc in ARGUMENT_ERRORS


def _check_u64(name: str, v) -> int:
    """Bounds cross the ABI as uint64_t; ctypes would silently wrap anything outside
    [0, 2^64-1] (2**64+5 -> 5), so out-of-range or non-integer values are refused here."""
    if isinstance(v, bool) or not isinstance(v, int):
        raise TypeError(f"{name} must be an int, got {type(v).__name__}")
    if not 0 <= v <= UINT64_MAX:
        raise ValueError(f"{name}={v} outside [0, 2^64-1]")
    return v


class Stats(ctypes.Structure):
    _fields_ = [
        ("nonces", ctypes.c_uint64),
        ("launches", ctypes.c_uint32),
        ("ndevices", ctypes.c_uint32),
        ("wall_ms", ctypes.c_double),
        ("kernel_ms", ctypes.c_double),
        ("max_dev_kernel_ms", ctypes.c_double),
    ]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


def compressions_per_nonce(rec: dict) -> int:
    """SHA-256 compressions one nonce of a launch costs: its `c` nonce-bearing blocks, plus
    the all-constant padding block an EX layout compresses from a per-nonce state (message
    lengths 44-53 mod 64 at 10-12 digits).  The roofline charges
    OPS_PER_BLOCK per compression; SURVEY 8(d)'s c-based figure
    undercounts an EX launch's work by half."""
    return int(rec["c"]) + (1 if rec["EX"] else 0)


class LaunchRecord(ctypes.Structure):
    """gpuhash_launch_record (include/gpuhash.h)."""
    _fields_ = [(n, ctypes.c_int32) for n in ("device", "J", "C2", "EX", "digits", "c", "shard",
                                               "stream_device")] + [
        ("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64),
        ("nonces", ctypes.c_uint64), ("ms", ctypes.c_double), ("sclk_mhz", ctypes.c_double)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


_LIB = None


def _lib(path: str | None = None) -> ctypes.CDLL:
    """Loads libgpuhash.so (raises if it was not built: run __graft_entry__.build())."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(f"{p} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(p)
    u64, sz, u8p = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_char_p
    vp = ctypes.c_void_p
    lib.gpuhash_open.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(vp)]
    lib.gpuhash_open.restype = ctypes.c_int
    lib.gpuhash_ndevices.argtypes = [vp]
    lib.gpuhash_ndevices.restype = ctypes.c_int
    lib.gpuhash_device_count.argtypes = []
    lib.gpuhash_device_count.restype = ctypes.c_int
    lib.gpuhash_shard_range.argtypes = [sz, u64, u64, ctypes.c_int, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.gpuhash_shard_range.restype = ctypes.c_int
    lib.gpuhash_shard_range_policy.argtypes = [sz, u64, u64, ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.gpuhash_shard_range_policy.restype = ctypes.c_int
    lib.gpuhash_min.argtypes = [vp, u8p, sz, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.gpuhash_min.restype = ctypes.c_int
    lib.gpuhash_set_layout_policy.argtypes = [vp, ctypes.c_int]
    lib.gpuhash_set_layout_policy.restype = ctypes.c_int
    lib.gpuhash_min_ex.argtypes = [vp, u8p, sz, u64, u64, ctypes.c_uint32,
                                   ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.gpuhash_min_ex.restype = ctypes.c_int
    lib.gpuhash_hash_range.argtypes = [vp, u8p, sz, u64, u64, vp]
    lib.gpuhash_hash_range.restype = ctypes.c_int
    lib.gpuhash_hash_cpu.argtypes = [u8p, sz, u64]
    lib.gpuhash_hash_cpu.restype = u64
    lib.gpuhash_last_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    lib.gpuhash_last_stats.restype = ctypes.c_int
    lib.gpuhash_last_launches.argtypes = [vp, ctypes.POINTER(LaunchRecord), ctypes.c_int]
    lib.gpuhash_last_launches.restype = ctypes.c_int
    lib.gpuhash_close.argtypes = [vp]
    lib.gpuhash_close.restype = None
    lib.gpuhash_strerror.argtypes = [ctypes.c_int]
    lib.gpuhash_strerror.restype = ctypes.c_char_p
    lib.gpuhash_version.argtypes = []
    lib.gpuhash_version.restype = ctypes.c_char_p
    if path is None:
        _LIB = lib
    return lib


def build_id(lib_path: str | None = None) -> str:
    """Hash of the sources the loaded library was built from (gpuhash_version's build=)."""
    v = _lib(lib_path).gpuhash_version().decode()
    for tok in v.split():
        if tok.startswith("build="):
            return tok[len("build="):]
    return "unknown"


def device_count() -> int:
    """Visible HIP devices (gpuhash_device_count)."""
    return int(_lib().gpuhash_device_count())


def shard_range(msg_len: int, lower: int, upper: int, nshards: int,
                policy: int | None = None) -> list[tuple[int, int] | None]:
    """gpuhash_shard_range(_policy): the engine's cost-balanced contiguous partition of the
    inclusive [lower, upper] into nshards pieces (None = empty shard), priced under the
    layout `policy` (default AUTO) as gpuhash_min's own shards are.  Host-only."""
    _check_u64("lower", lower)
    _check_u64("upper", upper)
    if isinstance(nshards, bool) or not isinstance(nshards, int) or nshards < 1:
        raise ValueError(f"nshards={nshards!r} must be an int >= 1")
    lo = (ctypes.c_uint64 * nshards)()
    hi = (ctypes.c_uint64 * nshards)()
    if policy is None:
        rc = _lib().gpuhash_shard_range(int(msg_len), lower, upper, nshards, lo, hi)
    else:
        rc = _lib().gpuhash_shard_range_policy(int(msg_len), lower, upper, nshards, int(policy), lo, hi)
    if rc < 0:
        raise GpuHashError(rc, "gpuhash_shard_range")
    return [(int(a), int(b)) if a <= b else None for a, b in zip(lo, hi)]


def _bytes(msg) -> bytes:
    return msg.encode() if isinstance(msg, str) else bytes(msg)


class Engine:
    """One gpuhash context (one or more gfx950 devices)."""

    def __init__(self, devices: list[int] | None = None, lib_path: str | None = None):
        lib = self._lib = _lib(lib_path)
        ctx = ctypes.c_void_p()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = lib.gpuhash_open(arr, len(devices), ctypes.byref(ctx))
        else:
            rc = lib.gpuhash_open(None, 0, ctypes.byref(ctx))
        if rc != GPUHASH_OK:
            raise GpuHashError(rc, "gpuhash_open")
        self._ctx = ctx

    @property
    def ndevices(self) -> int:
        return self._lib.gpuhash_ndevices(self._ctx)

    def set_layout_policy(self, policy: int) -> None:
        """LAYOUT_AUTO / LAYOUT_UNIFORM / LAYOUT_CLASSIC / LAYOUT_LANETABLE, optionally OR
        LAYOUT_TAIL_ALWAYS or LAYOUT_TAIL_NEVER (gpuhash_set_layout_policy)."""
        rc = self._lib.gpuhash_set_layout_policy(self._ctx, policy)
        if rc != GPUHASH_OK:
            raise GpuHashError(rc, "gpuhash_set_layout_policy")

    def min(self, msg, lower: int, upper: int, rchunk: int = 0) -> tuple[int, int]:
        """argmin over inclusive [lower, upper] of (Hash(msg, n), n).  Bounds outside
        [0, 2^64-1] raise ValueError; lower > upper raises GpuHashError(EINVAL)."""
        _check_u64("lower", lower)
        _check_u64("upper", upper)
        if isinstance(rchunk, bool) or not isinstance(rchunk, int) or not 0 <= rchunk < 1 << 32:
            raise ValueError(f"rchunk={rchunk!r} outside [0, 2^32)")
        m = _bytes(msg)
        h, n = ctypes.c_uint64(), ctypes.c_uint64()
        rc = self._lib.gpuhash_min_ex(self._ctx, m, len(m), lower, upper, rchunk,
                                   ctypes.byref(h), ctypes.byref(n))
        if rc != GPUHASH_OK:
            raise GpuHashError(rc, "gpuhash_min")
        return int(h.value), int(n.value)

    def hash_range(self, msg, lower: int, count: int):
        """numpy uint64 array of Hash(msg, lower + i), computed by the scan kernels."""
        import numpy as np
        _check_u64("lower", lower)
        _check_u64("count", count)
        m = _bytes(msg)
        out = np.empty(count, dtype=np.uint64)
        rc = self._lib.gpuhash_hash_range(self._ctx, m, len(m), lower, count, out.ctypes.data)
        if rc != GPUHASH_OK:
            raise GpuHashError(rc, "gpuhash_hash_range")
        return out

    def stats(self) -> dict:
        s = Stats()
        self._lib.gpuhash_last_stats(self._ctx, ctypes.byref(s))
        return s.as_dict()

    def launches(self) -> list[dict]:
        """Per-launch records (variant, nonces, HIP-event ms) of the last call."""
        n = self._lib.gpuhash_last_launches(self._ctx, None, 0)
        arr = (LaunchRecord * max(n, 1))()
        n = self._lib.gpuhash_last_launches(self._ctx, arr, n)
        return [arr[i].as_dict() for i in range(n)]

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.gpuhash_close(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- mirror of the reference's bitcoin package (bitcoin/message.go, hash.go) ----

class MsgType(enum.IntEnum):
    """bitcoin/message.go:8-12 (iota order)."""
    Join = 0
    Request = 1
    Result = 2


@dataclass
class Message:
    """bitcoin.Message, message.go:16-21 (JSON field names match Go's)."""
    Type: MsgType
    Data: str = ""
    Lower: int = 0
    Upper: int = 0
    Hash: int = 0
    Nonce: int = 0

    def to_json(self) -> dict:
        return {"Type": int(self.Type), "Data": self.Data, "Lower": self.Lower,
                "Upper": self.Upper, "Hash": self.Hash, "Nonce": self.Nonce}

    def __str__(self) -> str:  # Message.String, message.go:49-60
        if self.Type == MsgType.Request:
            return f"[Request {self.Data} {self.Lower} {self.Upper}]"
        if self.Type == MsgType.Result:
            return f"[Result {self.Hash} {self.Nonce}]"
        return "[Join]"


def NewRequest(data: str, lower: int, upper: int) -> Message:  # message.go:25-32
    return Message(MsgType.Request, Data=data, Lower=lower, Upper=upper)


def NewResult(hash_: int, nonce: int) -> Message:  # message.go:36-42
    return Message(MsgType.Result, Hash=hash_, Nonce=nonce)


def NewJoin() -> Message:  # message.go:45-47
    return Message(MsgType.Join)


def Hash(msg, nonce: int) -> int:
    """bitcoin.Hash(msg, nonce), hash.go:11-15 (one nonce, host)."""
    m = _bytes(msg)
    return int(_lib().gpuhash_hash_cpu(m, len(m), _check_u64("nonce", nonce)))


class Miner:
    """The miner's Request -> Result step (miner.go:15 TODO; p1.pdf pp.13-14), on GPU.

    Go strings are byte strings: Data is hashed as its UTF-8 bytes, as
    []byte(fmt.Sprintf("%s %d", ...)) does (hash.go:13).
    """

    def __init__(self, devices: list[int] | None = None, engine: Engine | None = None):
        self.engine = engine or Engine(devices)

    def handle(self, req: Message) -> Message:
        if req.Type != MsgType.Request:
            raise ValueError(f"miner expects a Request, got {req}")
        h, n = self.engine.min(req.Data, req.Lower, req.Upper)
        return NewResult(h, n)
