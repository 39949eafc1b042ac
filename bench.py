#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X nonce-search engine.

Metric (BASELINE.json): nonces hashed/sec (GH/s) per GPU and per 8-GPU node; % of
VALU int32 peak.  One "step" = one full search of config 2 -- msg "bradfitz" (one
SHA block), 2^32 nonces -- per GPU, i.e. gpuhash_min over the rank's shard plus the
16-byte cross-rank merge.  Weak scaling: rank r searches [r*2^32, (r+1)*2^32).

  python bench.py                       # N=1, defaults finish in well under a minute
  python bench.py --gpus N              # ONE process drives devices 0..N-1 (the north_star
                                        # design: cost-balanced shards, a host thread +
                                        # stream per device, 16-byte host argmin); exits
                                        # non-zero when fewer than N devices are visible
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
                                        # one process per GPU (the driver's N>1 launch);
                                        # --gpus must equal WORLD_SIZE

Inputs are resident on the device before timing (the message is a kernel argument;
the nonce space is generated in registers), so value = whole-job nonces / max-over-
ranks wall time of K steps.  Extra keys: roofline (dominant scan kernel, HIP-event
timed in this run on the library's own stream), cpu_baseline (oracle/ C restatement
of the reference loop, timed on this host on a bounded sample, rank 0 at N=1 only), and
search_2p40: after the timed steps, ONE search of 'bradfitz' over [0, 2^40) on the same
N devices (north_star: "near-linear 1->8 GPU GH/s scaling on a 2^40-nonce search"), its
time, GH/s, per-shard device ordinals, and its (hash, nonce) checked against the CPU
golden (exit 3 on a mismatch).  ~33 s on one GPU, ~33/N s on N; --no-search skips it.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))

METRIC = "nonces hashed/sec (GH/s) per GPU and per 8-GPU node; % of VALU int32 peak"
# VALU peak of gfx950 from /opt/skills/guides/MI355X_MICROARCH.md: 4 SIMD-32 per CU, one
# wave64 instruction per 2 cycles per SIMD -> 256 CU x 128 lanes/clk x 2.4 GHz = 78.6 T
# lane-ops/s.  No instruction stream can issue above it, so it is `peak`.
VALU_PEAK_T = 256 * 128 * 2.4e9 / 1e12
# SURVEY.md 8(d)'s figure, 256 CU x 64 lanes/clk x 2.4 GHz = 39.3 T: every instruction at
# 4 cycles per wave64, which is what v_alignbit / v_add3 / v_bfi cost on gfx950 and what
# any stream containing them settles at.  Reported beside `frac`.
SURVEY_PEAK_T = 256 * 64 * 2.4e9 / 1e12
NORTH_STAR_FRAC = 0.70  # BASELINE.json north_star: ">= 70% of gfx950 VALU int32 peak per GPU"
OPS_PER_BLOCK = 1378  # minimal gfx950 VALU ops of one generic SHA-256 compression
MSG = b"bradfitz"
PER_GPU = 1 << 32
M120 = (b"The quick brown fox jumps over the lazy dog. " * 3)[:120]
# BASELINE.json configs measurable by this script (configs 1 and 5 are LSP plumbing):
#   2 (headline): 'bradfitz', 2^32 nonces per GPU, weak scaling
#   3: the 120-byte message over the 9->10 and 10->11 digit windows (2 x (2^29+1) nonces)
#   4: 'bradfitz', 2^37 nonces per GPU at offset rank*2^37 -> at N=8 exactly [0, 2^40)
CONFIGS = {
    "2": {"msg": MSG, "windows": lambda r: [(r * PER_GPU, (r + 1) * PER_GPU - 1)],
          "desc": "config 2: msg 'bradfitz' (1 SHA block), 2^32 nonces per GPU (rank r: [r*2^32, (r+1)*2^32)), argmin (hash, nonce)"},
    "3": {"msg": M120, "windows": lambda r: [(10 ** 9 - (1 << 28), 10 ** 9 + (1 << 28)),
                                             (10 ** 10 - (1 << 28), 10 ** 10 + (1 << 28))],
          "desc": "config 3: 120-byte msg (3 SHA blocks, host midstate for block 0), windows 10^9 +- 2^28 and 10^10 +- 2^28 per GPU"},
    "4": {"msg": MSG, "windows": lambda r: [(r << 37, ((r + 1) << 37) - 1)],
          "desc": "config 4: msg 'bradfitz', 2^37 nonces per GPU (rank r: [r*2^37, (r+1)*2^37)); N=8 covers [0, 2^40)"},
}


def _time_min(fn, seconds: float, n0: int) -> tuple[int, int, float]:
    """Times fn(lo, hi) on the top of config 2's range (the d=10 nonces), first on n0
    nonces, then on a sample sized to take ~`seconds`; returns (lo, n, dt)."""
    t = time.perf_counter()
    fn(PER_GPU - n0, PER_GPU - 1)
    dt = time.perf_counter() - t
    n = max(n0, int(n0 * seconds / max(dt, 1e-6)))
    lo = PER_GPU - n
    t = time.perf_counter()
    fn(lo, PER_GPU - 1)
    return lo, n, time.perf_counter() - t


def _cgroup_cpus() -> float | None:
    """CPUs' worth of time the cgroup v2 quota grants (cpu.max "quota period"), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        return None


def host_cpus() -> dict:
    """The host the CPU baselines ran on: nproc (every CPU of the machine), the CPUs this
    process may run on (sched_getaffinity), the cgroup CPU quota if one is set, the CPU
    model, and `usable` = the affinity count, lowered to the quota when a quota caps it
    (threads beyond the quota would only time-slice)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = _cgroup_cpus()
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "model": model,
            "usable": usable}


def _threads() -> int:
    """One worker per usable CPU (one goroutine per core)."""
    return host_cpus()["usable"]


def cpu_baseline(seconds: float = 12.0) -> dict:
    """The reference miner loop (fresh "%s %d" buffer + SHA-256 per nonce, ascending,
    strict '<') on one core, on a bounded sample of the same workload: the d=10 nonces
    at the top of config 2's range.  SHA-256 is OpenSSL's (oracle/cpu_baseline.c; SHA-NI
    where the host has it), the closest stand-in here for Go's assembly crypto/sha256;
    without libcrypto it falls back to the plain-C oracle."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import hash_oracle as ho
    b = ho.load_cpu_baseline()
    if b.available():
        lo, n, dt = _time_min(lambda a, z: b.min(MSG, a, z), seconds, 1 << 18)
        what = "oracle/cpu_baseline.c (OpenSSL SHA-256 per nonce, as Go's asm crypto/sha256)"
    else:
        c = ho.load_c_oracle()
        lo, n, dt = _time_min(lambda a, z: c.min(MSG, a, z), seconds, 1 << 16)
        what = "oracle/hash_oracle.c (plain-C SHA-256; libcrypto unavailable)"
    return {"value": n / dt / 1e9, "unit": "GH/s", "cores": 1, "kind": "port",
            "sample": f"{what} scan of bradfitz [{lo}, {PER_GPU - 1}] ({n} nonces, 10 digits), "
                      f"{dt:.1f} s; reference Go miner unavailable (no Go toolchain)"}


def cpu_baseline_plain_c(seconds: float = 5.0) -> dict:
    """The same loop with the oracle's plain-C SHA-256 (the checker), one core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import hash_oracle as ho
    c = ho.load_c_oracle()
    lo, n, dt = _time_min(lambda a, z: c.min(MSG, a, z), seconds, 1 << 16)
    return {"value": n / dt / 1e9, "unit": "GH/s", "cores": 1, "kind": "port",
            "sample": f"oracle/hash_oracle.c scan of bradfitz [{lo}, {PER_GPU - 1}] ({n} nonces), {dt:.1f} s"}


def cpu_baseline_multicore(seconds: float = 5.0) -> dict:
    """The loop over contiguous per-thread sub-ranges (the SURVEY's 'one goroutine per
    core' variant), one thread per CPU in this process's affinity set, OpenSSL SHA-256."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import hash_oracle as ho
    threads = _threads()
    b = ho.load_cpu_baseline()
    if b.available():
        fn, what = (lambda a, z: b.min(MSG, a, z, threads=threads)), "cpu_baseline.c (OpenSSL SHA-256)"
    else:
        c = ho.load_c_oracle()
        fn, what = (lambda a, z: c.min(MSG, a, z, threads=threads)), "oracle_min_mt (plain C)"
    lo, n, dt = _time_min(fn, seconds, 1 << 20)
    return {"value": n / dt / 1e9, "unit": "GH/s", "cores": threads, "kind": "port",
            "host": host_cpus(),
            "sample": f"{what} over bradfitz [{lo}, {PER_GPU - 1}] ({n} nonces), {dt:.1f} s"}


# committed rocprofv3 PMC summary per bench config (tools/summarize_prof.py): each was
# collected on the same bench.py workload, so its per-launch counters match this run's
# launches of the same kernel
PMC_SUMMARY = {"2": "r06_pmc_summary.json", "3": "r06c3_pmc_summary.json", "4": "r06c4_pmc_summary.json"}


def pmc_source(config: str, key, launch_cycles: float | None = None) -> tuple[dict | None, dict]:
    """(per-kernel PMC entry or None, provenance).  PMC counters cannot be read inside
    this process, so they come from the committed rocprofv3 summary of the same bench
    command -- but only if that summary was collected on a library with this library's
    build id (the hash of its sources, gpuhash_version): after any source change the
    values are stale and the fields they feed are null until the passes are re-run.
    Its counters are per launch, so they also need a launch of the same size: with
    `launch_cycles` (this run's dominant launch, HIP-event ms x in-kernel clock) the entry
    is used only while the profiled launch's GPU cycles are within 0.8-1.25x of it (a
    profiled run clocks a few per cent lower).  --inproc rehearsals and non-default
    ranges launch other sizes of the same kernel."""
    import gpuhash
    lib_id = gpuhash.build_id()
    prov = {"file": None, "build_id": None, "library_build_id": lib_id, "used": False}
    name = PMC_SUMMARY.get(config)
    if name is None:
        prov["reason"] = f"no PMC summary for config {config}"
        return None, prov
    prov["file"] = f"profiles/{name}"
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            t = json.load(f)
    except (OSError, ValueError) as e:
        prov["reason"] = f"unreadable: {e}"
        return None, prov
    prov["build_id"] = t.get("build_id")
    if t.get("build_id") != lib_id:
        prov["reason"] = "collected on a different build: PMC-derived fields are null"
        return None, prov
    e = t.get("kernels", {}).get(f"k_scan<{key[0]}, {int(key[1])}, {str(bool(key[2])).lower()}, 0>")
    if e is None:
        prov["reason"] = "dominant kernel not in the summary"
        return None, prov
    prof_cycles = e.get("gpu_cycles_per_launch")
    if launch_cycles and prof_cycles:
        ratio = launch_cycles / prof_cycles
        if not 0.8 <= ratio <= 1.25:
            prov["reason"] = (f"profiled launch is another size ({prof_cycles:.3g} GPU cycles vs "
                              f"{launch_cycles:.3g} here): PMC-derived fields are null")
            return None, prov
    prov["used"] = True
    return e, prov


def pmc_traffic(e: dict | None) -> float | None:
    """HBM bytes per launch of the dominant kernel: FETCH_SIZE x2 (gfx950 correction) +
    WRITE_SIZE, collected in separate --pmc passes (tools/gpu_session.sh pmc / pmc3)."""
    return e.get("hbm_bytes_per_launch") if e else None


def pmc_issued(e: dict | None) -> float | None:
    """VALU wave-instructions per launch of the dominant kernel (SQ_INSTS_VALU, its own
    --pmc pass); x64 lanes / nonces = issued lane-instructions per nonce, the
    hardware-counted work behind `achieved`."""
    return e["per_launch"].get("SQ_INSTS_VALU") if e else None


_JSON_FD = None


def _quiet_stdout() -> None:
    """Keeps stdout for the ONE result line: fd 1 is pointed at stderr for the rest of the
    run, so library banners (RCCL prints its version block to stdout at communicator
    init) cannot land next to it; emit() writes to the saved original stdout."""
    global _JSON_FD
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)


def emit(out: dict) -> None:
    line = (json.dumps(out) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


def dominant(recs: list[dict]) -> tuple[tuple, dict]:
    """The dominant scan variant of a list of launch records: the one with the most
    algorithmic work (nonces x blocks).  On a GPU of its own that is also the one with the
    most HIP-event time; ranks rehearsed on one shared GPU wait behind each other's
    launches, so their event time would pick a short launch that happened to queue."""
    from gpuhash import compressions_per_nonce
    by = {}
    for r in recs:
        k = (r["J"], r["C2"], r["EX"])
        e = by.setdefault(k, {"ms": 0.0, "n": 0, "nonces": 0, "c": r["c"], "clk_ms": 0.0,
                              "comp": compressions_per_nonce(r)})
        e["ms"] += r["ms"]
        e["clk_ms"] += r["sclk_mhz"] * r["ms"]  # ms-weighted in-kernel shader clock
        e["n"] += 1
        e["nonces"] += r["nonces"]
    return max(by.items(), key=lambda kv: kv[1]["nonces"] * kv[1]["comp"])


def roofline(config: str, recs: list[dict]) -> dict:
    """roofline object of the bench line for the dominant kernel of `recs` (HIP-event
    timed on the library's own stream in this run)."""
    key, dom = dominant(recs)
    avg_ms = dom["ms"] / dom["n"]
    # OPS_PER_BLOCK per compression a nonce costs: c nonce-bearing blocks, plus the padding
    # block of an EX layout (gpuhash.compressions_per_nonce)
    ops_per_launch = dom["nonces"] / dom["n"] * OPS_PER_BLOCK * dom["comp"]
    achieved_T = ops_per_launch / (avg_ms * 1e-3) / 1e12
    kernel_ghs = dom["nonces"] / (dom["ms"] * 1e-3) / 1e9
    sclk = dom["clk_ms"] / dom["ms"] if dom["ms"] > 0 else 0.0  # MHz, measured in the kernel
    peak_at_clk = 256 * 128 * sclk * 1e6 / 1e12  # the guide's peak at the measured clock
    pmc, prov = pmc_source(config, key, avg_ms * 1e-3 * sclk * 1e6 if sclk > 0 else None)
    insts = pmc_issued(pmc)
    issued_per_nonce = insts * 64 / (dom["nonces"] / dom["n"]) if insts else None
    issued_T = kernel_ghs * issued_per_nonce / 1e3 if issued_per_nonce else None
    return {
        "bound": "valu",
        # algorithmic: SURVEY 8(d)'s 1,378 lane-ops per nonce-bearing block x the
        # launch's nonces / its HIP-event time
        "achieved": round(achieved_T, 3),
        "peak": round(VALU_PEAK_T, 3),
        "unit": "T int32 lane-ops/s",
        "frac": round(achieved_T / VALU_PEAK_T, 4),
        # the north_star's target, stated in every line: >= 70% of the VALU
        # int32 peak per GPU.  Not met: SHA-256's rotates and 3-input adds issue at 4.2
        # cycles per wave64 on gfx950, the loop's instruction count is at its floor, and its
        # mix bounds the additive issue rate at 0.674 of peak
        "target_frac": NORTH_STAR_FRAC,
        "target_met": achieved_T / VALU_PEAK_T >= NORTH_STAR_FRAC,
        "frac_basis": "algorithmic ops / the guide's SIMD-32 VALU peak (2-cycle wave64 issue)"
                      + ("; the algorithmic count charges c=2 blocks per nonce but this layout "
                         "compresses block B-1 once per lane row, so frac exceeds 1: issued_frac "
                         "is the hardware-bounded figure" if achieved_T > VALU_PEAK_T else ""),
        "traffic": pmc_traffic(pmc),
        "kernel": f"k_scan<J={key[0]},C2={key[1]},EX={key[2]},MODE=0>",
        "avg_launch_ms": round(avg_ms, 4),
        "nonces_per_launch": dom["nonces"] / dom["n"],
        "ops_per_nonce": OPS_PER_BLOCK * dom["comp"],
        "compressions_per_nonce": dom["comp"],
        "ops_per_nonce_c_based": OPS_PER_BLOCK * dom["c"],  # nonce-bearing blocks only
        "kernel_GHs": round(kernel_ghs, 4),
        # hardware-counted view: SQ_INSTS_VALU x 64 / nonce from the committed PMC
        # pass of this build (pmc_source), times this run's kernel rate
        "issued_lane_instr_per_nonce": round(issued_per_nonce, 1) if issued_per_nonce else None,
        "issued_T": round(issued_T, 3) if issued_T else None,
        "issued_frac": round(issued_T / VALU_PEAK_T, 4) if issued_T else None,
        # SURVEY 8(d)'s 39.3 T = every instruction at 4 cycles per wave64, the cost of
        # v_alignbit / v_add3 / v_bfi: where a rotate-bearing stream settles
        "survey_peak": round(SURVEY_PEAK_T, 3),
        "frac_vs_survey_peak": round(achieved_T / SURVEY_PEAK_T, 4),
        "issued_frac_vs_survey_peak": round(issued_T / SURVEY_PEAK_T, 4) if issued_T else None,
        "peak_basis": "MI355X_MICROARCH.md: 4 SIMD-32/CU, wave64 VALU issue every 2 cycles, "
                      "256 CU at 2.4 GHz; SURVEY 8(d) 4-cycle figure as survey_peak",
        "pmc_source": prov,
        # shader clock over the dominant launches, from s_memtime / s_memrealtime in
        # workgroup 0 (record the sustained sclk beside every GH/s)
        "sclk_mhz": round(sclk, 1),
        "peak_at_sclk": round(peak_at_clk, 3),
        "frac_at_sclk": round(achieved_T / peak_at_clk, 4) if peak_at_clk else None,
    }


def per_device(recs: list[dict], steps: int) -> tuple[list[dict], int, list[dict]]:
    """Per device (shard) of the in-process path: its launches' HIP-event time per step,
    nonces per step and kernel rate; plus the SLOWEST device (most kernel time: it sets the
    step time) and its launch records, whose dominant kernel is the line's roofline."""
    by = {}
    for r in recs:
        e = by.setdefault(r["device"], {"recs": [], "ms": 0.0, "nonces": 0})
        e["recs"].append(r)
        e["ms"] += r["ms"]
        e["nonces"] += r["nonces"]
    slow = max(by, key=lambda d: by[d]["ms"])
    rows = [{"device": d, "kernel_ms_per_step": round(e["ms"] / steps, 3),
             "nonces_per_step": e["nonces"] // steps,
             "kernel_GHs": round(e["nonces"] / (e["ms"] * 1e-3) / 1e9, 4) if e["ms"] > 0 else None}
            for d, e in sorted(by.items())]
    return rows, slow, by[slow]["recs"]


def base_line(args, value: float, n: int, dt: float, workload: str, msg: bytes, parallelism: str,
              scaling: str, **config) -> dict:
    return {
        "metric": METRIC, "value": round(value, 4), "unit": "GH/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (the nonce space itself; fixed message)",
        "config": {"workload": workload, "msg_len": len(msg), "parallelism": parallelism, **config},
        "per_gpu_GHs": round(value / n, 4),
    }


# ---- the north_star's 2^40 search (BASELINE configs[3]) at every N ----
#
# After the timed steps, one search of `bradfitz` over [0, 2^40) -- the range the
# north_star's "near-linear 1->8 GPU GH/s scaling on a 2^40-nonce search" names -- on the
# same devices: in-process, one gpuhash_min over the context's devices (cost-balanced
# shards, a host thread + stream each, host argmin); under torchrun, each rank's
# cost-balanced window (gpuhash.dist.split_range) and the 24-byte gloo merge.  The result
# is checked against the CPU golden of the same range (tests/golden/golden.json,
# cfg4_bradfitz_2p40, computed by oracle/golden_scan.c), so the line proves the search
# bit-exact at every N; a mismatch exits non-zero after the line is printed.
SEARCH_DEFAULT = (0, (1 << 40) - 1)
GOLDEN_PATH = os.path.join(ROOT, "tests", "golden", "golden.json")


def parse_search(s: str):
    """--search: "LO:HI" (inclusive, ints; "2^40" style powers allowed) or "off"."""
    if s == "off":
        return None

    def num(x: str) -> int:
        x = x.strip()
        if "^" in x:  # "2^40-1"
            base, rest = x.split("^", 1)
            sub = 0
            if "-" in rest:
                rest, sub = rest.split("-", 1)
                sub = int(sub)
            return int(base) ** int(rest) - sub
        return int(x)
    lo, hi = (num(x) for x in s.split(":"))
    if not 0 <= lo <= hi < 1 << 64:
        raise ValueError(f"--search {s}: need 0 <= LO <= HI < 2^64")
    return lo, hi


def golden_for(msg: bytes, lo: int, hi: int):
    """((hash, nonce), name) of the committed CPU golden for exactly this range, or
    (None, None).  The fixture travels with the repo; nothing here reads the reference."""
    try:
        with open(GOLDEN_PATH) as f:
            g = json.load(f)
    except (OSError, ValueError):
        return None, None
    for r in g.get("ranges", []):
        if r.get("msg_hex") == msg.hex() and r.get("lower") == lo and r.get("upper") == hi:
            return (int(r["hash"]), int(r["nonce"])), r["name"]
    return None, None


def shard_rows(recs: list[dict]) -> list[dict]:
    """Per shard (position in the context's device list) of one or more gpuhash_min calls:
    its HIP ordinal, the ordinal the runtime reports for its stream, the distinct nonce
    windows it searched (one per slice: a search longer than 2^38 nonces per device runs as
    slices, each cut over every shard, so a shard's windows interleave with the others'),
    and its scan kernels' time, rate and clock.  Every record of one slice of a shard
    carries that slice's [lo, hi] and the nonces of its own kernel group.

    `nonces` = the windows' size (each window once); `nonces_hashed` = the records' nonces
    summed over every call, which is what `kernel_ms` was spent on: over K timed steps of
    the same window it is K x `nonces`, so `kernel_GHs` is the shard's rate, not 1/K of it
    (VERDICT r04 weak 5).  `sclk_mhz` is the ms-weighted in-kernel shader clock."""
    by = {}
    for r in recs:
        e = by.setdefault(r["shard"], {"shard": r["shard"], "device": r["device"], "stream_devices": set(),
                                       "windows": set(), "kernel_ms": 0.0, "hashed": 0, "clk_ms": 0.0})
        e["stream_devices"].add(r["stream_device"])
        e["windows"].add((r["lo"], r["hi"]))
        e["kernel_ms"] += r["ms"]
        e["hashed"] += r["nonces"]
        e["clk_ms"] += r.get("sclk_mhz", 0.0) * r["ms"]
    rows = []
    for k in sorted(by):
        e = by[k]
        wins = sorted(e["windows"])
        nonces = sum(b - a + 1 for a, b in wins)
        ms = e["kernel_ms"]
        rows.append({"shard": k, "device": e["device"], "stream_device": sorted(e["stream_devices"]),
                     "windows": [list(w) for w in wins], "slices": len(wins), "nonces": nonces,
                     "nonces_hashed": e["hashed"], "kernel_ms": round(ms, 3),
                     "kernel_GHs": round(e["hashed"] / (ms * 1e-3) / 1e9, 4) if ms else None,
                     "sclk_mhz": round(e["clk_ms"] / ms, 1) if ms else None})
    return rows


def step_check(msg: bytes, windows, res) -> dict:
    """The timed step's (hash, nonce) against the committed CPU goldens:
    the step searches `windows` (inclusive), so its answer must be the lexicographic min of
    the goldens of exactly those windows.  When a window has no golden (config 2 over
    N > 1 GPUs: [0, N*2^32), config 4's 2^37-nonce windows) the check is skipped and says
    so; a mismatch exits 3 after the line (search_exit), like the 2^40 search."""
    want, names = [], []
    for lo, hi in windows:
        g, name = golden_for(msg, lo, hi)
        if g is None:
            return {"matches_golden": None, "golden": None, "golden_names": None,
                    "reason": f"no committed golden for [{lo}, {hi}]"}
        want.append(g)
        names.append(name)
    best = min(want)
    return {"matches_golden": tuple(res) == best, "golden": list(best), "golden_names": names}


def merge_windows(wins) -> list[tuple[int, int]]:
    """Sorted union of inclusive windows, adjacent ones joined."""
    out: list[tuple[int, int]] = []
    for lo, hi in sorted(set(tuple(w) for w in wins)):
        if out and out[-1][1] + 1 >= lo:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def tiles(rows: list[dict], lo: int, hi: int) -> bool:
    """The shards' windows, all slices together, cover [lo, hi] exactly once."""
    wins = sorted(tuple(w) for r in rows for w in r["windows"])
    return bool(wins) and wins[0][0] == lo and wins[-1][1] == hi and all(
        b[0] == a[1] + 1 for a, b in zip(wins, wins[1:]))


def pci_id(dev: int) -> str | None:
    """domain:bus:device of a HIP ordinal (torch's device properties): a physical GPU's
    identity, whatever ordinal a process's visibility mask gives it."""
    try:
        import torch
        p = torch.cuda.get_device_properties(dev)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    except Exception:  # noqa: BLE001 -- evidence only; None says it was unavailable
        return None


def _one_visible_device() -> bool:
    """True when a visibility variable leaves this process exactly one GPU."""
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(k)
        if v is not None and len([x for x in v.split(",") if x.strip()]) == 1:
            return True
    return False


def check_shards(rows: list[dict], devs: list[int]) -> list[str]:
    """Device evidence of a search's shards: shard k ran on devs[k] (the record's ordinal and
    the stream's runtime ordinal agree with it), and -- when the device list has no
    repeats -- every shard ran on a different device.  Returns the problems found (empty =
    fine)."""
    bad = []
    for r in rows:
        if r["shard"] >= len(devs) or r["device"] != devs[r["shard"]]:
            bad.append(f"shard {r['shard']} reports device {r['device']}, context lists {devs}")
        if r["stream_device"] != [r["device"]]:
            bad.append(f"shard {r['shard']} stream on device(s) {r['stream_device']}, not {r['device']}")
    if len(set(devs)) == len(devs) and len({r["device"] for r in rows}) != len(rows):
        bad.append("distinct devices requested but shards share a device")
    return bad


def search_line(res, dt: float, n: int, lo: int, hi: int, mode: str, devices, shards) -> dict:
    want, name = golden_for(MSG, lo, hi)
    total = hi - lo + 1
    return {"msg": MSG.decode(), "range": [lo, hi], "nonces": total, "mode": mode,
            "seconds": round(dt, 3), "GHs": round(total / dt / 1e9, 4),
            "per_gpu_GHs": round(total / dt / 1e9 / n, 4), "n_gpus": n, "devices": devices,
            "result": list(res), "golden": list(want) if want else None, "golden_name": name,
            "matches_golden": (tuple(res) == want) if want else None, "shards": shards}


def alone_rerun(make_engine, row: dict, t_all: float, barrier) -> dict:
    """Same-run scaling evidence: shard 0's exact window(s) of the
    N-device search, searched again ALONE on its device with the same engine code, after
    every other device has gone idle.  Perfect scaling means the N-device search took as
    long as its shard 0 takes alone, so scaling_efficiency = t_alone / t_all (shards are
    cost-balanced, so shard 0 stands for each of them).  The driver runs one N at a time;
    this puts a same-run baseline into every N > 1 line.  It is evidence only: a host-side
    failure is recorded in the object instead of ending the run (under torchrun the other
    ranks wait at a barrier for this one), like rank 0's in-process repeat."""
    launches = []
    try:
        with make_engine() as eng:  # closed even when a call raises
            # a fresh context's first call reserves its buffers and events: one small search
            # before the clock starts, so t_alone is hashing, as the N-device time is
            lo0, hi0 = row["windows"][0]
            eng.min(MSG, lo0, min(hi0, lo0 + (1 << 20)))
            barrier()
            t0 = time.perf_counter()
            for lo, hi in row["windows"]:
                eng.min(MSG, lo, hi)
                launches += eng.launches()
            barrier()
            t_alone = time.perf_counter() - t0
    except Exception as e:  # noqa: BLE001 -- see above
        return {"shard": row["shard"], "device": row["device"], "windows": row["windows"],
                "error": f"{type(e).__name__}: {e}"}
    return {"shard": row["shard"], "device": row["device"], "windows": row["windows"],
            "t_alone_s": round(t_alone, 3), "t_all_s": round(t_all, 3),
            "scaling_efficiency": round(t_alone / t_all, 4) if t_all > 0 else None,
            "alone_sclk_mhz": shard_rows(launches)[0]["sclk_mhz"] if launches else None}


def distinct_gpu_summary(out: dict) -> str | None:
    """One stderr line for a run over two or more distinct physical GPUs (VERDICT r05 item
    5), so the tail of the driver's 8-GPU log reads on its own: per GPU of the search (else
    of the timed steps) its kernel GH/s, in-kernel clock and (host,) PCI id, then the run's
    scaling_efficiency.  None when the run had one physical GPU (rehearsals on one GPU)."""
    for key in ("search_2p40", "search_2p40_inproc"):
        s = out.get(key)
        if s and s.get("shards"):
            rows, what = s["shards"], key
            break
    else:
        rows, what = out.get("shards") or [], "timed steps"
    ids = [(r.get("host"), r.get("pci")) if r.get("pci") else (None, f"ordinal {r['device']}") for r in rows]
    if len(set(ids)) < 2:
        return None
    parts = []
    for r, (host, pci) in zip(rows, ids):
        where = f"{host}/{pci}" if host else pci
        parts.append(f"gpu {r['device']} [{where}] {r.get('kernel_GHs')} GH/s @ {r.get('sclk_mhz')} MHz")
    eff = ((out.get("search_2p40") or {}).get("scaling") or {}).get("scaling_efficiency")
    return (f"bench.py: {len(set(ids))} distinct GPUs ({what}): " + "; ".join(parts)
            + f"; scaling_efficiency {eff}")


def search_exit(out: dict, problems: list[str]) -> None:
    """Non-zero exit AFTER the line is printed when the timed step or the search missed its
    golden or a shard ran somewhere other than its device: the line stays readable, the run
    counts as failed."""
    if out.get("matches_golden") is False:
        print(f"bench.py: the timed step returned {out.get('result')}, golden "
              f"{out['result_check']['golden']} ({out['result_check']['golden_names']})", file=sys.stderr)
        sys.exit(3)
    for key in ("search_2p40", "search_2p40_inproc"):
        s = out.get(key)
        if s is not None and s.get("matches_golden") is False:
            print(f"bench.py: {key} {s['range']} returned {s['result']}, golden {s['golden']}", file=sys.stderr)
            sys.exit(3)
    if problems:
        print("bench.py: device check failed: " + "; ".join(problems), file=sys.stderr)
        sys.exit(3)


def add_cpu_baselines(out: dict, args) -> None:
    if not args.no_cpu_baseline and args.config == "2":
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        out["cpu_baseline_multicore"] = cpu_baseline_multicore(args.cpu_seconds / 2)
        out["cpu_baseline_plain_c"] = cpu_baseline_plain_c(args.cpu_seconds / 4)


def fail(msg: str) -> None:
    print(f"bench.py: {msg}", file=sys.stderr)
    sys.exit(2)


def main_inproc(args, devs: list[int]) -> None:
    """All devices in ONE process, the north_star's design: one gpuhash context over
    devices `devs`, each step one gpuhash_min over the union of the per-GPU windows of
    ranks 0..N-1 (config 2/4: [0, N*per_gpu), weak scaling; config 3: the same two windows
    split over N devices, strong scaling).  Inside the call the engine cuts the range into
    N contiguous shards of equal estimated cost (gpuhash_shard_range), runs each on its
    device's own host thread + HIP stream, and takes the 16-byte host argmin: no
    collective, no torch.distributed."""
    import torch
    import gpuhash
    from gpuhash.dist import merge_min
    eng = gpuhash.Engine(devs)
    n = eng.ndevices
    cfg = CONFIGS[args.config]
    msg = cfg["msg"]
    # contiguous per-rank windows merge into one call
    merged = merge_windows(w for r in range(n) for w in cfg["windows"](r))
    total_per_step = sum(hi - lo + 1 for lo, hi in merged)

    def step(recs=None):
        parts = []
        for lo, hi in merged:
            parts.append(eng.min(msg, lo, hi))  # blocking: every device's stream is synced
            if recs is not None:
                recs.extend(eng.launches())
        return merge_min(parts)

    def barrier():  # gpuhash_min returns after its streams finish; torch's are idle
        for d in sorted(set(devs)):
            torch.cuda.synchronize(d)

    for _ in range(args.warmup):
        step()
    barrier()
    recs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step(recs)
    barrier()
    dt = time.perf_counter() - t0
    value = total_per_step * args.steps / dt / 1e9
    scaling = "strong" if args.config == "3" else "weak"
    out = base_line(args, value, n, dt, cfg["desc"] + (" -- in-process, one gpuhash context over all devices"
                                                      if n > 1 else ""),
                    msg, f"inproc{n}" if n > 1 else "single", scaling,
                    nonces_per_step=total_per_step, ranges=[list(w) for w in merged], devices=devs)
    out["per_device"], slow, slow_recs = per_device(recs, args.steps)
    out["result"] = list(res)
    out["result_check"] = step_check(msg, merged, res)
    out["matches_golden"] = out["result_check"]["matches_golden"]
    out["launches_per_step"] = len(recs) // max(args.steps, 1)
    out["roofline"] = roofline(args.config, slow_recs)
    out["roofline"]["device"] = slow
    out["shards"] = shard_rows(recs)  # device evidence of the timed steps (kernel_ms over all K)
    problems = check_shards(out["shards"], devs)
    if args.search is not None:
        lo, hi = args.search
        barrier()
        t0 = time.perf_counter()
        sres = eng.min(MSG, lo, hi)
        barrier()
        sdt = time.perf_counter() - t0
        rows = shard_rows(eng.launches())
        for r in rows:
            r["pci"] = pci_id(r["device"])
        problems += check_shards(rows, devs)
        pcis = [r["pci"] for r in rows]
        if len(set(devs)) == len(devs) and None not in pcis and len(set(pcis)) != len(rows):
            problems.append("distinct ordinals requested but two shards share a PCI device")
        if not tiles(rows, lo, hi):
            problems.append("the search's shard windows do not tile its range")
        out["search_2p40"] = search_line(sres, sdt, n, lo, hi, "inproc", devs, rows)
        if n > 1 and rows:
            out["search_2p40"]["scaling"] = alone_rerun(lambda: gpuhash.Engine([devs[0]]), rows[0], sdt, barrier)
    if problems:
        out["device_check"] = problems
    if n == 1:
        add_cpu_baselines(out, args)
    emit(out)
    summary = distinct_gpu_summary(out)
    if summary:
        print(summary, file=sys.stderr, flush=True)
    eng.close()
    search_exit(out, problems)


def main_ranks(args, world: int, rank: int, local: int) -> None:
    """One process per GPU (torch.distributed.run): rank r searches its own window(s) on
    device LOCAL_RANK.  No collective on the data path: the ranks' 24-byte results are
    merged on the host (a gloo all_gather over TCP, once per step), and the only other
    traffic is the timing contract's barrier and max-over-ranks.  GPUHASH_DIST_BACKEND=nccl
    moves those onto RCCL instead (GPUHASH_FORCE_DIST=1 runs this path at WORLD_SIZE=1)."""
    import torch
    import torch.distributed as dist
    import gpuhash
    from gpuhash.dist import gather_results, merge_min
    backend = os.environ.get("GPUHASH_DIST_BACKEND", "gloo")
    ndev = torch.cuda.device_count()
    if ndev < 1:
        fail("no visible GPU")
    shared = os.environ.get("GPUHASH_SHARE_GPU") == "1"  # rehearsal: ranks share device 0..
    # a launcher may instead give every rank exactly one visible GPU (HIP/ROCR/CUDA
    # _VISIBLE_DEVICES): then device 0 is the rank's own GPU, and the PCI check below
    # proves the ranks' GPUs distinct
    pinned = ndev == 1 and _one_visible_device()
    if local >= ndev and not (shared or pinned):
        fail(f"LOCAL_RANK {local} but only {ndev} visible device(s); "
             "set GPUHASH_SHARE_GPU=1 to rehearse several ranks on one GPU")
    local = local % ndev
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    coll_dev = dev if backend == "nccl" else None  # gloo moves CPU tensors

    eng = gpuhash.Engine([local])
    cfg = CONFIGS[args.config]
    msg, windows = cfg["msg"], cfg["windows"](rank)
    per_gpu = sum(hi - lo + 1 for lo, hi in windows)

    def step(recs=None):
        parts = []
        for lo, hi in windows:
            parts.append(eng.min(msg, lo, hi))
            if recs is not None:
                recs.extend(eng.launches())  # HIP-event time of every scan launch
        return merge_min(gather_results(merge_min(parts), coll_dev))

    def barrier():
        torch.cuda.synchronize(dev)
        dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    recs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step(recs)
    barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=coll_dev or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    roof = roofline(args.config, recs)
    # device evidence of every rank: its shard of the timed steps ran on LOCAL_RANK's device
    mine = shard_rows(recs)
    problems = check_shards(mine, [local])
    search = None
    if args.search is not None:
        from gpuhash.dist import split_range
        lo, hi = args.search
        win = split_range(lo, hi, world, msg_len=len(MSG))[rank]  # the engine's cost model
        barrier()
        t0 = time.perf_counter()
        sres = eng.min(MSG, *win) if win is not None else None
        sres = merge_min(gather_results(sres, coll_dev))
        barrier()
        sdt = time.perf_counter() - t0
        t = torch.tensor([sdt], dtype=torch.float64, device=coll_dev or "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sdt = float(t.item())
        srows = shard_rows(eng.launches()) if win is not None else []
        problems += check_shards(srows, [local])
        for r in srows:  # one process per GPU: the rank is the shard
            r["shard"] = rank
        search = (sres, sdt, srows)
        # rank 0's window again, alone, while the other ranks wait at the barrier
        alone = None
        if world > 1:
            barrier()
            if rank == 0 and srows:
                alone = alone_rerun(lambda: gpuhash.Engine([local]), srows[0], sdt,
                                    lambda: torch.cuda.synchronize(dev))
            barrier()
    pci = pci_id(local)
    host = socket.gethostname()
    if search is not None:
        for r in search[2]:
            r["pci"] = pci
            r["host"] = host
    # the north_star's own design -- ONE process, one context over all N GPUs, a host
    # thread + stream per device, 16-byte host argmin -- on the same node: rank 0 repeats
    # the search in-process over devices 0..N-1 while the other ranks wait at the barrier
    # (when every rank has a GPU of its own; a GPUHASH_SHARE_GPU rehearsal repeats ordinal
    # 0), so a torchrun-launched run measures both modes and exercises the in-process path
    # on DISTINCT devices.  A host-side failure here is recorded, not fatal: it must not cost
    # the run its ranks' numbers; a wrong result still fails the run (search_exit)
    inproc = None
    inproc_devs = [0] * world if shared else (list(range(world)) if ndev >= world and not pinned else None)
    if args.search is not None and world > 1 and inproc_devs is not None:
        barrier()
        if rank == 0:
            lo, hi = args.search
            devs = inproc_devs
            try:
                with gpuhash.Engine(devs) as all_eng:
                    # devices 1..N-1 are cold in this process: one small search over the
                    # top of the range (every device gets a shard) loads the scan kernels'
                    # code objects there, so the timed search measures hashing, as the
                    # ranks' (warmed by their timed steps) does
                    all_eng.min(MSG, max(lo, hi - (len(devs) << 24) + 1), hi)
                    t0 = time.perf_counter()
                    ires = all_eng.min(MSG, lo, hi)
                    idt = time.perf_counter() - t0
                    irows = shard_rows(all_eng.launches())
                for r in irows:
                    r["pci"] = pci_id(r["device"])
                iprob = check_shards(irows, devs)
                if not tiles(irows, lo, hi):
                    iprob.append("in-process search: shard windows do not tile the range")
                ipcis = [r["pci"] for r in irows]
                if len(set(devs)) == len(devs) and None not in ipcis and len(set(ipcis)) != len(irows):
                    iprob.append("in-process search: two shards share a PCI device")
                problems += iprob
                inproc = search_line(ires, idt, world, lo, hi, "inproc (rank 0, one context over all GPUs)",
                                     devs, irows)
            except Exception as e:  # noqa: BLE001 -- see above
                inproc = {"error": f"{type(e).__name__}: {e}", "devices": devs}
        barrier()
    gathered = [None] * world
    dist.all_gather_object(gathered, {"rank": rank, "local_rank": local, "pci": pci, "host": host,
                                      "problems": problems, "search_shards": search[2] if search else None})
    if rank == 0:
        value = per_gpu * world * args.steps / dt / 1e9
        out = base_line(args, value, world, dt, cfg["desc"], msg, f"dp{world}", "weak",
                        nonces_per_gpu=per_gpu, processes=world, backend=backend)
        out["result"] = list(res)  # (hash, nonce) argmin over every rank's windows
        out["result_check"] = step_check(msg, merge_windows(w for r in range(world) for w in cfg["windows"](r)), res)
        out["matches_golden"] = out["result_check"]["matches_golden"]
        out["roofline"] = roof
        problems = [f"rank {g['rank']}: {p}" for g in gathered for p in g["problems"]]
        out["rank_devices"] = [{"rank": g["rank"], "device": g["local_rank"], "pci": g["pci"], "host": g["host"]}
                               for g in gathered]
        # distinct GPUs are judged by physical identity, (host, PCI id), not by ordinal: ranks
        # pinned to one visible GPU each all report ordinal 0, and ordinals repeat across the
        # nodes of a multi-node launch
        gpus = [(g["host"], g["pci"]) for g in gathered]
        if not shared and None not in (g["pci"] for g in gathered) and len(set(gpus)) != world:
            problems.append("ranks on distinct GPUs expected but two ranks share a (host, PCI) device")
        if search is not None:
            shards = [s for g in gathered for s in (g["search_shards"] or [])]
            devices = [g["local_rank"] for g in gathered]
            out["search_2p40"] = search_line(search[0], search[1], world, *args.search,
                                             f"ranks ({backend} merge)", devices, shards)
            if alone is not None:
                out["search_2p40"]["scaling"] = alone
            sgpus = [(s.get("host"), s.get("pci")) for s in shards]
            if not shared and None not in (s.get("pci") for s in shards) and len(set(sgpus)) != len(shards):
                problems.append("ranks on distinct GPUs but two search shards share a (host, PCI) device")
            if not tiles(shards, *args.search):
                problems.append("the ranks' search windows do not tile the range")
            if inproc is not None:
                out["search_2p40_inproc"] = inproc
        if problems:
            out["device_check"] = problems
        if world == 1:
            add_cpu_baselines(out, args)
        emit(out)
        summary = distinct_gpu_summary(out)
        if summary:
            print(summary, file=sys.stderr, flush=True)
    eng.close()
    dist.destroy_process_group()
    if rank == 0:
        search_exit(out, problems)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs to drive: under torch.distributed.run it must equal WORLD_SIZE "
                         "(one process per GPU); otherwise ONE process drives devices 0..N-1 "
                         "through one gpuhash context")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--config", default="2", choices=sorted(CONFIGS))
    ap.add_argument("--inproc", default=None, metavar="DEVICES",
                    help="explicit device list for the one-process path (comma list, ordinals "
                         "may repeat to rehearse N shards on one GPU); overrides --gpus")
    ap.add_argument("--search", default="0:2^40-1", metavar="LO:HI|off",
                    help="after the timed steps, one search of 'bradfitz' over [LO, HI] on the "
                         "same devices, checked against the committed CPU golden of that range "
                         "(default: the north_star's 2^40-nonce search; 'off' skips it)")
    ap.add_argument("--no-search", action="store_true", help="same as --search off")
    args = ap.parse_args()
    if args.gpus < 1:
        fail("--gpus must be >= 1")
    try:
        args.search = None if args.no_search else parse_search(args.search)
    except ValueError as e:
        fail(str(e))
    _quiet_stdout()
    # torch before libgpuhash: both link libamdhip64, and the process must load torch's
    # HIP runtime first, or torch later finds "No HIP GPUs are available"
    import torch  # noqa: F401
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None and (int(world_env) > 1 or os.environ.get("GPUHASH_FORCE_DIST") == "1"):
        world = int(world_env)
        if args.inproc is not None:
            fail("--inproc is the one-process path; do not launch it under torch.distributed.run")
        if world != args.gpus:
            fail(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU")
        return main_ranks(args, world, int(os.environ.get("RANK", "0")),
                          int(os.environ.get("LOCAL_RANK", "0")))
    import gpuhash
    visible = gpuhash.device_count()
    if args.inproc is not None:
        devs = [int(x) for x in args.inproc.split(",")]
    else:
        devs = list(range(args.gpus))
    if not devs or max(devs) >= visible or min(devs) < 0:
        fail(f"asked for device(s) {devs} but {visible} HIP device(s) are visible")
    return main_inproc(args, devs)


if __name__ == "__main__":
    main()
