"""Test helpers: host-side evidence for the multi-process system tests.

  CgroupSampler   samples the cgroup v2 cpu.stat (CPU used, CFS throttling) every 0.25 s
  proc_cpu        CPU seconds (user + sys, all threads) a live process has used
  lsp_lateness    the worst epoch lateness the LSP endpoints reported under LSP_DIAG=1
                  (lsp/endpoint.py, csrc/lsp_native.h), per role
  write_diag      a JSON record under $GPUHASH_DIAG_DIR (the GPU runs set it to gpurun_out/)
"""
from __future__ import annotations

import json
import os
import re
import threading
import time

CPU_STAT = "/sys/fs/cgroup/cpu.stat"


def _cpu_stat() -> dict:
    try:
        with open(CPU_STAT) as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return {}


class CgroupSampler(threading.Thread):
    """usage_usec / throttled_usec / nr_throttled of this job's cgroup, every `period` s."""

    def __init__(self, period: float = 0.25):
        super().__init__(daemon=True)
        self.period = period
        self.samples: list[tuple[float, dict]] = []
        self._halt = threading.Event()

    def run(self) -> None:
        while not self._halt.is_set():
            self.samples.append((time.monotonic(), _cpu_stat()))
            self._halt.wait(self.period)

    def stop(self) -> dict:
        self._halt.set()
        self.join(5)
        self.samples.append((time.monotonic(), _cpu_stat()))
        return self.summary()

    def summary(self) -> dict:
        s = [(t, d) for t, d in self.samples if d]
        if len(s) < 2:
            return {"available": False}
        (t0, a), (t1, b) = s[0], s[-1]
        wall = t1 - t0
        worst_cpus, worst_thr = 0.0, 0.0
        for (ta, x), (tb, y) in zip(s, s[1:]):
            dt = tb - ta
            if dt <= 0:
                continue
            worst_cpus = max(worst_cpus, (y.get("usage_usec", 0) - x.get("usage_usec", 0)) / 1e6 / dt)
            worst_thr = max(worst_thr, (y.get("throttled_usec", 0) - x.get("throttled_usec", 0)) / 1e3)
        return {"available": True, "wall_s": round(wall, 2),
                "cpus_used_avg": round((b.get("usage_usec", 0) - a.get("usage_usec", 0)) / 1e6 / wall, 2),
                "cpus_used_max_window": round(worst_cpus, 2),
                "throttled_ms": round((b.get("throttled_usec", 0) - a.get("throttled_usec", 0)) / 1e3, 1),
                "throttled_ms_max_window": round(worst_thr, 1),
                "nr_throttled": b.get("nr_throttled", 0) - a.get("nr_throttled", 0),
                "nr_periods": b.get("nr_periods", 0) - a.get("nr_periods", 0),
                "window_s": self.period}


def proc_cpu(pid: int) -> float | None:
    """utime + stime (seconds) of a live process, every thread included; None if gone."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            st = f.read()
        f_ = st[st.rindex(")") + 2:].split()
        return (int(f_[11]) + int(f_[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError):
        return None


_LATE = re.compile(r"(lsp-\w+)\[(\d+)\]: (?:epoch fired (\d+) ms late|window max lateness ([\d.]+) ms, run max ([\d.]+) ms)")


def lsp_lateness(texts: dict[str, str]) -> dict:
    """{label: stderr text} -> per label the worst epoch lateness (ms) its LSP loops
    reported, and the lines of epochs that fired more than one epoch late."""
    out = {}
    for label, text in texts.items():
        worst, late_lines = 0.0, []
        for m in _LATE.finditer(text or ""):
            if m.group(3) is not None:
                worst = max(worst, float(m.group(3)))
                late_lines.append(m.group(0))
            else:
                worst = max(worst, float(m.group(5)))
        out[label] = {"max_late_ms": worst, "late_epochs": late_lines[:20]}
    return out


def write_diag(name: str, obj: dict) -> str | None:
    d = os.environ.get("GPUHASH_DIAG_DIR")
    if not d:
        return None
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, name)
    with open(p, "w") as f:
        json.dump(obj, f, indent=1)
    return p
