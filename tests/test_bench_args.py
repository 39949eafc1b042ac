"""CPU: bench.py's mode selection.  `--gpus N` either drives N
devices or exits non-zero; it never silently measures one GPU.  No GPU here, so every
N >= 1 without torchrun must be refused with the visible-device count, and a torchrun
launch whose WORLD_SIZE differs from --gpus must be refused too.  Also the per-device
summary / roofline helpers the in-process path reports, on synthetic launch records."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, env=env, timeout=120)


def test_gpus_n_above_visible_devices_is_refused():
    sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd"))
    import gpuhash
    visible = gpuhash.device_count()  # 0 here; the test also holds on a GPU box
    for n in (visible + 1, visible + 2, 8 + visible):
        r = _run(["--gpus", str(n), "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
        assert r.returncode == 2, r.stderr
        assert "HIP device(s) are visible" in r.stderr
        assert r.stdout == ""  # no bench line


def test_gpus_zero_is_refused():
    r = _run(["--gpus", "0"])
    assert r.returncode == 2 and "--gpus must be >= 1" in r.stderr


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_inproc_under_torchrun_is_refused():
    r = _run(["--gpus", "2", "--inproc", "0,0"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "--inproc" in r.stderr


def _rec(dev, J, nonces, ms, c=1, C2=0, EX=0):
    return {"device": dev, "J": J, "C2": C2, "EX": EX, "digits": 10, "c": c,
            "nonces": nonces, "ms": ms, "sclk_mhz": 2400.0}


def test_per_device_picks_the_slowest_shard():
    recs = [_rec(0, 4, 4_000_000_000, 120.0), _rec(0, 3, 1000, 0.05),
            _rec(1, 4, 4_000_000_000, 125.0),
            _rec(0, 4, 4_000_000_000, 121.0), _rec(1, 4, 4_000_000_000, 124.0)]
    rows, slow, slow_recs = bench.per_device(recs, steps=2)
    assert slow == 1 and len(slow_recs) == 2
    assert [r["device"] for r in rows] == [0, 1]
    assert rows[0]["nonces_per_step"] == 4_000_000_500
    assert rows[1]["kernel_ms_per_step"] == pytest.approx(124.5)


def test_roofline_of_the_dominant_kernel(monkeypatch):
    monkeypatch.setattr(bench, "pmc_source", lambda cfg, key, cycles=None: (None, {"used": False}))
    recs = [_rec(0, 4, 1 << 32, 123.0), _rec(0, 2, 10**6, 5.0)]
    r = bench.roofline("2", recs)
    assert r["kernel"] == "k_scan<J=4,C2=0,EX=0,MODE=0>"
    want = (1 << 32) * bench.OPS_PER_BLOCK / 0.123 / 1e12
    assert r["achieved"] == pytest.approx(want, rel=1e-3)
    assert r["frac"] == pytest.approx(want / bench.VALU_PEAK_T, rel=1e-3)
    assert r["traffic"] is None and r["issued_frac"] is None
