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
    assert r["target_frac"] == 0.70 and r["target_met"] is (r["frac"] >= 0.70)


def test_roofline_charges_an_extra_block_layout_two_compressions(monkeypatch):
    """an EX launch (message length 44-53 mod 64 at 10-12 digits) has
    c = 1 nonce-bearing block but compresses the constant padding block per nonce too."""
    monkeypatch.setattr(bench, "pmc_source", lambda cfg, key, cycles=None: (None, {"used": False}))
    recs = [_rec(0, 13, 1 << 30, 51.7, c=1, EX=1)]  # 20.77 GH/s
    r = bench.roofline("2", recs)
    assert r["kernel"] == "k_scan<J=13,C2=0,EX=1,MODE=0>"
    assert (r["compressions_per_nonce"], r["ops_per_nonce"], r["ops_per_nonce_c_based"]) == (
        2, 2 * bench.OPS_PER_BLOCK, bench.OPS_PER_BLOCK)
    want = (1 << 30) * 2 * bench.OPS_PER_BLOCK / 0.0517 / 1e12
    assert r["achieved"] == pytest.approx(want, rel=1e-3)
    assert 0.70 < r["frac"] < 0.75  # at the c-based count it read 0.36
    import gpuhash
    assert gpuhash.compressions_per_nonce({"c": 2, "EX": 0}) == 2
    assert gpuhash.compressions_per_nonce({"c": 1, "EX": 0}) == 1


# ---- the 2^40 search leg ----

def _srec(shard, dev, lo, hi, ms, stream_dev=None, J=4):
    return {"device": dev, "shard": shard, "stream_device": dev if stream_dev is None else stream_dev,
            "J": J, "C2": 0, "EX": 0, "digits": 10, "c": 1, "lo": lo, "hi": hi,
            "nonces": hi - lo + 1, "ms": ms, "sclk_mhz": 2400.0}


def test_search_range_parsing():
    assert bench.parse_search("0:2^40-1") == (0, (1 << 40) - 1)
    assert bench.parse_search("5:4294967295") == (5, (1 << 32) - 1)
    assert bench.parse_search("off") is None
    for bad in ("9:3", "0:2^64", "-1:5"):
        with pytest.raises(ValueError):
            bench.parse_search(bad)
    r = _run(["--search", "9:3"])
    assert r.returncode == 2 and "LO <= HI" in r.stderr


def test_search_golden_is_the_committed_2p40_fixture():
    """The default search range is exactly config 4's golden range, so every bench line's
    search_2p40 is checked against oracle/golden_scan.c's [0, 2^40) result."""
    want, name = bench.golden_for(bench.MSG, *bench.SEARCH_DEFAULT)
    assert name == "cfg4_bradfitz_2p40" and want == (16555811, 890536971553)
    assert bench.golden_for(bench.MSG, 0, (1 << 32) - 1)[1] == "cfg2_bradfitz_2p32"
    assert bench.golden_for(b"nope", 0, 1) == (None, None)
    line = bench.search_line((16555811, 890536971553), 4.0, 8, *bench.SEARCH_DEFAULT, "inproc",
                             list(range(8)), [])
    assert line["matches_golden"] is True and line["GHs"] == pytest.approx((1 << 40) / 4e9, rel=1e-4)
    assert line["per_gpu_GHs"] == pytest.approx(line["GHs"] / 8, rel=1e-3)
    bad = bench.search_line((16555811, 890536971554), 4.0, 8, *bench.SEARCH_DEFAULT, "inproc", [0], [])
    assert bad["matches_golden"] is False
    with pytest.raises(SystemExit) as e:
        bench.search_exit({"search_2p40": bad}, [])
    assert e.value.code == 3


def test_shard_rows_and_device_checks():
    # 2 shards on devices 3 and 5, two slices each, two kernel groups in the second slice
    # (their records carry the slice's window and the nonces of their own group)
    g1, g2 = _srec(0, 3, 200, 299, 1.0), _srec(0, 3, 200, 299, 0.5, J=3)
    g1["nonces"], g2["nonces"] = 60, 40
    g2["sclk_mhz"] = 2100.0
    recs = [_srec(0, 3, 0, 99, 1.0), _srec(1, 5, 100, 199, 1.5), g1, g2, _srec(1, 5, 300, 399, 1.0)]
    rows = bench.shard_rows(recs)
    assert [(r["shard"], r["device"], r["windows"], r["slices"], r["nonces"]) for r in rows] == \
        [(0, 3, [[0, 99], [200, 299]], 2, 200), (1, 5, [[100, 199], [300, 399]], 2, 200)]
    assert bench.tiles(rows, 0, 399) and not bench.tiles(rows, 0, 400) and not bench.tiles(rows[:1], 0, 299)
    assert rows[0]["kernel_ms"] == pytest.approx(2.5)
    assert rows[0]["nonces_hashed"] == 200 and rows[0]["kernel_GHs"] == round(200 / 2.5e-3 / 1e9, 4)
    assert rows[0]["sclk_mhz"] == pytest.approx((2400 * 2.0 + 2100 * 0.5) / 2.5, abs=0.1)
    assert bench.check_shards(rows, [3, 5]) == []
    assert bench.check_shards(rows, [5, 3])  # shard 0 did not run on the listed device
    # a stream the runtime placed on another device is caught
    rows2 = bench.shard_rows([_srec(0, 3, 0, 9, 1.0, stream_dev=0), _srec(1, 5, 10, 19, 1.0)])
    assert any("stream" in p for p in bench.check_shards(rows2, [3, 5]))
    # distinct devices requested, but two shards report the same one
    rows3 = bench.shard_rows([_srec(0, 3, 0, 9, 1.0), _srec(1, 3, 10, 19, 1.0)])
    assert bench.check_shards(rows3, [3, 3]) == []  # a rehearsal on one GPU: allowed
    assert any("share" in p for p in bench.check_shards(rows3, [3, 4]))


def test_host_cpus_reports_the_usable_share():
    h = bench.host_cpus()
    assert h["nproc"] >= h["affinity"] >= h["usable"] >= 1
    if h["cgroup_quota_cpus"] is not None:
        assert h["usable"] <= max(1, int(h["cgroup_quota_cpus"]))


def test_shard_rates_over_repeated_steps():
    """K timed steps search the same window K times: the shard's rate is K x the window's
    nonces over the K steps' kernel time, not the window once over it (VERDICT r04 weak 5:
    BENCH_r04 printed 1.74 GH/s for a 34.7 GH/s shard)."""
    recs = [_srec(0, 0, 0, (1 << 32) - 1, 123.7) for _ in range(20)]
    (row,) = bench.shard_rows(recs)
    assert row["nonces"] == 1 << 32 and row["nonces_hashed"] == 20 << 32
    assert row["kernel_GHs"] == pytest.approx((1 << 32) / 0.1237 / 1e9, rel=1e-3)
    pd, _, _ = bench.per_device(recs, steps=20)
    assert pd[0]["kernel_GHs"] == row["kernel_GHs"]


def test_timed_step_is_checked_against_the_goldens():
    """the headline step's (hash, nonce) is compared with the golden of
    exactly its windows, and a mismatch exits 3 after the line."""
    c = bench.step_check(bench.MSG, [(0, (1 << 32) - 1)], (5256245051, 1626825724))
    assert c["matches_golden"] is True and c["golden_names"] == ["cfg2_bradfitz_2p32"]
    bad = bench.step_check(bench.MSG, [(0, (1 << 32) - 1)], (5256245051, 1626825725))
    assert bad["matches_golden"] is False
    with pytest.raises(SystemExit) as e:
        bench.search_exit({"matches_golden": False, "result": [5256245051, 1626825725], "result_check": bad}, [])
    assert e.value.code == 3
    # config 3: the min over both windows' goldens
    w3 = bench.CONFIGS["3"]["windows"](0)
    c3 = bench.step_check(bench.M120, w3, (0, 0))
    assert c3["golden_names"] and len(c3["golden_names"]) == 2 and c3["matches_golden"] is False
    assert bench.step_check(bench.M120, w3, tuple(c3["golden"]))["matches_golden"] is True
    # config 2's timed step at N = 2, 4, 8 GPUs ([0, N * 2^32)) has a golden since round 5;
    # N = 3 does not: skipped, and says why
    for n in (2, 4, 8):
        merged = bench.merge_windows(w for r in range(n) for w in bench.CONFIGS["2"]["windows"](r))
        assert bench.step_check(bench.MSG, merged, (0, 0))["golden_names"] == [f"cfg2_bradfitz_{n}gpu"]
    assert bench.step_check(bench.MSG, [(0, (1 << 37) - 1)], (0, 0))["golden_names"] == ["cfg4_bradfitz_2p37"]
    sk = bench.step_check(bench.MSG, [(0, (3 << 32) - 1)], (1, 2))
    assert sk["matches_golden"] is None and "no committed golden" in sk["reason"]
    bench.search_exit({"matches_golden": None}, [])  # a skipped check does not fail the run


def test_merge_windows():
    assert bench.merge_windows([(5, 9), (0, 4), (20, 30)]) == [(0, 9), (20, 30)]
    assert bench.merge_windows(w for r in range(3) for w in bench.CONFIGS["2"]["windows"](r)) == \
        [(0, (3 << 32) - 1)]


def test_alone_rerun_reports_scaling_efficiency():
    """shard 0's window(s) searched again alone; efficiency = t_alone /
    t_all, with the alone run's clock."""
    import time as _t

    class Eng:
        def __init__(self):
            self.calls, self.closed = [], False

        def min(self, msg, lo, hi):
            self.calls.append((lo, hi))
            _t.sleep(0.05)
            return (1, lo)

        def launches(self):
            lo, hi = self.calls[-1]
            return [_srec(0, 0, lo, hi, 50.0)]

        def close(self):
            self.closed = True

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            self.close()

    eng = Eng()
    row = {"shard": 0, "device": 0, "windows": [[0, 99], [200, 299]]}
    s = bench.alone_rerun(lambda: eng, row, 0.3, lambda: None)
    # one untimed warm-up call on the fresh context, then the windows
    assert eng.calls == [(0, 99), (0, 99), (200, 299)] and eng.closed
    assert 0.1 <= s["t_alone_s"] < 0.15 and s["scaling_efficiency"] == pytest.approx(s["t_alone_s"] / 0.3, rel=1e-2)
    assert s["alone_sclk_mhz"] == 2400.0


def test_alone_rerun_closes_the_engine_when_a_call_fails():
    class Eng:
        closed = False

        def min(self, msg, lo, hi):
            raise RuntimeError("device lost")

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            Eng.closed = True

    s = bench.alone_rerun(Eng, {"shard": 0, "device": 0, "windows": [[0, 9]]}, 1.0, lambda: None)
    assert s["error"] == "RuntimeError: device lost" and Eng.closed


def test_distinct_gpu_summary():
    rows = [{"device": 0, "pci": "0000:10:00", "host": "n1", "kernel_GHs": 34.6, "sclk_mhz": 2365.0},
            {"device": 1, "pci": "0000:20:00", "host": "n1", "kernel_GHs": 34.5, "sclk_mhz": 2360.0}]
    out = {"search_2p40": {"shards": rows, "scaling": {"scaling_efficiency": 0.991}}}
    line = bench.distinct_gpu_summary(out)
    assert line.startswith("bench.py: 2 distinct GPUs (search_2p40): gpu 0 [n1/0000:10:00] 34.6 GH/s @ 2365.0 MHz")
    assert line.endswith("scaling_efficiency 0.991")
    same = [dict(r, pci="0000:10:00", device=0) for r in rows]  # shards on one GPU: no line
    assert bench.distinct_gpu_summary({"search_2p40": {"shards": same}}) is None
    assert bench.distinct_gpu_summary({"shards": [{"device": 0}, {"device": 0}]}) is None


def test_alone_rerun_records_a_failure_instead_of_raising():
    """Under torchrun the other ranks wait at a barrier while rank 0 re-runs its window: a
    host-side exception there must not end rank 0 (the others would hang), so it is
    recorded, like the in-process repeat's."""
    def boom():
        raise RuntimeError("no device")
    s = bench.alone_rerun(boom, {"shard": 0, "device": 0, "windows": [[0, 9]]}, 1.0, lambda: None)
    assert s["error"] == "RuntimeError: no device" and "scaling_efficiency" not in s
