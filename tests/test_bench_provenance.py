"""CPU: bench.py only reports PMC-derived roofline fields (traffic, issued rate) from a
committed profile collected on the library build it is running (gpuhash_version's
build id, a hash of the library's sources); a stale profile yields nulls, not numbers."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import gpuhash  # noqa: E402

KEY = (4, 0, False)
KNAME = "k_scan<4, 0, false, 0>"


@pytest.fixture
def profile(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setitem(bench.PMC_SUMMARY, "2", "x_pmc_summary.json")

    def write(build_id, cycles=None):
        e = {"per_launch": {"SQ_INSTS_VALU": 1000.0}, "hbm_bytes_per_launch": 4096.0}
        if cycles is not None:
            e["gpu_cycles_per_launch"] = cycles
        (prof / "x_pmc_summary.json").write_text(json.dumps({"tag": "x", "build_id": build_id,
                                                             "kernels": {KNAME: e}}))
    return write


def test_build_id_is_a_source_hash():
    bid = gpuhash.build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0


def test_matching_build_is_used(profile):
    profile(gpuhash.build_id())
    e, prov = bench.pmc_source("2", KEY)
    assert prov["used"] and prov["build_id"] == prov["library_build_id"]
    assert bench.pmc_traffic(e) == 4096.0 and bench.pmc_issued(e) == 1000.0


@pytest.mark.parametrize("stale", [None, "0000000000000000"])
def test_stale_or_unstamped_profile_gives_nulls(profile, stale):
    profile(stale)
    e, prov = bench.pmc_source("2", KEY)
    assert e is None and not prov["used"] and "different build" in prov["reason"]
    assert bench.pmc_traffic(e) is None and bench.pmc_issued(e) is None


def test_profile_of_another_launch_size_gives_nulls(profile):
    # per-launch counters of a 2.9e8-cycle launch must not be divided by the nonces of a
    # launch 6x longer (an --inproc rehearsal, a non-default range)
    profile(gpuhash.build_id(), cycles=2.9e8)
    e, prov = bench.pmc_source("2", KEY, launch_cycles=2.9e8 * 0.97)  # profiled clocks lower
    assert prov["used"] and bench.pmc_issued(e) == 1000.0
    e, prov = bench.pmc_source("2", KEY, launch_cycles=2.9e8 * 6.7)
    assert e is None and not prov["used"] and "another size" in prov["reason"]
    assert bench.pmc_traffic(e) is None and bench.pmc_issued(e) is None


def test_config_without_profile(profile):
    e, prov = bench.pmc_source("4", KEY)
    assert e is None and not prov["used"]


def test_peak_is_the_guides_simd32_rate():
    # 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md): nothing issues above it
    assert bench.VALU_PEAK_T == pytest.approx(78.643, abs=1e-3)
    assert bench.SURVEY_PEAK_T == pytest.approx(39.322, abs=1e-3)
