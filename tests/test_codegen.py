"""CPU: code-generation properties the measured performance depends on.

The plain-layout scan kernels (config 2 and config 4 run on them) are issue-bound, and
their rate rests on 8 resident waves per SIMD: <= 64 VGPRs, and no scratch spills in the
per-nonce loop.  That follows from computing each schedule word just before the round that
reads it (scan_kernel.h) plus -DGPUHASH_WAVES_PER_EU=8 (Makefile).  A source change that
lengthens live ranges would silently bring back spills (7 GB of scratch traffic per config
2 launch, measured) or drop occupancy; this reads the gfx950 code object's metadata from
the build and fails instead.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bitcoin-miner_amd")
LLVM = "/opt/rocm/lib/llvm/bin"


def kernel_metadata(obj, tmp_path):
    fat = tmp_path / "fatbin.bin"
    co = tmp_path / "k.co"
    subprocess.check_call(["objcopy", f"--dump-section=.hip_fatbin={fat}", obj])
    subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                           f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)], text=True)
    out = {}
    for block in notes.split("  - .")[1:]:
        name = re.search(r"\.name:\s+(\S+)", block)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", block)
        sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", block)
        if name and vg and sp:
            out[name.group(1)] = (int(vg.group(1)), int(sp.group(1)))
    return out


def test_plain_scan_kernels_fit_8_waves(tmp_path):
    if not (shutil.which("objcopy") and os.path.exists(os.path.join(LLVM, "llvm-readelf"))):
        pytest.skip("binutils / ROCm LLVM tools not present")
    obj = os.path.join(PKG, "build", "kernels_plain.o")
    if not os.path.exists(obj):
        subprocess.check_call(["make", "-s", "-C", PKG, "build/kernels_plain.o"])
    meta = kernel_metadata(obj, tmp_path)
    scans = {}
    for name, v in meta.items():
        m = re.search(r"k_scanILi(\d+)ELi0ELb0ELi0E", name)  # MODE 0 = the search kernels
        if m:
            scans[int(m.group(1))] = v
    assert sorted(scans) == list(range(14)), scans
    for J, (vgpr, spill) in scans.items():
        assert vgpr <= 64, (J, vgpr)        # 512 / 64 = 8 waves per SIMD
        assert spill <= 4, (J, spill)       # at most a handful of cold values
    assert scans[4][1] == 0 and scans[5][1] == 0, scans  # the config 2 / config 4 kernels
