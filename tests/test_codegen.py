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
    # an explicit output file: objcopy with only an input rewrites it in place
    subprocess.check_call(["objcopy", f"--dump-section=.hip_fatbin={fat}", obj, str(tmp_path / "copy.o")])
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


def pinned_runs(co, kernel):
    """For each straight-line run of >= 500 VALU instructions in the kernel (the per-nonce
    loop bodies, and per-row setup blocks): the address of the instruction after the phase
    pin (`.p2align 3` + `s_nop 0`, scan_kernel.h GPUHASH_LOOP_ALIGN) if the run opens with
    one in its first 10%, else None."""
    d = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", str(co)], text=True)
    i = d.index("<" + kernel)
    j = d.index("s_endpgm", i)
    runs, cur = [], []
    for line in d[i:j].split("\n"):
        m = re.match(r"\s+([vs]_\S+|global_\S+|scratch_\S+|ds_\S+|buffer_\S+|flat_\S+)\s(.*)//\s*([0-9A-Fa-f]+):", line)
        if not m:
            continue
        cur.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
        if m.group(1).startswith(("s_cbranch", "s_branch")):
            runs.append(cur)
            cur = []
    runs.append(cur)
    out = []
    for r in runs:
        if sum(1 for _, op, _ in r if op.startswith("v_")) < 500:
            continue
        pin = None
        for n, (addr, op, args) in enumerate(r[: max(len(r) // 10, 2)]):
            if op == "s_nop" and args == "0" and addr % 8 == 0 and n + 1 < len(r):
                pin = r[n + 1][0]
                break
        out.append(pin)
    return out


def test_hot_loops_start_at_4_mod_8(tmp_path):
    """scan_kernel.h pins the code phase of the per-nonce loop bodies of the plain and
    K+W-table kernels at 4 mod 8 bytes: the identical instruction stream measured ~3.5%
    slower at 0 mod 8.  The pin lands after the loop's first SALU instructions (the
    scheduler moves them above it); everything after it, i.e. the VALU body, is phased."""
    if not (shutil.which("objcopy") and os.path.exists(os.path.join(LLVM, "llvm-objdump"))):
        pytest.skip("binutils / ROCm LLVM tools not present")
    for tu, kernel in [("kernels_plain", "_ZN7gpuhash6k_scanILi4ELi0ELb0ELi0EE"),
                       ("kernels_plain", "_ZN7gpuhash6k_scanILi13ELi0ELb0ELi0EE"),
                       ("kernels_ut", "_ZN7gpuhash6k_scanILi0ELi1ELb0ELi0EE")]:
        obj = os.path.join(PKG, "build", tu + ".o")
        if not os.path.exists(obj):
            subprocess.check_call(["make", "-s", "-C", PKG, f"build/{tu}.o"])
        d = tmp_path / tu
        d.mkdir(exist_ok=True)
        fat, co = d / "fatbin.bin", d / "k.co"
        subprocess.check_call(["objcopy", f"--dump-section=.hip_fatbin={fat}", obj, str(d / "copy.o")])
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        pins = [p for p in pinned_runs(co, kernel) if p is not None]
        assert len(pins) == 1, (tu, kernel, pins)   # exactly the per-nonce loop body
        assert pins[0] % 8 == 4, (tu, kernel, hex(pins[0]))


def test_kernel_source_has_no_tuning_hooks():
    """The measured-negative tuning hooks of round 4 live in tools/tuning_hooks.patch, not
    in the product kernel source: the only conditionals left in
    scan_kernel.h are the loop-phase pin, the tie-test build and the waves-per-SIMD
    attribute the Makefile sets for the plain kernels."""
    src = open(os.path.join(PKG, "csrc", "scan_kernel.h")).read()
    conds = re.findall(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b(.*)$", src, re.M)
    allowed = ("GPUHASH_LOOP_PHASE", "GPUHASH_TIE_TEST_BITS", "GPUHASH_WAVES_PER_EU")
    assert conds and all(any(a in c for a in allowed) for c in conds), conds
    for hook in ("SALU_SIGMA", "FOLD_PLAIN", "FOLD_EX", "FOLD_LT", "EXTRA_SALU", "LT_ALIGN"):
        assert "GPUHASH_" + hook not in src
    patch = open(os.path.join(ROOT, "tools", "tuning_hooks.patch")).read()
    assert all("GPUHASH_" + h in patch for h in ("SALU_SIGMA", "FOLD_PLAIN", "EXTRA_SALU", "LT_ALIGN"))


def test_config2_kernel_code_is_the_measured_one(tmp_path):
    """The config-2 search kernel (J = 4, plain) as profiled in round 4: 64 VGPRs, no
    spills, and a per-nonce loop body of 1,271 instructions (1,196 VALU, 75 SALU; PMC
    counted 1,197.9 VALU per nonce, profiles/r04e_pmc_summary.json).  Removing the tuning
    hooks left the machine code byte-identical; this keeps it from drifting unnoticed."""
    if not (shutil.which("objcopy") and os.path.exists(os.path.join(LLVM, "llvm-objdump"))):
        pytest.skip("binutils / ROCm LLVM tools not present")
    obj = os.path.join(PKG, "build", "kernels_plain.o")
    if not os.path.exists(obj):
        subprocess.check_call(["make", "-s", "-C", PKG, "build/kernels_plain.o"])
    meta = kernel_metadata(obj, tmp_path)
    k4 = [v for n, v in meta.items() if "k_scanILi4ELi0ELb0ELi0E" in n]
    assert k4 == [(64, 0)], k4
    d = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", str(tmp_path / "k.co")], text=True)
    kern = "_ZN7gpuhash6k_scanILi4ELi0ELb0ELi0EE"
    i = d.index("<" + kern)
    body = d[i:d.index("s_endpgm", i)]
    runs, cur = [], []
    for line in body.split("\n"):
        m = re.match(r"\s+([vs]_\S+|global_\S+|scratch_\S+|ds_\S+|buffer_\S+|flat_\S+)\s.*//\s*[0-9A-Fa-f]+:", line)
        if not m:
            continue
        cur.append(m.group(1))
        if m.group(1).startswith(("s_cbranch", "s_branch")):
            runs.append(cur)
            cur = []
    loops = [(len(r), sum(op.startswith("v_") for op in r), sum(op.startswith("s_") for op in r))
             for r in runs if sum(op.startswith("v_") for op in r) >= 500]
    assert loops == [(1271, 1196, 75)], loops
