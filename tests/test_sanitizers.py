"""CPU: the host-side planner under AddressSanitizer + UndefinedBehaviorSanitizer.

The reference's graders run its Go tests under `go test -race` (README.md:179-188); the
analogue for this build's host code is a sanitizer pass.  plan.cpp does all the index
arithmetic that shapes a search (digit groups, lane/loop splits, midstates, descriptor
words), so tests/test_plan.py -- planner tiling plus the per-variant CPU replay against the
oracle -- is rerun in a subprocess against libgpuhash_hostcheck_asan.so (same sources,
-fsanitize=address,undefined, no recovery) with libasan preloaded into the interpreter.
GPU-side sanitizers are not available on this pool; device code is covered by the GPU
parity suite instead.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bitcoin-miner_amd")
ASAN_LIB = os.path.join(PKG, "lib", "libgpuhash_hostcheck_asan.so")


def _runtime(name):
    try:
        p = subprocess.check_output(["gcc", f"-print-file-name={name}"], text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_planner_under_asan_ubsan():
    libasan = _runtime("libasan.so")
    if libasan is None:
        pytest.skip("gcc's libasan runtime is not installed")
    subprocess.check_call(["make", "-s", "-C", PKG, "lib/libgpuhash_hostcheck_asan.so"])
    env = dict(os.environ)
    env.update(GPUHASH_HOSTCHECK_LIB=ASAN_LIB, LD_PRELOAD=libasan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_plan.py")],
                       env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
