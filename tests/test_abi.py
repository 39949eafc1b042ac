"""CPU: the C-ABI library loads, exports every symbol include/gpuhash.h declares, and
its host-only pieces behave (no compute call needs a GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gpuhash.h")
LIB = os.path.join(ROOT, "bitcoin-miner_amd", "lib", "libgpuhash.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "bitcoin-miner_amd"), "-j4",
                               "lib/libgpuhash.so"])
    import gpuhash
    return gpuhash._lib()


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gpuhash_[a-z_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("gpuhash_open", "gpuhash_min", "gpuhash_hash_cpu", "gpuhash_close", "gpuhash_strerror"):
        assert f in fns


def test_library_exports_every_declared_symbol(lib):
    import gpuhash
    fns = declared_functions()
    assert sorted(gpuhash.EXPORTED) == fns
    for f in fns:
        assert hasattr(lib, f), f


def test_exports_are_plain_c(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for f in declared_functions():
        assert f in syms, f  # unmangled extern "C"


def test_strerror_and_version(lib):
    assert lib.gpuhash_strerror(0) == b"ok"
    for rc in (-1, -2, -3, -4, -5):
        assert lib.gpuhash_strerror(rc) != b"unknown gpuhash error"
    assert lib.gpuhash_version().startswith(b"gpuhash ")


def test_hash_cpu_matches_oracle(lib, oracle):
    import gpuhash
    import hash_oracle as ho
    for m, n, h in ho.SPEC_KATS:
        assert gpuhash.Hash(m, n) == h
    for m in (b"", b"bradfitz", b"x" * 55, b"y" * 64, b"z" * 200):
        for n in (0, 9, 10, 999999999, 10 ** 10, (1 << 64) - 1):
            assert gpuhash.Hash(m, n) == oracle.hash(m, n)


def test_invalid_arguments_rejected_before_any_device_work(lib):
    h, n = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.gpuhash_min(None, b"x", 1, 0, 1, ctypes.byref(h), ctypes.byref(n)) == -1
    assert lib.gpuhash_open(None, 0, None) == -1
    assert lib.gpuhash_open(None, -1, ctypes.byref(ctypes.c_void_p())) == -1


def test_message_mirror():
    import gpuhash as g
    r = g.NewRequest("bradfitz", 0, 9999)
    assert (r.Type, r.Data, r.Lower, r.Upper) == (g.MsgType.Request, "bradfitz", 0, 9999)
    assert str(r) == "[Request bradfitz 0 9999]"
    res = g.NewResult(1419516646206828, 9898)
    assert str(res) == "[Result 1419516646206828 9898]"
    assert str(g.NewJoin()) == "[Join]"
    assert res.to_json()["Type"] == 2


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present on this machine")
def test_no_silent_cpu_fallback(lib):
    """Without a gfx950 device the engine refuses to open (no CPU fallback)."""
    import gpuhash
    with pytest.raises(gpuhash.GpuHashError) as e:
        gpuhash.Engine()
    assert e.value.rc == gpuhash.GPUHASH_ENODEV


CLI = os.path.join(ROOT, "bitcoin-miner_amd", "lib", "gpuhash_cli")


def _gpu_visible():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_plain_c_client_links_and_fails_loudly_without_gpu():
    """The C client (the cgo binding's call sequence, no Python in the process) links
    against the in-tree library; with no gfx950 device it exits with the ENODEV error
    instead of computing anything on the host."""
    if not os.path.exists(CLI):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "bitcoin-miner_amd"), "lib/gpuhash_cli"])
    v = subprocess.run([CLI, "--version"], capture_output=True, text=True)
    assert v.returncode == 0 and v.stdout.startswith("gpuhash ")
    assert subprocess.run([CLI, "bradfitz", "5"], capture_output=True).returncode == 2
    assert subprocess.run([CLI, "bradfitz", "-1", "5"], capture_output=True).returncode == 2
    if _gpu_visible():
        pytest.skip("a GPU is visible: the no-device path is not reachable here")
    r = subprocess.run([CLI, "bradfitz", "0", "9999"], capture_output=True, text=True)
    assert r.returncode == 3 and "no usable gfx950" in r.stderr and r.stdout == ""


def _split_args(s: str) -> list[str]:
    """Top-level comma split of a call's argument text."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _calls(src: str, prefix: str):
    """(name, args) of every call `prefix<name>(...)` in src, balanced parentheses."""
    for m in re.finditer(re.escape(prefix) + r"(gpuhash_[a-z_]+)\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        yield m.group(1), _split_args(src[m.end():i - 1])


def test_go_binding_matches_the_header():
    # The cgo binding (integration/go) cannot be compiled here (no Go toolchain), so
    # check it against include/gpuhash.h: every C.<name> it uses is declared, and every
    # call passes as many arguments as the prototype takes.
    hdr = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = {}
    for name, args in _calls(hdr, ""):
        protos.setdefault(name, 0 if args == ["void"] else len(args))
    go_dir = os.path.join(ROOT, "integration", "go")
    srcs = [open(os.path.join(d, f)).read() for d, _, fs in os.walk(go_dir) for f in fs if f.endswith(".go")]
    assert srcs
    used = set()
    for src in srcs:
        used |= set(re.findall(r"\bC\.(gpuhash_\w+|GPUHASH_\w+)", src))
        for name, args in _calls(src, "C."):
            assert name in protos, name
            assert len(args) == protos[name], (name, args, protos[name])
    for ident in used:
        if ident.startswith("GPUHASH_"):
            assert re.search(r"\b" + ident + r"\b", hdr), ident
        elif ident not in protos:  # a type, e.g. gpuhash_ctx
            assert re.search(r"typedef\s+struct\s+" + ident + r"\b", hdr), ident
    assert {"gpuhash_open", "gpuhash_min", "gpuhash_close"} <= used


def test_ctypes_structs_match_the_header(tmp_path):
    """gpuhash.Stats / gpuhash.LaunchRecord lay out exactly like the header's structs (a C
    program compiled against include/gpuhash.h prints sizeof/offsetof): a field added to
    the header without the mirror -- or in another order -- would shift every later field
    the bench and the tests read."""
    import ctypes
    import subprocess
    import gpuhash
    fields = {"gpuhash_stats": [f for f, _ in gpuhash.Stats._fields_],
              "gpuhash_launch_record": [f for f, _ in gpuhash.LaunchRecord._fields_]}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "gpuhash.h"', "int main(void) {"]
    for st, fs in fields.items():
        src.append(f'  printf("{st} %zu\\n", sizeof({st}));')
        for f in fs:
            src.append(f'  printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    src += ["  return 0;", "}"]
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src) + "\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)])
    got = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)], text=True).splitlines())
    for st, cls in (("gpuhash_stats", gpuhash.Stats), ("gpuhash_launch_record", gpuhash.LaunchRecord)):
        assert int(got[st]) == ctypes.sizeof(cls), st
        for f, _ in cls._fields_:
            assert int(got[f"{st}.{f}"]) == getattr(cls, f).offset, (st, f)
