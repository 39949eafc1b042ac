"""Builds the compiled programs for the CPU tests (test infrastructure).

The miner (bitcoin-miner_amd/csrc/miner_main.cpp) is linked against
oracle/gpuhash_oracle_abi.c, the ABI's entry points on the CPU oracle, so its protocol
and failure handling can be tested without a GPU; the server
(bitcoin-miner_amd/csrc/server_main.cpp) never touches the engine and is built as is.
`san` adds host sanitizers to the program's own code (the reference graders run
`go test -race`; SURVEY 5: sanitizers on the host code stand in for it).
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bitcoin-miner_amd", "csrc")
SAN_MARKERS = ("ThreadSanitizer", "AddressSanitizer", "runtime error:", "LeakSanitizer")
_BUILDS = {}


def _flags(san):
    base = ["-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include")]
    if san is None:
        return ["-O2"] + base
    return ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}", "-fno-sanitize-recover=all"] + base


def build_miner(d, san=None):
    key = ("miner", san)
    if key in _BUILDS:
        return _BUILDS[key]
    tag = (san or "plain").replace(",", "_")
    objs = []
    for src in ("hash_oracle.c", "gpuhash_oracle_abi.c"):
        o = str(d / f"{tag}_{src}.o")
        subprocess.check_call(["gcc", "-O2", "-c", "-I", os.path.join(ROOT, "include"),
                               os.path.join(ROOT, "oracle", src), "-o", o])
        objs.append(o)
    exe = str(d / f"miner_oracle_{tag}")
    subprocess.check_call(["g++", *_flags(san), os.path.join(CSRC, "miner_main.cpp"), *objs, "-lpthread", "-o", exe])
    _BUILDS[key] = exe
    return exe


def build_program(d, name, san=None):
    """csrc/<name>_main.cpp, for the programs that do not call the engine (server, client)."""
    key = (name, san)
    if key in _BUILDS:
        return _BUILDS[key]
    exe = str(d / f"{name}_{(san or 'plain').replace(',', '_')}")
    subprocess.check_call(["g++", *_flags(san), os.path.join(CSRC, f"{name}_main.cpp"), "-lpthread", "-o", exe])
    _BUILDS[key] = exe
    return exe


def build_server(d, san=None):
    return build_program(d, "server", san)


def build_client(d, san=None):
    return build_program(d, "client", san)


class Procs:
    """Started program processes; stops them and keeps their stderr."""

    def __init__(self):
        self.ps, self.errs = [], []

    def start(self, argv, env):
        e = dict(os.environ)
        e.update({k: str(v) for k, v in env.items()})
        p = subprocess.Popen(argv, env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        self.ps.append(p)
        return p

    def stop_all(self):
        for p in self.ps:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(5)
                except subprocess.TimeoutExpired:
                    p.kill()
            try:
                self.errs.append(p.stderr.read() if p.stderr and not p.stderr.closed else "")
            except ValueError:
                pass
            p.wait(10)

    def sanitizer_reports(self):
        return [e for e in self.errs if any(k in e for k in SAN_MARKERS)]
