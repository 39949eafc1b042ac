import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bitcoin-miner_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU and the built HIP library")


@pytest.fixture(scope="session")
def oracle():
    """The C restatement (oracle/hash_oracle.c) -- the checker, never the product."""
    import hash_oracle
    return hash_oracle.load_c_oracle()


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def engine():
    """One gpuhash context on the visible GPU(s) -- the product under test."""
    import gpuhash
    eng = gpuhash.Engine()
    yield eng
    eng.close()
