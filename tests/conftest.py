"""Test configuration: `gpu` marks tests that need an MI355X (HIP device).

CPU tests (-m "not gpu") cover the oracle against golden fixtures, the host
logic of libdlp (loadable and callable without a GPU for host-only entry
points), and the row-block protocol over gloo.  GPU tests call the HIP path
through the C ABI and compare it with the oracle (tests/oracle_py.py)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(TESTS, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950) HIP device")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden
