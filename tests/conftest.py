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


def tableau_sha256(sessions, width, chunk=512):
    """sha256 of a row-block tableau in global row order: every rank's constraint
    rows (first `width` doubles each), then the objective row (replicated: every
    rank's must be identical) — the stream tests/golden/make_digests.py hashes
    for the oracle's tableau (c3_tableau)."""
    import hashlib

    import numpy as np
    h = hashlib.sha256()
    for s in sorted(sessions, key=lambda s: s.row_first):
        for first in range(0, s.rows, chunk):
            cnt = min(chunk, s.rows - first)
            h.update(np.ascontiguousarray(s.read_rows(first, cnt)[:, :width]).tobytes())
    objs = [np.ascontiguousarray(s.read_rows(s.rows, 1)[0, :width]).tobytes() for s in sessions]
    assert all(o == objs[0] for o in objs), "replicated objective rows differ between ranks"
    h.update(objs[0])
    return h.hexdigest()
