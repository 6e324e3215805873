import json
import os
import sys

import pytest

# PyTorch's HIP runtime first (charon_amd/_lib.py load_library explains why); no GPU is touched
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libhipbls.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_report_header(config):
    """Which library the run tests: its embedded build id against the tree's sources."""
    from charon_amd import _lib
    path = os.environ.get("HBLS_LIBRARY") or _lib.LIB_PATH
    if not os.path.exists(path):
        return f"libhipbls.so: not built ({path})"
    lib_id, tree = _lib.embedded_build_id(path), _lib.source_build_id()
    return f"libhipbls.so: {lib_id} (tree {tree}: {'match' if tree in lib_id else 'STALE'})"


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "kat_reference.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def fixtures():
    with open(os.path.join(GOLDEN, "fixtures_small.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def hipbls():
    """The GPU implementation (tests marked gpu only)."""
    from charon_amd import tbls
    return tbls.HIPBLS()
