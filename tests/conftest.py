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
