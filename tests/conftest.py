import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_10k():
    path = os.path.join(GOLDEN_DIR, "config1_10k.json")
    if not os.path.exists(path):
        pytest.skip("config1_10k.json not generated")
    with open(path) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_edges():
    with open(os.path.join(GOLDEN_DIR, "edges.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_wide():
    with open(os.path.join(GOLDEN_DIR, "wide_sets.json")) as f:
        return json.load(f)


def fromhex(d):
    return {k: float.fromhex(v) for k, v in d.items()}
