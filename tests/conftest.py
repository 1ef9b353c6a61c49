import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")


@pytest.fixture(scope="session")
def ref_kat():
    with open(os.path.join(GOLDEN, "reference_kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def sodium_vectors():
    with open(os.path.join(GOLDEN, "sodium_vectors.json")) as f:
        return json.load(f)
