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


@pytest.fixture(scope="session")
def fullsize():
    """The CPU oracle's pins of the full-size workloads (tests/golden/make_fullsize.py)."""
    with open(os.path.join(GOLDEN, "fullsize.json")) as f:
        return json.load(f)


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Name the native library the run loaded (its build id = sha256 of the sources it was built
    from, rclone_amd/build.py), last in the output so a log's tail carries it."""
    try:
        from rclone_amd import _lib
        if _lib._lib is not None:
            terminalreporter.write_line("rclone_amd library build id: " + _lib.build_id())
    except Exception as exc:  # noqa: BLE001 -- never fail the run over the report line
        terminalreporter.write_line(f"rclone_amd library build id unavailable: {exc}")
