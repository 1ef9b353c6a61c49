"""bench.py's secondary modes at small sizes: each run checks its own results (configs[2] mixed
objects: exact failing set + zero-fill + bytes; configs[3] object set: round trip + digest;
file names: encrypt/decrypt round trip) and must print one JSON line.  The default mode runs
at round end on its own, so it is not repeated here."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1", *args],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_mixed_objects_mode():
    res = _bench("--mixed-gib", "0.25")
    assert res["counters"]["verified"] is True
    assert res["counters"]["tag_failures_last_step"] == res["config"]["tampered_blocks"] >= 3
    assert res["value"] > 0 and res["roofline"]["kernel"] == "xs_open"


def test_bench_object_set_mode():
    res = _bench("--object-blocks", "20000", "--blocks", "8192", "--no-cpu")
    assert res["counters"]["blocks"] == 20000 and res["counters"]["tag_failures"] == 0
    assert res["counters"]["roundtrip_mismatch_words"] == 0


def test_bench_names_mode():
    res = _bench("--names", "20000", "--no-cpu")
    assert res["unit"] == "names/s" and res["value"] > 0
    assert res["kernel"]["segments_per_launch"] == 20000
