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


@pytest.mark.parametrize("force,why", [("1", "objectset leg failed"), ("2", "headline tag digest")],
                         ids=["objectset_digest", "headline_digest"])
def test_bench_wrong_result_fails_the_run(force, why):
    # the default line on the GPU with a forced digest mismatch (the objectset leg's, or the
    # headline's expected value): the line still prints, and the run ends non-zero
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, BENCH_FORCE_DIGEST_MISMATCH=force, BENCH_OBJECTSET_BLOCKS="200000")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--warmup-seconds", "0", "--blocks", "100000", "--no-cpu", "--no-pool-check",
                        "--objectset-steps", "1", "--objectset-warmup", "0"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode != 0 and why in r.stderr, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    if force == "1":
        assert res["objectset"]["ok"] is False and res["counters"]["tag_digest_ok"] is True
    else:
        assert res["counters"]["tag_digest_ok"] is False and res["objectset"]["ok"] is True


def test_bench_default_line_pins_and_measurements():
    # a short default run: the headline digest equals the CPU oracle's pin, and the line carries
    # the read-side roofline, the per-rank rows and the power / energy fields
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "4",
                        "--warmup-seconds", "0.5", "--no-cpu", "--no-pool-check", "--objectset-steps", "0"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    c = res["counters"]
    assert c["tag_digest_ok"] is True and c["tag_digest"] == c["tag_digest_expected"]
    ro = res["roofline"]
    assert 0 < ro["read_frac"] < ro["frac"] < 1 and 0 < ro["open"]["read_frac"] < 1
    assert res["per_rank"]["seal_kernel_ms"]["per_rank"][0] > 0
    assert "source" in res["power"]
    if res["power"].get("samples"):
        assert res["energy_J_per_GiB"] > 0
