"""CPU baselines of the drop-in's host paths, built and checked on the
CPU: the configs[4] harness (tools/e2e_sync.cpp) and the ranged-read latency tool
(tools/seek_latency.cpp) over the same host C++ (cipher.cpp, names.cpp), with the engine ABI on host
cores (tests/native/cpu_engine.cpp over the vectorised oracle, oracle/xsalsa_simd.c).  These are
measurement legs beside the GPU numbers, never a product path: nothing
in rclone_amd/ links them.  Here they run small, and their stored objects are checked against the
scalar oracle's crypt files (sync -> crypt(memory) -> cryptcheck, crypt.go:497-563, :784-852)."""
import hashlib
import json
import os
import subprocess

import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "-j4", "build/e2e_sync_cpu", "build/seek_latency_cpu"])
    return os.path.join(NATIVE, "build")


def test_cpu_engine_not_in_the_product():
    for f in os.listdir(os.path.join(ROOT, "rclone_amd", "csrc")):
        src = open(os.path.join(ROOT, "rclone_amd", "csrc", f), errors="replace").read()
        assert "cpu_engine" not in src and "orc_simd" not in src, f


@pytest.mark.parametrize("shape", [["--lanes", "4", "--transfers", "16"],
                                   ["--mode", "stream", "--transfers", "4", "--check-mode", "stream", "--checkers", "8"]],
                         ids=["batch", "stream"])
def test_e2e_cpu_baseline_small(built, tmp_path, shape):
    anchor = str(tmp_path / "anchor.jsonl")
    tee_all = str(tmp_path / "tee_all.txt")
    r = subprocess.run([os.path.join(built, "e2e_sync_cpu"), "--gib", "0.15", "--dir", str(tmp_path / "tree"),
                        "--anchor", anchor, "--tee-all", tee_all] + shape, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["engine"] == "cpu" and res["ok"] and res["corruption_flagged"] == 1
    assert res["put_hash_mismatches"] == 0 and res["cryptcheck_differences"] == 0 and res["verify_failures"] == 0
    key = hashlib.scrypt(b"potato", salt=bytes.fromhex("a80df43a8fbd0308a7cab83e581f86b1"), n=16384, r=8, p=1,
                         maxmem=2**26, dklen=80)[:32]
    rows = [json.loads(x) for x in open(anchor)]
    assert len(rows) >= 60
    for row in rows:
        ct = orc.encrypt_file(splitmix64_bytes(row["seed"], row["size"]), bytes.fromhex(row["nonce"]), key)
        assert hashlib.sha256(ct).hexdigest() == row["sha256"], row
        assert hashlib.md5(ct).hexdigest() == row["tee_md5"], row
    from tests.e2e_oracle import verify_tee_all
    n, _, bad = verify_tee_all(tee_all, key)
    assert n == res["objects"] == res["tee_listed"] and bad == []


def test_seek_latency_cpu_small(built):
    r = subprocess.run([os.path.join(built, "seek_latency_cpu"), "--mib", "16", "--reads", "300", "--len", "4096",
                        "--threads", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["bad"] == 0 and res["reads"] == 300 and res["p50_us"] > 0


def test_open_window_matches_the_scalar_oracle():
    # the windowed open the CPU engine uses for ranged reads: bytes [lo, hi) exact, the rest untouched,
    # at every SIMD level the host has
    import ctypes
    L = orc.lib()
    key, n = splitmix64_bytes(1, 32), splitmix64_bytes(2, 24)
    try:
        for level in range(L.orc_simd_level(), 0, -1):
            L.orc_simd_force(level)
            for ln in (1, 33, 4096, 65504, 65536):
                p = splitmix64_bytes(ln, ln)
                box = orc.seal(p, n, key)
                for lo, hi in ((0, ln), (ln - 1, ln), (31, 33), (1000, 5096), (4064, 8160), (ln // 2, ln)):
                    lo, hi = min(lo, ln), min(hi, ln)
                    out = ctypes.create_string_buffer(b"\xee" * ln, ln)
                    assert L.orc_simd_open_window(out, box, len(box), n, key, lo, hi) == 0
                    assert out.raw[lo:hi] == p[lo:hi] and out.raw[:lo] == b"\xee" * lo, (level, ln, lo, hi)
                    assert out.raw[hi:] == b"\xee" * (ln - hi), (level, ln, lo, hi)
                bad = bytearray(box)
                bad[-1] ^= 1
                assert L.orc_simd_open_window(out, bytes(bad), len(box), n, key, 0, 1) == -1
    finally:
        L.orc_simd_force(-1)
