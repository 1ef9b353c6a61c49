"""CPU checks of the drop-in's native boundary (no GPU):

* include/rclone_crypt_gpu.h compiles as strict C11 (cgo compiles a binding's preamble as C);
* a C11 client shaped like INTEGRATION.md's cgo binding -- handles carried as integers in the
  `user` field, Go callbacks behind C shims -- drives librclone_crypt.so's host-only paths
  (header / magic / short-file errors, reader and opener errors passed through, DecryptDataSeek's
  open arguments, nonce from the random source, sizes, nonce carry, scrypt keys, host name modes);
* the host C++ (cipher.cpp, names.cpp, scrypt.cpp) under AddressSanitizer + UBSan and under
  ThreadSanitizer, with the GPU side replaced by the CPU oracle (tests/native/stub_engine.cpp,
  test-only): stream round trips, truncation / bit-flip / reader-error fuzz with exact error
  positions, a seek/limit grid, name decoders and DecryptFileName on garbage, and concurrent
  streams plus a 16-thread names batch, all under TSan too (the reference runs `go test -race`,
  Makefile:103-104).
"""
import os
import subprocess

import pytest

from rclone_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.fixture(scope="module")
def built():
    _lib.lib()  # librclone_crypt.so, built if stale
    subprocess.check_call(["make", "-s", "-C", NATIVE, "-j4"])
    return os.path.join(NATIVE, "build")


def run(path, *args, timeout=300):
    env = dict(os.environ)
    env.setdefault("ASAN_OPTIONS", "detect_leaks=1")
    env.setdefault("TSAN_OPTIONS", "halt_on_error=1")
    p = subprocess.run([path, *args], capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    return p.stdout


def test_header_is_c11(built):
    assert os.path.exists(os.path.join(built, "header_c11.o"))


def test_c_client_integer_handles(built, ref_kat):
    out = run(os.path.join(built, "c_client"))
    assert "c client ok" in out
    kv = dict(line.split(" ", 1) for line in out.splitlines() if " " in line)
    kat = ref_kat["key_kat"][0]  # TestKey: password "potato", default salt (cipher_test.go:1609-1642)
    assert kat["password"] == "potato" and kat["salt"] == ""
    assert kv["data_key"] == kat["dataKey"]
    assert kv["name_key"] == kat["nameKey"]
    assert kv["name_tweak"] == kat["nameTweak"]


def test_host_cpp_asan_ubsan(built):
    out = run(os.path.join(built, "sanitize_asan"))
    assert "sanitize ok" in out
    assert int(out.split("(")[1].split()[0]) > 10000


def test_host_cpp_tsan(built):
    # every harness check under ThreadSanitizer (concurrent streams, the 16-thread names batch, the
    # MD5 worker tiers, and the single-threaded checks whose code paths those share)
    out = run(os.path.join(built, "sanitize_tsan"), timeout=900)
    assert "sanitize ok" in out
    assert int(out.split("(")[1].split()[0]) > 10000
