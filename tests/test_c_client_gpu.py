"""The cgo binding's data path: integration/gpucipher/shim.c sealing, opening, seeking and hashing
through librclone_crypt.so, driven by a C11 client (tests/native/c_client_gpu.c) that plays the Go
side with integer handles exactly as gpucipher.go's //export functions do.

This is the call sequence a Go build of backend/crypt makes in place of
/root/reference/backend/crypt/cipher.go:694-758 (encrypter), :793-927 (decrypter), :972-1039 and
:1112 (RangeSeek / DecryptDataSeek) and crypt.go:516-533 / :784-852 (put's tee MD5,
computeHashWithNonce).  Cases: the reference's own golden files (cipher_test.go:1122-1140: zero
key, nonce 01..18) and the libsodium crypt files of tests/golden/sodium_vectors.json, multi-block
ones with the 192-bit nonce carry included.  Checks:

* the crypt file the encrypter streams out equals the fixture (bytes / sha256), its put tee MD5,
  computeHashWithNonce and the batched hash all equal the fixture's MD5 of the crypt file;
* the client itself checks the decrypt round trip, a DecryptDataSeek window (offset 70000, limit
  50), a RangeSeek on the same handle, and a tampered payload byte / tag -> every byte before the
  bad block, then ErrorEncryptedBadBlock, at exactly that block.

`-m gpu`: the real library on the device, once on one thread and once with 4 threads running
every case at once over the one shared cipher (the Go side's --transfers goroutines calling
through the shim concurrently; every thread's bytes and digests must equal thread 0's).  CPU
suite: the same client over the host C++ with the GPU replaced by the CPU oracle
(tests/native/stub_engine.cpp, test-only), under ASan + UBSan with 3 threads, and under
ThreadSanitizer with 4.
"""
import hashlib
import os
import subprocess

import pytest

from rclone_amd.testdata import pattern_bytes, random_source, splitmix64_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
MAGIC = b"RCLONE\x00\x00"


def _plain(entry):
    if entry["plain"] == "random_source":
        return random_source(entry["size"])
    if entry["plain"] == "pattern":
        return pattern_bytes(entry["size"])
    return splitmix64_bytes(entry["plain_seed"], entry["size"])


def _cases(ref_kat, sodium_vectors, sodium_pick):
    """[(key, [(nonce, plain, expect_crypt_bytes_or_None, expect_sha256, expect_md5)])] groups."""
    n0 = bytes(range(1, 25))
    ref = []
    for name, plain in (("file0", b""), ("file1", b"\x01"), ("file16", bytes(range(1, 17)))):
        want = bytes.fromhex(ref_kat[name])
        ref.append((n0, plain, want, hashlib.sha256(want).hexdigest(), hashlib.md5(want).hexdigest()))
    sod = []
    for i in sodium_pick(sodium_vectors["files"]):
        f = sodium_vectors["files"][i]
        sod.append((bytes.fromhex(f["nonce0"]), _plain(f), None, f["sha256"], f["md5"]))
    return [(bytes(32), ref), (bytes.fromhex(sodium_vectors["key"]), sod)]


def _run_group(exe, tmp_path, tag, key, cases, timeout, threads=1, extra_env=None):
    manifest = tmp_path / f"{tag}.manifest"
    lines = [key.hex()]
    for i, (nonce, plain, *_rest) in enumerate(cases):
        p = tmp_path / f"{tag}_{i}.plain"
        p.write_bytes(plain)
        lines.append(f"{nonce.hex()} {p} {tmp_path / f'{tag}_{i}.crypt'}")
    manifest.write_text("\n".join(lines) + "\n")
    env = dict(os.environ)
    env.setdefault("ASAN_OPTIONS", "detect_leaks=0")
    env.update(extra_env or {})
    r = subprocess.run([exe, str(manifest), str(threads)], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.rstrip().endswith("c client gpu ok")
    if threads > 1:
        assert f"threads {threads} consistent" in r.stdout
    rows = {}
    batch = {}
    for line in r.stdout.splitlines():
        w = line.split()
        if w[0] == "case":
            rows[int(w[1])] = dict(zip(w[2::2], w[3::2]))
        elif w[0] == "batch":
            batch[int(w[1])] = w[2]
    assert sorted(rows) == list(range(len(cases))) and sorted(batch) == list(range(len(cases)))
    for i, (nonce, plain, want, sha, md5) in enumerate(cases):
        got = (tmp_path / f"{tag}_{i}.crypt").read_bytes()
        assert got[:32] == MAGIC + nonce, (tag, i)
        if want is not None:
            assert got == want, (tag, i)
        assert hashlib.sha256(got).hexdigest() == sha, (tag, i, len(plain))
        row = rows[i]
        assert int(row["size"]) == len(plain)
        # put's tee MD5 (crypt.go:516-533), computeHashWithNonce (crypt.go:784-806), batched
        assert row["tee"] == md5 and row["hash"] == md5 and batch[i] == md5, (tag, i)
        nblocks = (len(plain) + 65535) // 65536
        assert int(row["bad_block_at"]) == ((nblocks // 2) * 65536 if nblocks else -1)
        # DecryptDataSeek's opens (cipher.go:821-859, :997-1014): a RangeSeeker (even case) is
        # opened once for the header and moved; a plain reader (odd) is reopened at every seek
        off = (70000 if len(plain) > 70050 else len(plain) // 2)
        seeks = (1 if off else 0) + (1 if len(plain) else 0)
        assert int(row["opens"]) == (1 if i % 2 == 0 else 1 + seeks), (tag, i, row)
    return rows


def _all_multiblock_and_edges(files):
    # every multi-block file (nonce carry ones included) plus the short-length edges
    return [i for i, f in enumerate(files) if f["size"] > 65536 or f["size"] in (0, 1, 16, 17, 65535, 65536)]


@pytest.fixture(scope="module")
def stub_client():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "build/c_client_stub"])
    return os.path.join(NATIVE, "build", "c_client_stub")


def test_shim_data_path_cpu_stub(stub_client, tmp_path, ref_kat, sodium_vectors):
    """The client and the shim's data path on the CPU (oracle engine), ASan + UBSan."""
    pick = lambda files: [i for i, f in enumerate(files)  # noqa: E731
                          if f["plain"] == "splitmix64" and (f["size"] > 131072 or f["size"] in (0, 17, 65536))]
    for tag, (key, cases) in zip(("ref", "sod"), _cases(ref_kat, sodium_vectors, pick)):
        _run_group(stub_client, tmp_path, tag, key, cases, timeout=300, threads=3)


def test_shim_data_path_cpu_stub_tsan(tmp_path, ref_kat, sodium_vectors):
    """The same with 4 client threads under ThreadSanitizer: the shim's handle tables, the shared
    cipher and the per-handle state touched from several threads at once (go test -race's role)."""
    subprocess.check_call(["make", "-s", "-C", NATIVE, "build/c_client_stub_tsan"])
    exe = os.path.join(NATIVE, "build", "c_client_stub_tsan")
    pick = lambda files: [i for i, f in enumerate(files)  # noqa: E731
                          if f["plain"] == "splitmix64" and (f["size"] in (0, 17, 65536, 65537) or f["size"] > 196608)]
    for tag, (key, cases) in zip(("ref", "sod"), _cases(ref_kat, sodium_vectors, pick)):
        _run_group(exe, tmp_path, tag, key, cases, timeout=600, threads=4, extra_env={"TSAN_OPTIONS": "halt_on_error=1"})


@pytest.mark.gpu
def test_shim_data_path_gpu(tmp_path, ref_kat, sodium_vectors):
    """gpucipher_encrypt / decrypt / decrypt_seek / compute_hash / hash_batch on the device."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rclone_amd import _lib
    _lib.lib()  # librclone_crypt.so current (the build id the suite reports)
    subprocess.check_call(["make", "-s", "-C", NATIVE, "build/c_client_gpu"])
    exe = os.path.join(NATIVE, "build", "c_client_gpu")
    for threads in (1, 4):
        for tag, (key, cases) in zip(("ref", "sod"), _cases(ref_kat, sodium_vectors, _all_multiblock_and_edges)):
            rows = _run_group(exe, tmp_path, f"{tag}{threads}", key, cases, timeout=120, threads=threads)
            print(tag, len(rows), "cases through the shim on the GPU,", threads, "thread(s)")
