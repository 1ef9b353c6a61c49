"""GPU MD5 of crypt ciphertext (Fs.put's ciphertext hash,
crypt.go:516-533, and cryptcheck's computeHashWithNonce / ComputeHash, crypt.go:784-852).

Checkers: Python's hashlib.md5 (RFC 1321) over the oracle's crypt files, and the committed
config-1 fixture (1000 x 64 KiB objects under password "potato", MD5s generated with
libsodium in the build container -- tests/golden/make_golden.py).
"""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes
from tests.go_readers import Buffer, CloseDetector, ErrorReader, MultiReader, Potato

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MAGIC = b"RCLONE\x00\x00"
MD5_DESC = np.dtype([("off", "<u8"), ("len", "<u8"), ("prefix", "u1", (32,)), ("prefix_len", "<u4"),
                     ("res", "<u4", (3,))])


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_md5_kernel_vs_hashlib():
    from rclone_amd import device
    assert MD5_DESC.itemsize == 64
    lens = list(range(0, 200)) + [1000, 4095, 4096, 65535, 65536, 65584, (1 << 20) + 13]
    data = splitmix64_bytes(3, sum(((n + 15) & ~15) for n in lens) + 64)
    src = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    rows, expect = [], []
    off = 0
    rng = np.random.default_rng(9)
    for i, n in enumerate(lens):
        plen = [0, 16, 32][i % 3]
        pre = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        r = np.zeros(1, dtype=MD5_DESC)
        r["off"], r["len"], r["prefix_len"] = off, n, plen
        r["prefix"][0] = np.frombuffer(pre, dtype=np.uint8)
        rows.append(r)
        expect.append(hashlib.md5(pre[:plen] + data[off:off + n]).digest())
        off += (n + 15) & ~15
    # invalid descriptors: misaligned offset, bad prefix length, out of bounds
    for off_bad, len_bad, plen_bad in ((8, 10, 0), (0, 10, 8), (len(data) - 16, 32, 0)):
        r = np.zeros(1, dtype=MD5_DESC)
        r["off"], r["len"], r["prefix_len"] = off_bad, len_bad, plen_bad
        rows.append(r)
    desc = np.concatenate(rows)
    dig, ok = device.md5_batch(desc, src)
    torch.cuda.synchronize()
    dig, ok = dig.cpu().numpy(), ok.cpu().numpy()
    assert list(ok) == [1] * len(lens) + [0, 0, 0]
    for i in range(len(lens)):
        assert dig[i].tobytes() == expect[i], (i, lens[i])


def _sizes():
    # plaintext sizes whose crypt-file length (32 + n + 16*blocks) hits every MD5 tail case
    out = [0, 1, 15, 16, 31, 32, 33, 63, 64, 65, 65535, 65536, 65537, 3 * 65536 + 7]
    for r in (0, 1, 55, 56, 57, 63):
        n = 100
        while (32 + n + 16) % 64 != r:
            n += 1
        out.append(n)
    return out


def test_hash_batch_with_nonce_vs_oracle():
    from rclone_amd import crypt
    c = crypt.Cipher("", "")
    key = bytes(32)
    items, expect = [], []
    for i, n in enumerate(_sizes()):
        plain = splitmix64_bytes(100 + i, n)
        nonce = splitmix64_bytes(200 + i, 24) if i % 4 else b"\xfd" + b"\xff" * 7 + splitmix64_bytes(i, 16)
        items.append((nonce, Buffer(plain)))
        expect.append(hashlib.md5(orc.encrypt_file(plain, nonce, key)).digest())
    got = c.hash_batch_with_nonce(items)
    assert got == expect


def test_config1_cryptcheck_batch(sodium_vectors):
    # BASELINE configs[0] cryptcheck: all 1000 objects re-encrypted with their nonces and
    # hashed in one GPU batch; must equal the stored (reference-side) ciphertext MD5s
    from rclone_amd import crypt
    cfg = sodium_vectors["config1"]
    c = crypt.Cipher(cfg["password"], cfg["salt"])
    items = [(splitmix64_bytes(cfg["nonce_seed_base"] + i, 24), Buffer(splitmix64_bytes(cfg["plain_seed_base"] + i,
                                                                                       cfg["size"])))
             for i in range(cfg["n"])]
    got = c.hash_batch_with_nonce(items)
    assert [g.hex() for g in got] == cfg["md5"]


def test_hash_errors_pass_through():
    from rclone_amd import crypt
    c = crypt.Cipher("", "")
    key = bytes(32)
    good = splitmix64_bytes(5, 70000)
    n0 = splitmix64_bytes(6, 24)
    potato = Potato()

    class BadClose(Buffer):
        def close(self):
            raise potato

    items = [(n0, Buffer(good)),
             (n0, ErrorReader(potato)),                                     # error before data
             (n0, MultiReader(Buffer(good[:30000]), ErrorReader(potato))),         # data then error
             (n0, ErrorReader(crypt.ErrUnexpectedEOF())),
             (n0, BadClose(good)),                                          # fs.CheckClose error
             (n0, Buffer(good))]
    got = c.hash_batch_with_nonce(items)
    want = hashlib.md5(orc.encrypt_file(good, n0, key)).digest()
    assert got[0] == want and got[5] == want
    assert got[1] is potato and got[2] is potato and got[4] is potato
    assert isinstance(got[3], crypt.ErrUnexpectedEOF)
    # sources are closed (defer fs.CheckClose(in, &err))
    cd = CloseDetector(Buffer(good))
    assert c.hash_batch_with_nonce([(n0, cd)])[0] == want and cd.closed == 1


def test_compute_hash_reads_nonce_from_object():
    # ComputeHash (crypt.go:816): nonce from the encrypted object, re-encrypt src, MD5
    from rclone_amd import crypt
    from tests.go_readers import read_all

    class FixedNonce:
        def __init__(self, n):
            self.n = n

        def read_go(self, k):
            return self.n[:k], None

    c = crypt.Cipher("potato", "")
    plain = splitmix64_bytes(77, 3 * 65536 + 99)
    c.crypto_rand = FixedNonce(splitmix64_bytes(78, 24))
    ct, err = read_all(c.encrypt_data(Buffer(plain)))
    assert err is None
    cd = CloseDetector(Buffer(ct))
    assert c.compute_hash(cd, Buffer(plain)) == hashlib.md5(ct).hexdigest()
    assert cd.closed == 1
    # a different source gives a different hash (what cryptcheck reports as a mismatch)
    assert c.compute_hash(Buffer(ct), Buffer(plain[:-1] + b"\x00")) != hashlib.md5(ct).hexdigest()


def test_put_batch_bodies_and_md5_vs_oracle():
    # xs_engine_put_batch (Fs.put of many whole objects: crypt.go:497-563): wire bodies come
    # back packed (round16 each) and equal the oracle's crypt files minus the header; the MD5s
    # are those of the whole crypt files (the hash crypt.put tees off the ciphertext)
    import ctypes
    from rclone_amd import _lib
    L = _lib.lib()
    key = splitmix64_bytes(77, 32)
    sizes = _sizes() + [2 * 65536, 5 * 65536 + 3, 1 << 20]
    plains = [splitmix64_bytes(300 + i, n) for i, n in enumerate(sizes)]
    nonces = b"".join(splitmix64_bytes(400 + i, 24) if i % 5 else b"\xff" * 8 + splitmix64_bytes(i, 16)
                      for i in range(len(sizes)))
    offs, pos = [], 0
    for n in sizes:
        offs.append(pos)
        pos += (n + 15) & ~15
    stage = bytearray(pos + 16)
    for o, p in zip(offs, plains):
        stage[o:o + len(p)] = p
    n = len(sizes)
    u64s = ctypes.c_uint64 * n
    lens_c, offs_c = u64s(*sizes), u64s(*offs)
    total = L.xs_put_body_bytes(n, lens_c)
    assert total == sum(((n_ + 16 * ((n_ + 65535) // 65536)) + 15) & ~15 for n_ in sizes)
    body = (ctypes.c_uint8 * (total + 16))()
    md5 = (ctypes.c_uint8 * (16 * n))()
    e = L.xs_engine_create(0, 64, 1)
    assert e
    try:
        src = (ctypes.c_uint8 * len(stage)).from_buffer(stage)
        rc = L.xs_engine_put_batch(e, key, n, nonces, offs_c, lens_c, src, body, md5)
        assert rc == 0, _lib.last_error()
    finally:
        L.xs_engine_destroy(e)
    raw, dig = bytes(body), bytes(md5)
    bpos = 0
    for i, p in enumerate(plains):
        want = orc.encrypt_file(p, nonces[24 * i:24 * i + 24], key)
        blen = len(want) - 32
        assert raw[bpos:bpos + blen] == want[32:], (i, sizes[i])
        assert dig[16 * i:16 * i + 16] == hashlib.md5(want).digest(), (i, sizes[i])
        bpos += (blen + 15) & ~15


def test_e2e_sync_harness_small():
    # BASELINE configs[4] shape at 0.25 GiB: local tree -> crypt(memory) sync with the put hash
    # check, cryptcheck, sampled decrypts, corruption caught (tools/e2e_sync.cpp, built by build())
    import json
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tools", "e2e_sync")
    if not os.path.exists(exe):
        pytest.skip("tools/e2e_sync not built")
    shapes = [("batch", "encrypter", "batch"), ("stream", "encrypter", "stream"), ("stream", "reader", "batch")]
    for k, (mode, tee, check) in enumerate(shapes):
        r = subprocess.run([exe, "--gib", "0.25", "--mode", mode, "--transfers", "8", "--group-mib", "64",
                            "--tee", tee, "--check-mode", check, "--checkers", "8",
                            "--dir", "/tmp/rc_e2e_test_%d_%d" % (os.getpid(), k)],
                           capture_output=True, text=True, timeout=100)
        assert r.returncode == 0, r.stdout + r.stderr
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["ok"] and res["cryptcheck_differences"] == 0 and res["corruption_flagged"] == 1
        assert res["put_hash_mismatches"] == 0 and res["check_mode"] == check
