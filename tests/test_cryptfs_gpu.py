"""The crypt overlay's data-path surface (rclone_amd.cryptfs) over a memory remote, on the GPU
cipher: Fs.put with the ciphertext-hash check (crypt.go:497-563), Object.Open with Seek/Range
options (:1050-1088), sizes (:1026, :1168), ComputeHash (:816) and cryptcheck
(cmd/cryptcheck/cryptcheck.go:67-117) -- BASELINE configs[0] end to end: "rclone copy
1000 x 64 KiB random files into crypt(memory), then cryptcheck", bit-exact against the
committed MD5s of the reference-side ciphertext.
"""
import hashlib

import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes
from tests.go_readers import Buffer, read_all

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_config1_copy_then_cryptcheck(sodium_vectors):
    from rclone_amd import crypt
    from rclone_amd.cryptfs import CryptFs, MemoryRemote
    cfg = sodium_vectors["config1"]
    c = crypt.Cipher(cfg["password"], cfg["salt"])
    n = cfg["n"]
    # the nonces the reference run drew from crypto/rand, replayed in order (c.cryptoRand)
    c.crypto_rand = Buffer(b"".join(splitmix64_bytes(cfg["nonce_seed_base"] + i, 24) for i in range(n)))
    mem = MemoryRemote()
    fs = CryptFs(mem, c)
    plains = {f"file{i:04d}": splitmix64_bytes(cfg["plain_seed_base"] + i, cfg["size"]) for i in range(n)}
    for name in sorted(plains):
        fs.put(name, Buffer(plains[name]), len(plains[name]))
    # the wrapped remote holds exactly the reference ciphertext (its MD5s)
    assert [mem.hash(f"file{i:04d}.bin") for i in range(n)] == cfg["md5"]
    assert all(fs.size(k) == cfg["size"] for k in plains)
    res = fs.cryptcheck({k: (lambda v=v: Buffer(v)) for k, v in plains.items()})
    assert res == {"differ": [], "no_hash": [], "errors": {}, "ok": n}
    # the unchanged cryptcheck's shape: 8 checkers, one per-object ComputeHash each
    res = fs.cryptcheck({k: (lambda v=v: Buffer(v)) for k, v in plains.items()}, checkers=8)
    assert res == {"differ": [], "no_hash": [], "errors": {}, "ok": n}
    # a changed source file is reported as differing, and only it
    bad = dict(plains)
    bad["file0042"] = bad["file0042"][:-1] + bytes([bad["file0042"][-1] ^ 1])
    res = fs.cryptcheck({k: (lambda v=v: Buffer(v)) for k, v in bad.items()}, batch=300)
    assert res["differ"] == ["file0042"] and res["ok"] == n - 1 and not res["errors"]
    res = fs.cryptcheck({k: (lambda v=v: Buffer(v)) for k, v in bad.items()}, checkers=8)
    assert res["differ"] == ["file0042"] and res["ok"] == n - 1 and not res["errors"]


def test_open_seek_and_range():
    from rclone_amd import crypt
    from rclone_amd.cryptfs import CryptFs, MemoryRemote, RangeOption, SeekOption
    c = crypt.Cipher("potato", "")
    mem = MemoryRemote()
    fs = CryptFs(mem, c)
    plain = splitmix64_bytes(9, 3 * 65536 + 1234)
    fs.put("obj", Buffer(plain), len(plain))
    cases = [((), 0, None), ((SeekOption(70000),), 70000, None), ((RangeOption(70000, 70100),), 70000, 70101),
             ((RangeOption(-1, 500),), len(plain) - 500, None), ((RangeOption(65536, -1),), 65536, None),
             ((RangeOption(0, 0),), 0, 1), ((RangeOption(131071, 131072),), 131071, 131073)]
    for opts, lo, hi in cases:
        mem.opens.clear()
        data, err = read_all(fs.open("obj", *opts))
        assert err is None
        assert data == plain[lo:hi], opts
        # newDecrypterSeek (cipher.go:821-859): with an offset, open the 32-byte header first,
        # then RangeSeek re-opens at calculateUnderlying's (offset, limit) (cipher.go:935)
        if lo:
            u_off, u_lim, _, _ = crypt.calculate_underlying(lo, (hi - lo) if hi is not None else -1)
            assert len(mem.opens) == 2 and mem.opens[0][1:] == (0, 32)
            usize = len(mem.objects["obj.bin"])
            assert mem.opens[1][1] == u_off
            if u_lim >= 0 and u_off + u_lim - 1 < usize:
                assert mem.opens[1][2] == u_lim
            else:
                assert mem.opens[1][2] == -1
        elif hi is not None:  # offset 0 with a limit: one open of header + underlying limit
            _, u_lim, _, _ = crypt.calculate_underlying(0, hi)
            assert mem.opens == [("obj.bin", 0, 32 + u_lim)]
        else:
            assert mem.opens == [("obj.bin", 0, -1)]


def test_put_detects_corruption_and_removes():
    from rclone_amd import crypt
    from rclone_amd.cryptfs import CryptFs, MemoryRemote

    class Lying(MemoryRemote):
        def hash(self, remote):
            return "0" * 32

    c = crypt.Cipher("", "")
    mem = Lying()
    fs = CryptFs(mem, c)
    with pytest.raises(crypt.CryptError, match="corrupted on transfer"):
        fs.put("x", Buffer(b"hello"), 5)
    assert "x.bin" not in mem.objects
    fs = CryptFs(mem, c, ignore_checksum=True)
    fs.put("x", Buffer(b"hello"), 5)
    assert "x.bin" in mem.objects


def test_put_ciphertext_matches_oracle_and_compute_hash():
    from rclone_amd import crypt
    from rclone_amd.cryptfs import CryptFs, MemoryRemote
    c = crypt.Cipher("", "")
    n0 = b"\xff" * 8 + splitmix64_bytes(1, 16)
    c.crypto_rand = Buffer(n0)
    mem = MemoryRemote()
    fs = CryptFs(mem, c)
    plain = splitmix64_bytes(2, 5 * 65536 - 3)
    assert fs.put("big", Buffer(plain), len(plain)) == n0
    ct = mem.objects["big.bin"]
    assert ct == orc.encrypt_file(plain, n0, bytes(32))
    assert fs.compute_hash("big", Buffer(plain)) == hashlib.md5(ct).hexdigest() == mem.hash("big.bin")
