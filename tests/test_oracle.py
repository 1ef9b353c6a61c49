"""Pin the CPU oracle (oracle/xsalsa_oracle.c) before trusting it as the checker.

Against: the reference's own golden vectors (backend/crypt/cipher_test.go), and
libsodium 1.0.18 outputs committed by tests/golden/make_golden.py.
"""
import hashlib

import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import pattern_bytes, random_source, splitmix64_bytes

ZKEY = bytes(32)
N0 = bytes(range(1, 25))


def test_reference_golden_files(ref_kat):
    # TestEncryptData cipher_test.go:1142-1171 with the nonce from randomSource (01..18)
    assert orc.encrypt_file(b"", N0, ZKEY).hex() == ref_kat["file0"]
    assert orc.encrypt_file(b"\x01", N0, ZKEY).hex() == ref_kat["file1"]
    assert orc.encrypt_file(bytes(range(1, 17)), N0, ZKEY).hex() == ref_kat["file16"]
    for name, plain in (("file0", b""), ("file1", b"\x01"), ("file16", bytes(range(1, 17)))):
        out, code, _ = orc.decrypt_file(bytes.fromhex(ref_kat[name]), ZKEY)
        assert code == 0 and out == plain


def test_nonce_tables(ref_kat):
    for row in ref_kat["nonce_increment"]:
        assert orc.nonce_increment(bytes.fromhex(row["in"])).hex() == row["out"]
    for row in ref_kat["nonce_add"]:
        assert orc.nonce_add(bytes.fromhex(row["in"]), row["add"]).hex() == row["out"]


def test_size_tables(ref_kat):
    for n, e in ref_kat["encrypted_size"]:
        assert orc.encrypted_size(n) == e
        assert orc.decrypted_size(e) == n
    codes = {"ErrorEncryptedFileTooShort": -1, "ErrorEncryptedFileBadHeader": -2}
    for n, err in ref_kat["decrypted_size_errors"]:
        assert orc.decrypted_size(n) == codes[err]


def test_calculate_underlying(ref_kat):
    for off, lim, woff, wlim, wdisc, wblocks in ref_kat["calculate_underlying"]:
        assert orc.calculate_underlying(off, lim) == (woff, wlim, wdisc, wblocks)


def test_single_boxes(sodium_vectors):
    key = bytes.fromhex(sodium_vectors["key"])
    nonce = bytes.fromhex(sodium_vectors["nonce"])
    for v in sodium_vectors["single"]:
        msg = splitmix64_bytes(v["msg_seed"], v["len"])
        box = orc.seal(msg, nonce, key)
        assert hashlib.sha256(box).hexdigest() == v["sha256"], v["len"]
        assert box[:16].hex() == v["tag"]
        if "box" in v:
            assert box.hex() == v["box"]
        assert orc.open_box(box, nonce, key) == msg
        bad = bytearray(box)
        bad[len(bad) // 2] ^= 0x40
        assert orc.open_box(bytes(bad), nonce, key) is None


def _plain(entry):
    if entry["plain"] == "random_source":
        return random_source(entry["size"])
    if entry["plain"] == "pattern":
        return pattern_bytes(entry["size"])
    return splitmix64_bytes(entry["plain_seed"], entry["size"])


def test_crypt_files(sodium_vectors):
    key = bytes.fromhex(sodium_vectors["key"])
    for f in sodium_vectors["files"]:
        plain = _plain(f)
        ct = orc.encrypt_file(plain, bytes.fromhex(f["nonce0"]), key)
        assert len(ct) == f["enc_size"]
        assert hashlib.sha256(ct).hexdigest() == f["sha256"], (f["size"], f["plain"])
        out, code, _ = orc.decrypt_file(ct, key)
        assert code == 0 and out == plain


def test_decrypt_errors():
    plain = splitmix64_bytes(1, 3 * 65536 + 5)
    ct = bytearray(orc.encrypt_file(plain, N0, ZKEY))
    ct[32 + 65552 + 100] ^= 1   # corrupt block 1
    out, code, bad = orc.decrypt_file(bytes(ct), ZKEY)
    assert code == -4 and bad == 1
    out, code, _ = orc.decrypt_file(bytes(ct), ZKEY, pass_bad_blocks=True)
    assert code == 0 and out[65536:131072] == bytes(65536) and out[:65536] == plain[:65536]
    assert orc.decrypt_file(bytes(ct[:31]), ZKEY)[1] == -1
    assert orc.decrypt_file(b"RCLONX\0\0" + bytes(ct[8:]), ZKEY)[1] == -2


@pytest.mark.parametrize("n", [0, 1, 65535, 65536, 65537])
def test_seek_table_consistency(n):
    # the open-callback rows of TestNewDecrypterSeekLimit are calculateUnderlying outputs
    assert orc.encrypted_size(n) >= 32
