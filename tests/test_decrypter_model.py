"""CPU: the decrypter model (tests/go_decrypter_model.py), the checker of the GPU decrypter fuzz
test, pinned to the reference's own decrypter tests before it is trusted:
* TestNewDecrypterSeekLimit (cipher_test.go:1282-1431): every (offset, limit) of the reference's
  trial grid reads exactly plaintext[offset:offset+limit] on a fresh handle and after RangeSeek on
  one handle, and the open callback gets the reference's (offset, limit) pairs (:1367-1404);
* TestDecrypterRead (cipher_test.go:1485-1560): file16 truncated to every length and with every
  byte flipped gives the reference's error at the reference's point;
and the encrypter model to TestEncryptData (cipher_test.go:1142-1171: file0 / file1 / file16
byte for byte) and TestNewEncrypterErrUnexpectedEOF (:1194-1205: the 32-byte header, then the
reader's io.ErrUnexpectedEOF).
"""
import pytest

from oracle import pyoracle as orc
from rclone_amd import crypt
from rclone_amd.crypt import EOF
from rclone_amd.testdata import random_source
from tests.go_decrypter_model import ModelDecrypter, ModelEncrypter, kind
from tests.go_readers import Buffer, ErrorReader, read_all

ZERO_KEY = bytes(32)


def _opener(ct, calls=None):
    def open_fn(off, lim):
        if calls is not None:
            calls.append((off, lim))
        end = len(ct) if lim < 0 else min(off + lim, len(ct))
        return Buffer(ct[off:end])
    return open_fn


def test_model_seek_limit_grid(ref_kat):
    data_size = 150000
    plain = random_source(data_size)
    ct = orc.encrypt_file(plain, bytes(24), ZERO_KEY)
    trials = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511,
              512, 513, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097, 8191, 8192, 8193, 16383, 16384,
              16385, 32767, 32768, 32769, 65535, 65536, 65537, 131071, 131072, 131073, data_size - 1, data_size]
    limits = [-1, 0, 1, 65535, 65536, 65537, 131071, 131072, 131073]

    def check(fh, offset, limit):
        got, err = read_all(fh)
        assert err is None, (offset, limit, err)
        if limit >= 0:
            assert len(got) == limit, (offset, limit)
        assert got == plain[offset:offset + len(got)], (offset, limit)

    for offset in trials:
        for limit in limits:
            if offset + limit > data_size:
                continue
            check(ModelDecrypter(ZERO_KEY, _opener(ct), offset, limit), offset, limit)
    fh = ModelDecrypter(ZERO_KEY, _opener(ct), 0, -1)
    for offset in trials:
        for limit in limits:
            if offset + limit > data_size:
                continue
            assert fh.range_seek(offset, 0, limit) == (offset, None)
            check(fh, offset, limit)
    for offset, limit, want_off, want_lim in ref_kat["seek_open_callback"]:
        calls = []
        fh = ModelDecrypter(ZERO_KEY, _opener(ct, calls), 0, -1)
        assert fh.range_seek(offset, 0, limit) == (offset, None)
        assert calls == [(0, -1), (want_off, want_lim)], (offset, limit)


def test_model_decrypter_read(ref_kat):
    file16 = bytes.fromhex(ref_kat["file16"])
    for i in range(len(file16) - 1):
        if i < 32:
            with pytest.raises(crypt.ErrorEncryptedFileTooShort):
                ModelDecrypter(ZERO_KEY, _opener(file16[:i]), 0, -1)
            continue
        _, err = read_all(ModelDecrypter(ZERO_KEY, _opener(file16[:i]), 0, -1))
        if i == 32:
            assert err is None
        elif i <= 32 + 16:
            assert kind(err) == "ErrorEncryptedFileBadHeader", i
        else:
            assert kind(err) == "ErrorEncryptedBadBlock", i
    for i in range(len(file16)):
        bad = bytearray(file16)
        bad[i] ^= 0xFF
        if i < 8:
            with pytest.raises(crypt.ErrorEncryptedBadMagic):
                ModelDecrypter(ZERO_KEY, _opener(bytes(bad)), 0, -1)
        else:
            _, err = read_all(ModelDecrypter(ZERO_KEY, _opener(bytes(bad)), 0, -1))
            assert kind(err) == "ErrorEncryptedBadBlock", i
    bad = bytearray(file16)
    bad[-1] ^= 0xFF
    out, err = read_all(ModelDecrypter(ZERO_KEY, _opener(bytes(bad)), 0, -1, pass_bad_blocks=True))
    assert err is None and out == bytes(16)


def test_model_edges():
    # seeking to the end of a whole-block file: fillBuffer reads nothing, RangeSeek returns io.EOF;
    # past the end of a short last block: ErrorBadSeek; whence != io.SeekStart is sticky
    plain = random_source(2 * 65536)
    ct = orc.encrypt_file(plain, bytes(range(24)), ZERO_KEY)
    fh = ModelDecrypter(ZERO_KEY, _opener(ct), 0, -1)
    assert fh.range_seek(2 * 65536, 0, -1) == (0, EOF)
    assert fh.range_seek(5, 0, 3) == (5, None)  # EOF is not sticky for RangeSeek (unFinish)
    assert read_all(fh) == (plain[5:8], None)
    plain = random_source(65536 + 100)
    ct = orc.encrypt_file(plain, bytes(range(24)), ZERO_KEY)
    fh = ModelDecrypter(ZERO_KEY, _opener(ct), 0, -1)
    off, err = fh.range_seek(65536 + 101, 0, -1)
    assert off == 0 and kind(err) == "ErrorBadSeek"
    assert kind(fh.read_go(10)[1]) == "ErrorBadSeek"  # sticky
    fh = ModelDecrypter(ZERO_KEY, _opener(ct), 0, -1)
    off, err = fh.range_seek(1, 1, -1)
    assert kind(err) == "can only seek from the start"
    assert kind(fh.range_seek(1, 0, -1)[1]) == "can only seek from the start"
    assert fh.close() is None and kind(fh.close()) == "ErrorFileClosed"


def test_model_encrypter(ref_kat):
    n0 = bytes(range(1, 25))  # randomSource's first 24 bytes (cipher_test.go:1153)
    for name, plain in (("file0", b""), ("file1", b"\x01"), ("file16", bytes(range(1, 17)))):
        assert read_all(ModelEncrypter(ZERO_KEY, Buffer(plain), n0), 7) == (bytes.fromhex(ref_kat[name]), None), name
    fh = ModelEncrypter(ZERO_KEY, ErrorReader(crypt.ErrUnexpectedEOF("unexpected EOF")), n0)
    out, err = read_all(fh)
    assert len(out) == 32 and kind(err) == "ErrUnexpectedEOF"
