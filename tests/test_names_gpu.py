"""File-name cipher on the GPU: standard-mode names (EME-AES-256, xs_eme.hip) against the
reference's own vectors (backend/crypt/cipher_test.go:188-683) and against the oracle
(oracle/eme_oracle.c) on random batches with every block count 1..128."""
import ctypes
import json
import os
import random

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd import _lib, crypt, names

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    # torch's HIP runtime must come up before the library's name engine touches the device
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "name_vectors.json")
STD = names.NAME_ENCRYPTION_STANDARD
ENCS = ["base32", "base64", "base32768"]


@pytest.fixture(scope="module")
def nv():
    with open(GOLDEN, encoding="utf-8") as f:
        return json.load(f)


def _c(enc, dir_encrypt=True, password=""):
    c = crypt.new_cipher(STD, password, "", dir_encrypt, names.new_name_encoding(enc))
    return c


@pytest.mark.parametrize("enc", ENCS)
def test_encrypt_segment(nv, enc):
    # testEncryptSegment (:188-205) with TestEncryptSegmentBase32/64/32768
    c = _c(enc)
    for plain, want in nv["segment_" + enc]:
        assert c.encrypt_segment(plain) == want, plain
        assert c.decrypt_segment(want) == plain
        if enc == "base32":
            assert c.decrypt_segment(want.upper()) == plain
    # the same table as one batch (one kernel launch)
    got = c.names_run(names.OP_ENCRYPT_SEGMENT, [p for p, _ in nv["segment_" + enc]]).values
    assert got == [w for _, w in nv["segment_" + enc]]


@pytest.mark.parametrize("enc", ENCS)
def test_decrypt_segment_errors(enc):
    # TestDecryptSegmentBase32/64/32768 (:273-336)
    E = names.new_name_encoding(enc)
    c = _c(enc)
    long_name = {"base32": "a" * 3328, "base64": "a" * 2816, "base32768": "怪" * 1280}[enc]
    first = {"base32": ("64=", names.ErrorBadBase32Encoding()),
             "base64": ("6H=", names.Base64CorruptInputError(2)),
             "base32768": ("怪=", names.Base32768CorruptInputError(1))}[enc]
    bang = {"base32": names.Base32CorruptInputError(0), "base64": names.Base64CorruptInputError(0),
            "base32768": names.Base32768CorruptInputError(0)}[enc]
    cases = [first, ("!", bang), (long_name, names.ErrorTooLongAfterDecode()),
             (E.encode_to_string(b"a"), names.ErrorNotAMultipleOfBlocksize()),
             (E.encode_to_string(b"123456789abcdef"), names.ErrorNotAMultipleOfBlocksize()),
             (E.encode_to_string(b"123456789abcdef0"), names.ErrorPaddingTooLong())]
    for s, want in cases:
        with pytest.raises(names.NameError_) as ex:
            c.decrypt_segment(s)
        assert ex.value == want, s
    # and all of them in one batch
    got = c.names_run(names.OP_DECRYPT_SEGMENT, [s for s, _ in cases]).values
    assert got == [w for _, w in cases]


FILE_NAMES = {
    "base32": ["p0e52nreeaj0a5ea7s64m4j72s", "l42g6771hnv3an9cgc8cr2n1ng", "qgm4avr35m5loi1th53ato71v0"],
    "base64": ["yBxRX25ypgUVyj8MSxJnFw", "qQUDHOGN_jVdLIMQzYrhvA", "1CxFf2Mti1xIPYlGruDh-A"],
    "base32768": ["詮㪗鐮僀伎作㻖㢧⪟", "竢朧䉱虃光塬䟛⣡蓟", "遶㞟鋅缕袡鲅ⵝ蝁ꌟ"],
}
V = "-v2001-02-03-040506-123"


@pytest.mark.parametrize("enc", ENCS)
def test_standard_encrypt_file_name(enc):
    # testStandardEncryptFileName (:338-354) with TestStandardEncryptFileNameBase32/64/32768
    a, b, c3 = FILE_NAMES[enc]
    c = _c(enc)
    cases = [("1", a), ("1/12", f"{a}/{b}"), ("1/12/123", f"{a}/{b}/{c3}"), ("1" + V, a + V),
             ("1/12" + V, f"{a}/{b}{V}")]
    for s, want in cases:
        assert c.encrypt_file_name(s) == want
    assert c.encrypt_file_names([s for s, _ in cases]) == [w for _, w in cases]
    c = _c(enc, False)
    cases = [("1", a), ("1/12", f"1/{b}"), ("1/12/123", f"1/12/{c3}"), ("1" + V, a + V), ("1/12" + V, f"1/{b}{V}")]
    for s, want in cases:
        assert c.encrypt_file_name(s) == want


@pytest.mark.parametrize("enc", ENCS)
def test_standard_decrypt_file_name(enc):
    # testStandardDecryptFileName (:433-458)
    a, b, c3 = FILE_NAMES[enc]
    E = names.new_name_encoding(enc)
    for s, want in [(a, "1"), (f"{a}/{b}", "1/12"), (f"{a}/{b}/{c3}", "1/12/123")]:
        c = _c(enc)
        assert c.decrypt_file_name(s) == want
        if enc == "base32":
            assert c.decrypt_file_name(s.upper()) == want
        with pytest.raises(names.ErrorNotAMultipleOfBlocksize):
            c.decrypt_file_name(E.encode_to_string(b"1") + s)
        no_dir = s
        if "/" in want:
            no_dir = want[:want.rindex("/")] + s[s.rindex("/"):]
        assert _c(enc, False).decrypt_file_name(no_dir) == want


@pytest.mark.parametrize("enc", ENCS)
def test_standard_dir_names(enc):
    # testStandardEncryptDirName (:552-574), testStandardDecryptDirName (:592-663),
    # TestNonStandardEncryptDirName (:576-590)
    a, b, c3 = FILE_NAMES[enc]
    E = names.new_name_encoding(enc)
    rows = [("1", a), ("1/12", f"{a}/{b}"), ("1/12/123", f"{a}/{b}/{c3}")]
    c = _c(enc)
    for plain, ct in rows:
        assert c.encrypt_dir_name(plain) == ct
        assert c.decrypt_dir_name(ct) == plain
        if enc == "base32":
            assert c.decrypt_dir_name(ct.upper()) == plain
        with pytest.raises(names.ErrorNotAMultipleOfBlocksize):
            c.decrypt_dir_name(E.encode_to_string(b"1") + ct)
        c2 = _c(enc, False)
        assert c2.decrypt_dir_name(ct) == ct and c2.decrypt_dir_name(plain) == plain
    assert _c(enc, False).encrypt_dir_name("1/12/123") == "1/12/123"


@pytest.mark.parametrize("enc", ENCS)
def test_enc_dec_matches_standard(enc):
    # TestEncDecMatches (:522-550), standard mode
    c = _c(enc)
    assert c.decrypt_file_name(c.encrypt_file_name("1/2/3/4")) == "1/2/3/4"


def _random_names(rng, n):
    out = []
    for i in range(n):
        if i < 128:
            ln = 16 * i + rng.randrange(16)  # every block count 1..128 (padded)
        else:
            ln = rng.choice([rng.randrange(1, 40), rng.randrange(1, 255), rng.randrange(1, 2032)])
        out.append(bytes(rng.randrange(256) for _ in range(ln)))
    return out


@pytest.mark.parametrize("enc", ENCS)
def test_random_batch_against_oracle(enc):
    rng = random.Random({"base32": 1, "base64": 2, "base32768": 3}[enc])
    c = _c(enc, password="potato")
    key, tweak = c.name_key, c.name_tweak
    E = names.new_name_encoding(enc)
    segs = _random_names(rng, 1500)
    got = c.names_run(names.OP_ENCRYPT_SEGMENT, segs, as_bytes=True).values
    for s, g in zip(segs, got):
        want = E.encode_to_string(orc.eme_transform(key, tweak, orc.pkcs7_pad(s), True))
        assert g.decode("utf-8", "surrogateescape") == want
    back = c.names_run(names.OP_DECRYPT_SEGMENT, got, as_bytes=True).values
    assert back == segs
    # tampered ciphertexts: the unpad verdict of the oracle's decryption
    bad, expect = [], []
    for g in got[:300]:
        raw = bytearray(E.decode_string(g))
        raw[rng.randrange(len(raw))] ^= 1 << rng.randrange(8)
        bad.append(E.encode_to_string(bytes(raw)))
        u = orc.pkcs7_unpad(orc.eme_transform(key, tweak, bytes(raw), False))
        expect.append(u if isinstance(u, bytes) else getattr(names, u)())
    assert c.names_run(names.OP_DECRYPT_SEGMENT, bad, as_bytes=True).values == expect


def test_paths_batch_mixed_errors():
    c = _c("base32", password="potato")
    paths = ["a/b/c.txt", "dir/sub/file-v2001-02-03-040506-123.txt", "x", "", "a//b", "/lead"]
    enc = c.encrypt_file_names(paths)
    assert c.decrypt_file_names(enc) == paths
    # the first failing segment's error wins, later segments are not reported
    bad = [enc[0].replace("/", "/=", 1), "!!!/" + enc[2], enc[2] + "/00", enc[1]]
    got = c.decrypt_file_names(bad)
    assert got[0] == names.Base32CorruptInputError(0)
    assert got[1] == names.Base32CorruptInputError(0)
    assert got[2] == names.ErrorNotAMultipleOfBlocksize()
    assert got[3] == paths[1]


def test_xs_eme_batch_dev_direct():
    L = _lib.lib()
    rng = random.Random(11)
    key, tweak = bytes(rng.randrange(256) for _ in range(32)), bytes(rng.randrange(256) for _ in range(16))
    blocks = [1, 2, 3, 16, 17, 64, 127, 128, 5]
    offs, data = [], bytearray()
    for m in blocks:
        offs.append(len(data))
        data += bytes(rng.randrange(256) for _ in range(16 * m))
        data += bytes(16)  # gap
    desc = np.zeros(len(blocks) + 1, dtype=[("off", "<u8"), ("nblk", "<u4"), ("res", "<u4")])
    for i, (o, m) in enumerate(zip(offs, blocks)):
        desc[i] = (o, m, 0)
    desc[-1] = (len(data) - 16, 2, 0)  # out of range: skipped
    src = torch.tensor(list(data), dtype=torch.uint8, device="cuda")
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    for inplace in (False, True):
        dst = src.clone() if inplace else torch.zeros_like(src)
        s = dst if inplace else src
        rc = L.xs_eme_batch_dev(1, key, tweak, d_desc.data_ptr(), len(desc), s.data_ptr(), dst.data_ptr(),
                                len(data), None)
        _lib.check(rc, "xs_eme_batch_dev")
        torch.cuda.synchronize()
        out = bytes(dst.cpu().numpy())
        for o, m in zip(offs, blocks):
            want = orc.eme_transform(key, tweak, bytes(data[o:o + 16 * m]), True)
            assert out[o:o + 16 * m] == want
        # decrypt back in place
        rc = L.xs_eme_batch_dev(0, key, tweak, d_desc.data_ptr(), len(desc) - 1, dst.data_ptr(), dst.data_ptr(),
                                len(data), None)
        _lib.check(rc, "xs_eme_batch_dev")
        torch.cuda.synchronize()
        back = bytes(dst.cpu().numpy())
        for o, m in zip(offs, blocks):
            assert back[o:o + 16 * m] == bytes(data[o:o + 16 * m])


def test_large_listing_round_trip():
    # a listing-sized batch: 200k names of 1..64 bytes, one launch each way
    rng = np.random.default_rng(12)
    n = 200_000
    lens = rng.integers(1, 65, n)
    pool = rng.integers(ord("a"), ord("z") + 1, int(lens.sum()), dtype=np.uint8).tobytes()
    segs, p = [], 0
    for ln in lens:
        segs.append(pool[p:p + ln])
        p += ln
    c = _c("base32768", password="potato")
    r = c.names_run(names.OP_ENCRYPT_SEGMENT, segs, as_bytes=True)
    assert r.kernel_ms > 0
    back = c.names_run(names.OP_DECRYPT_SEGMENT, r.values, as_bytes=True).values
    assert back == segs
    key, tweak = c.name_key, c.name_tweak
    E = names.new_name_encoding("base32768")
    for i in range(0, n, 9973):
        assert r.values[i].decode() == E.encode_to_string(orc.eme_transform(key, tweak, orc.pkcs7_pad(segs[i]), True))
