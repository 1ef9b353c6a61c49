"""One object past 4 GiB through the stream API (the maximum-size edge of cipher.go's encrypter /
decrypter, cipher.go:681-1039): 5 GiB + 12 345 bytes = 81 921 blocks, so

* the block nonce carries out of its low two bytes (block 65 536 onwards, nonce.add, cipher.go:660-678),
* plaintext and wire offsets pass 2^32 (calculateUnderlying / RangeSeek, cipher.go:935-1039),
* the encrypter's tee MD5 hashes more than 2^32 bytes (crypt.go:516-533: the length word's high half),
* the object ends in a ragged block.

The plaintext is SplitMix64 blocks generated on the fly (never held whole); the wire is kept in
host memory (~5 GiB) for the decrypt legs.  Checks: blocks either side of each carry and the
ragged last block against the oracle's secretbox, the whole-wire MD5 against hashlib and the
encrypter's tee, the full decrypt against the generator, ranged reads that start, end and
straddle 2^32 against the generator, and a tampered block past 4 GiB (error at that block,
zeros under pass_bad_blocks).  Sizes: RCLONE_AMD_BIG_OBJECT_BYTES overrides the default.
"""
import hashlib
import os

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

BLOCK = 65536
WIRE_BLOCK = BLOCK + 16
HEADER = 32
SEED = 0xB16B0B
SIZE = int(os.environ.get("RCLONE_AMD_BIG_OBJECT_BYTES", str(5 * 2**30 + 12345)))
CHUNK = 4 << 20


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _block(b):
    from rclone_amd.testdata import splitmix64_block
    return splitmix64_block(SEED, b)


def expected(off, n):
    """Plaintext bytes [off, off + n) of the object."""
    n = max(0, min(n, SIZE - off))
    out, pos = [], off
    while pos < off + n:
        b, o = divmod(pos, BLOCK)
        take = min(off + n - pos, BLOCK - o)
        out.append(_block(b)[o:o + take])
        pos += take
    return b"".join(out)


class BlockSource:
    """io.Reader of the object's plaintext, one 64 KiB block generated at a time."""

    def __init__(self):
        self.pos, self.cur, self.data = 0, -1, b""

    def read_go(self, n):
        from rclone_amd.crypt import EOF
        if self.pos >= SIZE:
            return b"", EOF
        out, want = [], min(n, SIZE - self.pos)
        while want:
            b, o = divmod(self.pos, BLOCK)
            if b != self.cur:
                self.cur, self.data = b, _block(b)
            take = min(want, BLOCK - o)
            out.append(self.data[o:o + take])
            self.pos += take
            want -= take
        return b"".join(out), None


class MemReader:
    """bytes.Reader over a slice of the wire (no copy of the whole)."""

    def __init__(self, mv):
        self.mv, self.pos = mv, 0

    def read_go(self, n):
        from rclone_amd.crypt import EOF
        if self.pos >= len(self.mv):
            return b"", EOF
        d = bytes(self.mv[self.pos:self.pos + n])
        self.pos += len(d)
        return d, None


@pytest.fixture(scope="module")
def big():
    from oracle import pyoracle as orc
    from rclone_amd import crypt
    from rclone_amd.testdata import splitmix64_bytes
    c = crypt.Cipher("big object", "salt")
    # nonces count little-endian: block 65 536 carries out of byte 1 through bytes 2..7 into byte 8
    nonce = bytes(2) + b"\xff" * 6 + splitmix64_bytes(99, 16)
    wsize = orc.encrypted_size(SIZE)
    wire = bytearray(wsize)
    enc = c.encrypt_data(BlockSource(), nonce)
    enc.set_md5(True)
    h = hashlib.md5()
    pos = 0
    while True:
        d, err = enc.read_go(CHUNK)
        if d:
            wire[pos:pos + len(d)] = d
            h.update(d)
            pos += len(d)
        if err is not None:
            assert err is crypt.EOF, err
            break
    assert pos == wsize
    assert enc.md5() == h.digest()
    return {"c": c, "nonce": nonce, "wire": wire, "key": c.data_key}


def test_big_object_blocks_vs_oracle(big):
    from oracle import pyoracle as orc
    nblk = (SIZE + BLOCK - 1) // BLOCK
    wire, nonce, key = big["wire"], big["nonce"], big["key"]
    assert bytes(wire[8:HEADER]) == nonce
    picks = sorted({0, 1, 255, 256, 65535, 65536, 65537, (2**32 // BLOCK) - 1, 2**32 // BLOCK, nblk - 2, nblk - 1}
                   & set(range(nblk)))
    for b in picks:
        plain = expected(b * BLOCK, BLOCK)
        w0 = HEADER + b * WIRE_BLOCK
        got = bytes(wire[w0:w0 + len(plain) + 16])
        assert got == orc.seal(plain, orc.nonce_add(nonce, b), key), b
    # the last block is ragged
    assert SIZE % BLOCK == 0 or len(wire) - (HEADER + (nblk - 1) * WIRE_BLOCK) == SIZE % BLOCK + 16


def test_big_object_full_decrypt(big):
    from rclone_amd import crypt
    d = big["c"].decrypt_data(MemReader(memoryview(big["wire"])))
    pos = 0
    while True:
        data, err = d.read_go(CHUNK)
        if data:
            assert data == expected(pos, len(data)), pos
            pos += len(data)
        if err is not None:
            assert err is crypt.EOF, (pos, err)
            break
    assert pos == SIZE


def _open_fn(wire):
    mv = memoryview(wire)

    def open_fn(off, lim):
        end = len(wire) if lim < 0 else min(off + lim, len(wire))
        return MemReader(mv[off:end])
    return open_fn


def _read(rc, n):
    from rclone_amd import crypt
    got = bytearray()
    while len(got) < n:
        d, e = rc.read_go(min(CHUNK, n - len(got)))
        got += d
        if e is not None:
            assert e is crypt.EOF, e
            break
    return bytes(got)


def test_big_object_ranged_reads_across_4gib(big):
    if SIZE <= 2**32 + 3 * BLOCK:
        pytest.skip("object smaller than 4 GiB (RCLONE_AMD_BIG_OBJECT_BYTES)")
    c, open_fn = big["c"], _open_fn(big["wire"])
    cases = [(2**32 - 5, 10), (2**32, 1), (2**32 - BLOCK, 2 * BLOCK + 3), (2**32 + 3 * BLOCK + 7, 70000),
             (65535 * BLOCK - 1, 3), (65536 * BLOCK, BLOCK), (SIZE - 100, -1), (SIZE - 12345, 12345), (SIZE, -1)]
    for off, lim in cases:
        want = expected(off, (SIZE - off) if lim < 0 else lim)
        rc = c.decrypt_data_seek(open_fn, off, lim)
        assert _read(rc, len(want) + 1) == want, (off, lim)
    fh = c.decrypt_data_seek(open_fn, 0, -1)
    for off, lim in cases:
        want = expected(off, (SIZE - off) if lim < 0 else lim)
        assert fh.range_seek(off, 0, lim) == off
        assert _read(fh, len(want) + 1) == want, ("range_seek", off, lim)


def test_big_object_bad_block_past_4gib(big):
    from rclone_amd import crypt
    nblk = (SIZE + BLOCK - 1) // BLOCK
    bad = min(nblk - 2, 2**32 // BLOCK + 4)
    wire = big["wire"]
    at = HEADER + bad * WIRE_BLOCK + 16 + 1000
    wire[at] ^= 0x01
    try:
        open_fn = _open_fn(wire)
        start = (bad - 1) * BLOCK
        rc = big["c"].decrypt_data_seek(open_fn, start, 3 * BLOCK)
        got = bytearray()
        err = None
        while True:
            d, err = rc.read_go(CHUNK)
            got += d
            if err is not None:
                break
        assert isinstance(err, crypt.ErrorEncryptedBadBlock), err
        assert bytes(got) == expected(start, BLOCK)
        pb = crypt.Cipher("big object", "salt", pass_bad_blocks=True)
        rc = pb.decrypt_data_seek(open_fn, start, 3 * BLOCK)
        want = expected(start, BLOCK) + bytes(BLOCK) + expected(start + 2 * BLOCK, BLOCK)
        assert _read(rc, 3 * BLOCK + 1) == want
    finally:
        wire[at] ^= 0x01
