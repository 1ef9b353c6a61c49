"""Randomised operation sequences on the GPU decrypter against the reference's state machine.

Each case encrypts a random-size object with the CPU oracle (sometimes with one block tampered),
opens it through DecryptDataSeek at a random (offset, limit) -- beyond the end included -- and runs
a random sequence of Read (1 byte .. 100 KB), RangeSeek (random offset and limit) and Seek calls
(io.SeekStart, and now and then io.SeekCurrent, which the reference refuses and makes sticky).
The GPU decrypter (librclone_crypt.so through the rc_* C ABI: read-ahead batches, the engine's
ranged opens that decrypt only the 4 KiB groups a limit reaches, pass_bad_blocks) must return,
call by call, the same bytes and the same error as tests/go_decrypter_model.py, the step-by-step
restatement of backend/crypt/cipher.go:776-1087 that tests/test_decrypter_model.py pins to the
reference's own decrypter tests.  Construction errors (the header, a seek past the end) must
match too, and Close must close once.  The encrypter gets the same treatment against
ModelEncrypter.  Both also run from 8 threads at once over the shared engine, and
RCLONE_AMD_FUZZ_SCALE / RCLONE_AMD_FUZZ_SEED turn any of them into a longer soak.
"""
import os
import random

import pytest

from oracle import pyoracle as orc
from rclone_amd import crypt
from rclone_amd.crypt import EOF
from tests.go_decrypter_model import ModelDecrypter, ModelEncrypter, kind
from tests.go_readers import Buffer

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

BLOCK_DATA = 65536
BLOCK_SIZE = 65552
# longer soaks: RCLONE_AMD_FUZZ_SCALE multiplies the case counts, RCLONE_AMD_FUZZ_SEED shifts the seeds
SCALE = int(os.environ.get("RCLONE_AMD_FUZZ_SCALE", "1"))
SEED = int(os.environ.get("RCLONE_AMD_FUZZ_SEED", "0"))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _opener(ct):
    def open_fn(off, lim):
        end = len(ct) if lim < 0 else min(off + lim, len(ct))
        return Buffer(ct[off:end])
    return open_fn


def _size(rng):
    return rng.choice([0, 1, 17, 4096, 65535, 65536, 65537, 131072, 131073, 200000, 5 * 65536 + 4321,
                       rng.randrange(1, 6 * 65536)])


def _offset_limit(rng, size):
    off = rng.choice([0, 0, size, max(size - 1, 0), rng.randrange(0, size + 2), rng.randrange(0, size + 70000),
                      (rng.randrange(0, 7) * BLOCK_DATA)])
    lim = rng.choice([-1, -1, 0, 1, 4096, rng.randrange(0, 200000), max(size - off, 0)])
    return off, lim


def _construct(cls, *a, **kw):
    try:
        return cls(*a, **kw), None
    except crypt.CryptError as e:
        return None, e


def _decrypter_run(rng, ncases, batch):
    """ncases random handles, each with a random call sequence, against the model; (handles, calls)."""
    cases = ops_run = 0
    for case in range(ncases):
        size = _size(rng)
        plain = bytes(rng.getrandbits(8) for _ in range(min(size, 64))) * (size // 64 + 1)
        plain = plain[:size]
        nonce = bytes(rng.getrandbits(8) for _ in range(24))
        if case % 5 == 0:
            nonce = b"\xff" * 8 + nonce[8:]  # block nonces carry past byte 8
        ct = bytearray(orc.encrypt_file(plain, nonce, bytes(32)))
        nblk = (size + BLOCK_DATA - 1) // BLOCK_DATA
        if nblk and rng.random() < 0.3:  # one tampered block: tag or payload byte
            b = rng.randrange(nblk)
            blen = min(BLOCK_SIZE, len(ct) - 32 - b * BLOCK_SIZE)
            ct[32 + b * BLOCK_SIZE + rng.randrange(blen)] ^= 1 << rng.randrange(8)
        ct = bytes(ct)
        pbb = rng.random() < 0.25
        c = crypt.Cipher("", "", batch_blocks=batch, pass_bad_blocks=pbb)
        off, lim = _offset_limit(rng, size)
        model, merr = _construct(ModelDecrypter, bytes(32), _opener(ct), off, lim, pass_bad_blocks=pbb)
        try:
            gpu, gerr = c.decrypt_data_seek(_opener(ct), off, lim), None
        except crypt.CryptError as e:
            gpu, gerr = None, e
        where = f"case {case} size {size} open ({off}, {lim}) pbb {pbb}"
        assert kind(gerr) == kind(merr), (where, gerr, merr)
        cases += 1
        if model is None:
            continue
        for step in range(14):
            r = rng.random()
            if r < 0.6:
                n = rng.choice([1, 7, 4096, 65536, 65537, 100000, rng.randrange(1, 140000)])
                got, gerr = gpu.read_go(n)
                want, merr = model.read_go(n)
                assert (got == want, kind(gerr)) == (True, kind(merr)), (where, step, "read", n, len(got), len(want),
                                                                         gerr, merr)
            elif r < 0.95:
                o, l2 = _offset_limit(rng, size)
                try:
                    gres, gerr = gpu.range_seek(o, 0, l2), None
                except crypt.CryptError as e:
                    gres, gerr = 0, e
                mres, merr = model.range_seek(o, 0, l2)
                assert (gres, kind(gerr)) == (mres, kind(merr)), (where, step, "range_seek", o, l2, gerr, merr)
            else:
                o = rng.randrange(0, size + 2)
                try:
                    gres, gerr = gpu.seek(o, 1), None
                except crypt.CryptError as e:
                    gres, gerr = 0, e
                mres, merr = model.range_seek(o, 1, -1)
                assert (gres, kind(gerr)) == (mres, kind(merr)), (where, step, "seek whence 1", gerr, merr)
            ops_run += 1
        gpu.close()
        assert model.close() is None
        with pytest.raises(crypt.ErrorFileClosed):
            gpu.close()
    return cases, ops_run


@pytest.mark.parametrize("batch", [1, 3, 64])
def test_decrypter_sequences_match_reference(batch):
    cases, ops_run = _decrypter_run(random.Random(0xDEC0 + batch + (SEED << 16)), 400 * SCALE, batch)
    print(f"batch {batch}: {cases} handles, {ops_run} calls matched the reference's state machine")


def test_decrypter_sequences_concurrent():
    """The same sequences from 8 threads at once (rclone's --transfers / multi-thread streams): the
    handles share the device engine, whose coalescing queue and fused ranged opens then serve
    several callers' refills together; every call must still equal its own model's."""
    res = _threads(8, lambda t: _decrypter_run(random.Random(0xC0DE0 + t + (SEED << 16)), 60 * SCALE, (1, 3, 64)[t % 3]))
    print(f"8 threads: {sum(c for c, _ in res.values())} handles, "
          f"{sum(o for _, o in res.values())} calls matched the reference's state machine")


class _ChunkSource:
    """A Go io.Reader over `data` handing out random-size pieces (its own seeded stream, so two
    instances behave alike), ending as `tail` says: "eof" ((0, EOF) after the data), "eof_with_data"
    (the last piece comes with EOF), or an error value returned after the data (and again after)."""

    def __init__(self, data, seed, tail):
        self.data, self.pos, self.rng, self.tail = data, 0, random.Random(seed), tail

    def read_go(self, n):
        if self.pos >= len(self.data):
            return b"", (EOF if self.tail in ("eof", "eof_with_data") else self.tail)
        k = min(n, self.rng.choice([1, 17, 4096, 65536, 70000, self.rng.randrange(1, 100000)]))
        out = self.data[self.pos:self.pos + k]
        self.pos += len(out)
        if self.tail == "eof_with_data" and self.pos >= len(self.data):
            return out, EOF
        return out, None


class _Potato(Exception):
    pass


def _block_rest(pos):
    """Bytes left in the reference encrypter's current buffer (the header, then 65552-byte blocks)
    at stream offset pos: the most one of its Reads returns there."""
    return 32 - pos if pos < 32 else 65552 - (pos - 32) % 65552


def _encrypter_run(rng, ncases, batch):
    """ncases random encrypters read with random sizes against the model; (calls, calls crossing a
    block boundary, calls returning bytes together with the stream's end)."""
    import hashlib
    calls = spans = joint = 0
    for case in range(ncases):
        size = _size(rng)
        plain = bytes(rng.getrandbits(8) for _ in range(min(size, 64))) * (size // 64 + 1)
        plain = plain[:size]
        nonce = bytes(rng.getrandbits(8) for _ in range(24))
        if case % 5 == 0:
            nonce = b"\xff" * 8 + nonce[8:]
        tail = rng.choice(["eof", "eof", "eof_with_data", _Potato("potato"), crypt.ErrUnexpectedEOF("unexpected EOF")])
        seed = rng.getrandbits(32)
        c = crypt.Cipher("", "", batch_blocks=batch)
        gpu = c.encrypt_data(_ChunkSource(plain, seed, tail), nonce=nonce)
        model = ModelEncrypter(bytes(32), _ChunkSource(plain, seed, tail), nonce)
        tee = rng.random() < 0.5
        if tee:
            gpu.set_md5(True)
        got_all = bytearray()
        for step in range(200):
            n = rng.choice([1, 7, 31, 4096, 65552, 70000, rng.randrange(1, 150000)])
            got, gerr = gpu.read_go(n)
            # The reference's Read returns at most the rest of one block per call; the library may hand
            # out several buffered blocks at once (same stream, fewer calls).  The model is read up to
            # the same byte count, and when the library ends the stream the model's next Read must
            # give no bytes and the same error.
            want, merr = b"", None
            while len(want) < len(got) and merr is None:
                d, merr = model.read_go(len(got) - len(want))
                want += d
            if gerr is not None and merr is None:
                d, merr = model.read_go(n)
                want += d
            calls += 1
            spans += len(got) > _block_rest(len(got_all))
            joint += bool(got) and gerr is not None
            assert (got == want, kind(gerr)) == (True, kind(merr)), (case, size, tail, step, n, len(got), len(want),
                                                                     gerr, merr)
            got_all += got
            if merr is not None:
                break
        assert merr is not None, (case, "stream did not end")
        if tee:
            assert gpu.md5() == hashlib.md5(bytes(got_all)).digest(), case
    return calls, spans, joint


@pytest.mark.parametrize("batch", [1, 3, 64])
def test_encrypter_sequences_match_reference(batch):
    """EncryptData (cipher.go:694-758) call by call: random sources (piece sizes, io.EOF alone or
    with the last piece, a reader error or io.ErrUnexpectedEOF after the data), random Read sizes,
    the put tee MD5 on or off; bytes, errors and the tee digest equal the encrypter model's."""
    calls, spans, joint = _encrypter_run(random.Random(0xE9C0 + batch + (SEED << 16)), 300 * SCALE, batch)
    print(f"batch {batch}: {300 * SCALE} encrypters, {calls} calls matched the reference's stream and errors "
          f"({spans} of them crossed a block boundary and {joint} returned bytes with the end, which "
          "the reference's Read never does)")
    assert joint == 0  # bytes and the error of one Read come apart, as the reference's


def _threads(nthreads, fn):
    """fn(t) on nthreads threads at once; {t: result}, any thread's exception re-raised here."""
    import threading
    results, errors = {}, []

    def worker(t):
        try:
            results[t] = fn(t)
        except BaseException as exc:  # noqa: BLE001 -- reported below with its thread
            errors.append((t, repr(exc)[:2000]))
    threads = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors
    assert sorted(results) == list(range(nthreads))
    return results


def test_encrypter_sequences_concurrent():
    """The encrypter sequences from 8 threads at once: seals and tee MD5s of concurrent uploads
    meet in the shared engine and the MD5 workers; every stream, error and digest equal its model's."""
    res = _threads(8, lambda t: _encrypter_run(random.Random(0xC0E0 + t + (SEED << 16)), 40 * SCALE, (1, 3, 64)[t % 3]))
    assert all(j == 0 for _, _, j in res.values())
    print(f"8 threads: {40 * SCALE * 8} encrypters, {sum(c for c, _, _ in res.values())} calls matched the "
          "reference's stream and errors")
