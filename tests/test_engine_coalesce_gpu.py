"""Cross-caller coalescing in the host engine (§8(f) rank 2: many concurrent transfers):
concurrent xs_engine_seal / xs_engine_open calls are packed into combined GPU batches, and
every caller must get exactly the bytes / ok flags of a separate call -- checked against the
oracle (cipher.go:737 per block, nonce0 + first_block + i) with two keys, carry-edge nonces,
first_block offsets, partial last blocks and tampered blocks."""
import ctypes
import threading

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rclone_amd import _lib
    L = _lib.lib()
    e = L.xs_engine_create(0, 64, 3)
    assert e
    yield L, e
    L.xs_engine_destroy(e)


def _stats(L, e):
    out = (ctypes.c_uint64 * 3)()
    L.xs_engine_stats(e, out)
    return tuple(out)


def _seal_expected(plain, nonce0, first, key):
    out = []
    for j in range(0, max(1, (len(plain) + 65535) // 65536)):
        chunk = plain[j * 65536:(j + 1) * 65536]
        if not chunk:
            break
        out.append(orc.seal(chunk, orc.nonce_add(nonce0, first + j), key))
    return b"".join(out)


class _Pinned:
    """xs_host_alloc'd buffer (page-locked, device-mapped): the engine's zero-copy path."""

    def __init__(self, L, data_or_len):
        self.L = L
        n = data_or_len if isinstance(data_or_len, int) else len(data_or_len)
        self.n = n
        self.p = L.xs_host_alloc(max(n, 1))
        assert self.p
        if not isinstance(data_or_len, int):
            ctypes.memmove(self.p, bytes(data_or_len), n)

    @property
    def raw(self):
        return ctypes.string_at(self.p, self.n)

    def __del__(self):
        self.L.xs_host_free(self.p)


def _run(L, e, nthreads=12, calls=8, pinned=False):
    keys = [splitmix64_bytes(1, 32), splitmix64_bytes(2, 32)]
    errors = []
    start = threading.Barrier(nthreads)

    def worker(t):
        try:
            cases = []  # everything but the engine calls is prepared before the start line
            for i in range(calls):
                key = keys[(t + i) % 2]
                n = [1, 100, 65536, 65537, 3 * 65536 - 5, 200000][(t * 3 + i) % 6]
                plain = splitmix64_bytes(1000 * t + i, n)
                nonce0 = b"\xfe" + b"\xff" * 7 + splitmix64_bytes(t, 16) if i % 3 == 0 else splitmix64_bytes(7 * t + i, 24)
                first = [0, 1, 255, 1 << 33][i % 4]
                nb = (n + 65535) // 65536
                want = _seal_expected(plain, nonce0, first, key)
                wire = bytearray(want)
                bad = set()
                if i % 2 and nb > 1:
                    wire[65552 + 5] ^= 1  # a tag byte of block 1
                    bad.add(1)
                exp = bytearray(plain)
                for j in bad:
                    exp[j * 65536:(j + 1) * 65536] = bytes(len(exp[j * 65536:(j + 1) * 65536]))
                if pinned:
                    bufs = (_Pinned(L, plain), _Pinned(L, n + 16 * nb), _Pinned(L, wire), _Pinned(L, n))
                else:
                    bufs = (plain, ctypes.create_string_buffer(n + 16 * nb), bytes(wire), ctypes.create_string_buffer(n))
                cases.append((key, n, nonce0, first, nb, want, bad, bytes(exp), bufs))
            ptr = (lambda b: b.p) if pinned else (lambda b: b)
            start.wait()
            for i, (key, n, nonce0, first, nb, want, bad, exp, (src, body, win, out)) in enumerate(cases):
                assert L.xs_engine_seal(e, key, nonce0, first, ptr(src), n, ptr(body)) == 0
                assert body.raw == want, (t, i, n)
                ok = (ctypes.c_uint8 * nb)()
                assert L.xs_engine_open(e, key, nonce0, first, ptr(win), len(want), ptr(out), ok) == 0
                assert [j for j in range(nb) if not ok[j]] == sorted(bad), (t, i)
                assert out.raw == exp, (t, i)
        except BaseException as ex:  # noqa: BLE001
            errors.append((t, repr(ex)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:3]
    return nthreads * calls * 2


def test_coalesced_engine_matches_oracle(eng):
    L, e = eng
    L.xs_engine_set_coalesce(e, 1)
    b0, r0, k0 = _stats(L, e)
    ncalls = _run(L, e)
    b1, r1, k1 = _stats(L, e)
    assert r1 - r0 == ncalls               # every call went through the coalescer


def test_uncoalesced_engine_matches_oracle(eng):
    L, e = eng
    L.xs_engine_set_coalesce(e, 0)
    before = _stats(L, e)
    _run(L, e, nthreads=4, calls=6)
    assert _stats(L, e) == before
    L.xs_engine_set_coalesce(e, 1)


def test_coalesced_engine_zero_copy_pinned(eng):
    # pinned caller buffers: combined batches hand the callers' own memory to the kernels
    # (keygen reads the descriptors from pinned host memory, crypt reads/writes over PCIe)
    L, e = eng
    L.xs_engine_set_coalesce(e, 1)
    b0, r0, _ = _stats(L, e)
    ncalls = _run(L, e, pinned=True)
    b1, r1, _ = _stats(L, e)
    assert r1 - r0 == ncalls


@pytest.mark.parametrize("pinned", [False, True])
def test_concurrent_requests_share_batches(eng, pinned):
    # A combined batch holds one (direction, key) run: 12 threads sealing 5-block objects (above
    # the express lanes' 4) under one key queue behind the leader, so batches must be shared.
    # (_run's mixed keys and directions need not coalesce: each batch is one run.)
    L, e = eng
    L.xs_engine_set_coalesce(e, 1)
    key, nthreads, calls, n = splitmix64_bytes(3, 32), 12, 6, 5 * 65536
    start = threading.Barrier(nthreads)
    errors = []

    def worker(t):
        try:
            jobs = []
            for i in range(calls):
                plain = splitmix64_bytes(77 * t + i, n)
                nonce0 = splitmix64_bytes(91 * t + i, 24)
                want = _seal_expected(plain, nonce0, 0, key)
                bufs = (_Pinned(L, plain), _Pinned(L, len(want))) if pinned else \
                    (plain, ctypes.create_string_buffer(len(want)))
                jobs.append((nonce0, want, bufs))
            ptr = (lambda b: b.p) if pinned else (lambda b: b)
            start.wait()
            # back to back (the comparisons after): calls overlap instead of queueing on the GIL
            rcs = [L.xs_engine_seal(e, key, nonce0, 0, ptr(src), n, ptr(body)) for nonce0, _, (src, body) in jobs]
            assert rcs == [0] * calls
            for nonce0, want, (src, body) in jobs:
                assert body.raw == want
        except BaseException as ex:  # noqa: BLE001
            errors.append((t, repr(ex)))

    b0, r0, _ = _stats(L, e)
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:3]
    b1, r1, _ = _stats(L, e)
    assert r1 - r0 == nthreads * calls and b1 - b0 < r1 - r0, (b1 - b0, r1 - r0)


def test_direct_zero_copy_large_pinned(eng):
    # a pinned request larger than a combined batch: chunked keygen + crypt straight on the
    # caller's host memory (no staging copies), verdicts copied back per chunk
    L, e = eng
    key = splitmix64_bytes(3, 32)
    nonce0 = b"\xf0" + b"\xff" * 7 + splitmix64_bytes(4, 16)
    n = 150 * 65536 + 4321
    nb = (n + 65535) // 65536
    plain = splitmix64_bytes(5, n)
    src, body = _Pinned(L, plain), _Pinned(L, n + 16 * nb)
    assert L.xs_engine_seal(e, key, nonce0, 7, src.p, n, body.p) == 0
    want = _seal_expected(plain, nonce0, 7, key)
    assert body.raw == want
    wire = bytearray(want)
    wire[65552 * 70 + 16 + 100] ^= 0x10   # ciphertext byte of block 70
    wire[65552 * (nb - 1) + 3] ^= 0x01    # tag byte of the last (partial) block
    win, out = _Pinned(L, wire), _Pinned(L, n)
    ok = (ctypes.c_uint8 * nb)()
    assert L.xs_engine_open(e, key, nonce0, 7, win.p, len(wire), out.p, ok) == 0
    assert [j for j in range(nb) if not ok[j]] == [70, nb - 1]
    exp = bytearray(plain)
    for j in (70, nb - 1):
        exp[j * 65536:(j + 1) * 65536] = bytes(len(exp[j * 65536:(j + 1) * 65536]))
    assert out.raw == bytes(exp)
