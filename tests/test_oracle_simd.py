"""The vectorised CPU baseline (oracle/xsalsa_simd.c, bench.py's cpu_baseline leg) against the
scalar oracle (oracle/xsalsa_oracle.c, itself pinned to the reference's vectors in
tests/test_oracle.py): byte-identical boxes, tags and verdicts at every SIMD level the host has.
"""
import ctypes

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes

L = orc.lib()
vp = ctypes.c_void_p
LEVELS = [lv for lv in (1, 2) if lv <= L.orc_simd_level()]


@pytest.fixture(params=LEVELS or [None], ids=lambda lv: {1: "avx2", 2: "avx512", None: "none"}[lv])
def level(request):
    if request.param is None:
        pytest.skip("host has neither AVX2 nor AVX-512")
    L.orc_simd_force(request.param)
    yield request.param
    L.orc_simd_force(-1)


def _seal(fn, msg, nonce, key):
    out = ctypes.create_string_buffer(len(msg) + 16)
    fn(out, msg, len(msg), nonce, key)
    return out.raw


def test_boxes_equal_scalar_every_length(level):
    key = splitmix64_bytes(11, 32)
    for n in list(range(0, 200)) + [511, 512, 513, 1023, 1024, 1025, 4096, 65503, 65504, 65536]:
        msg = splitmix64_bytes(1000 + n, n)
        nonce = splitmix64_bytes(2000 + n, 24)
        want = _seal(L.orc_secretbox_seal, msg, nonce, key)
        got = _seal(L.orc_simd_secretbox_seal, msg, nonce, key)
        assert got == want, n
        out = ctypes.create_string_buffer(max(n, 1))
        assert L.orc_simd_secretbox_open(out, got, len(got), nonce, key) == 0
        assert out.raw[:n] == msg
        bad = bytearray(got)
        bad[(n * 7) % len(bad)] ^= 0x10
        assert L.orc_simd_secretbox_open(out, bytes(bad), len(bad), nonce, key) == -1


def test_blocks_equal_scalar_with_carry_nonce(level):
    nb = 24
    key = splitmix64_bytes(12, 32)
    nonce0 = bytes([0xFF] * 7 + [3] + [0] * 16)  # the block index carries into byte 8
    plain = np.frombuffer(splitmix64_bytes(13, nb * 65536), dtype=np.uint8).copy()
    want = np.empty(nb * 65552, dtype=np.uint8)
    got = np.empty_like(want)
    L.orc_seal_blocks(vp(want.ctypes.data), vp(plain.ctypes.data), nb, nonce0, key)
    assert L.orc_simd_seal_blocks(vp(got.ctypes.data), vp(plain.ctypes.data), nb, nonce0, key) >= 1
    assert np.array_equal(got, want)
    got[5 * 65552 + 3] ^= 1  # tag of block 5
    got[17 * 65552 + 40000] ^= 0x80  # ciphertext of block 17
    out = np.empty(nb * 65536, dtype=np.uint8)
    ok = np.empty(nb, dtype=np.uint8)
    assert L.orc_simd_open_blocks(vp(out.ctypes.data), vp(ok.ctypes.data), vp(got.ctypes.data), nb, nonce0, key) >= 1
    assert [i for i in range(nb) if not ok[i]] == [5, 17]
    exp = plain.copy()
    exp[5 * 65536:6 * 65536] = 0
    exp[17 * 65536:18 * 65536] = 0
    assert np.array_equal(out, exp)
