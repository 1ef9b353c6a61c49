"""Ciphertext at the extremes of the matrix-core Poly1305's operand range.

The full-block Poly1305 feeds every ciphertext byte to v_mfma_i32_16x16x64_i8 as byte - 128
(round 4: the bias is applied by LDS atomics on the staged words), so a
block whose ciphertext is all 0x00 or all 0xFF drives every B operand to -128 or +127 and every
accumulator to its bound.  Random data never does.  Here the plaintext is chosen as the
keystream XOR a target pattern (the oracle's seal of zeros is the keystream), so the GPU's seal
must produce exactly that ciphertext and the oracle's tag, and the GPU's open must verify it,
decrypt it and catch a flipped tag bit.  Partial last blocks (the VALU Horner) get the same
patterns.
"""
import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

BLOCK = 65536
PATTERNS = [
    b"\x00", b"\xff", b"\x80", b"\x7f",
    b"\x00\xff", b"\xff\x00\x00\xff",
    b"\x00" * 15 + b"\xff",                   # one extreme byte per 16-byte chunk
    b"\xff" * 16 + b"\x00" * 16,              # alternating chunks
]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rclone_amd import device
    return device


def _target(pattern: bytes, n: int) -> bytes:
    return (pattern * (n // len(pattern) + 1))[:n]


def _plain_for(targets, nonce0, key):
    """Plaintext whose block i seals to targets[i] (block i uses nonce0 + i, cipher.go:665)."""
    out = []
    for i, t in enumerate(targets):
        ks = orc.seal(bytes(len(t)), orc.nonce_add(nonce0, i), key)[16:]  # the keystream itself
        out.append(bytes(a ^ b for a, b in zip(ks, t)) if len(t) < 4096 else
                   (np.frombuffer(ks, np.uint8) ^ np.frombuffer(t, np.uint8)).tobytes())
    return b"".join(out)


# 8 full blocks run the small-batch kernels (four waves per block); 300 the bulk one-wave-per-block
# kernels (XS_SPLIT_MAX = 256)
@pytest.mark.parametrize("nfull,tail", [(8, 0), (8, 1), (8, 1000), (8, 65535), (300, 777)])
def test_extreme_ciphertext_blocks(dev, nfull, tail):
    key = splitmix64_bytes(0xE7, 32)
    nonce0 = bytes([0xF8] + [0xFF] * 7) + splitmix64_bytes(0xE8, 16)  # block index carries into byte 8
    targets = [_target(PATTERNS[i % len(PATTERNS)], BLOCK) for i in range(nfull)]
    if tail:
        targets.append(_target(PATTERNS[len(targets) % len(PATTERNS)], tail))
    plain = _plain_for(targets, nonce0, key)
    t = torch.from_numpy(np.frombuffer(plain, dtype=np.uint8).copy()).cuda()
    body = dev.seal_object(key, nonce0, t)
    torch.cuda.synchronize()
    got = body.cpu().numpy().tobytes()
    want = orc.encrypt_file(plain, nonce0, key)[32:]
    assert got == want
    pos = 0
    for i, tg in enumerate(targets):  # the ciphertext really is the extreme pattern
        assert got[pos + 16:pos + 16 + len(tg)] == tg, i
        pos += 16 + len(tg)
    out, ok = dev.open_object(key, nonce0, body)
    torch.cuda.synchronize()
    assert bool(ok[:len(targets)].all()) and out[:len(plain)].cpu().numpy().tobytes() == plain
    # a flipped tag bit in every other block: exactly those fail and are zero-filled
    bad = body.clone()
    pos, flipped = 0, []
    for i, tg in enumerate(targets):
        if i % 2 == 1:
            bad[pos + (i % 16)] ^= 0x01
            flipped.append(i)
        pos += 16 + len(tg)
    out, ok = dev.open_object(key, nonce0, bad)
    torch.cuda.synchronize()
    okl = ok[:len(targets)].cpu().numpy().tolist()
    assert [i for i, v in enumerate(okl) if v == 0] == flipped
    o = out[:len(plain)].cpu().numpy().tobytes()
    pos = 0
    for i, tg in enumerate(targets):
        seg = o[i * BLOCK:i * BLOCK + len(tg)]
        assert seg == (bytes(len(tg)) if i in flipped else plain[i * BLOCK:i * BLOCK + len(tg)]), i
