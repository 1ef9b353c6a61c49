"""Deterministic test-data generators shared by tests/, bench.py and tests/golden/make_golden.py.

These reproduce the reference's own test readers bit-exactly so fixtures generated in the
build container can be re-derived anywhere (including the GPU box) without shipping data:

* ``random_source``  -- backend/crypt/cipher_test.go:1007-1045 ``randomSource``:
  byte i (0-based) = (i + 1) % 257 truncated to a byte.
* ``pattern_bytes``  -- lib/readers/pattern_reader.go:11-39 ``PatternReader``:
  byte i = i % 251.
* ``splitmix64_bytes`` -- SplitMix64 stream (seeded), little-endian words; the same
  generator runs on-device for the synthetic benchmark objects.
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def random_source(n: int) -> bytes:
    i = np.arange(1, n + 1, dtype=np.int64)
    return (i % 257).astype(np.uint8).tobytes()


def pattern_bytes(n: int, offset: int = 0) -> bytes:
    i = np.arange(offset, offset + n, dtype=np.int64)
    return (i % 251).astype(np.uint8).tobytes()


def splitmix64_words(seed: int, nwords: int, first: int = 0) -> np.ndarray:
    """word k = mix(seed + (k + 1) * golden), the standard SplitMix64 sequence (k from first)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(first + 1, first + nwords + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix64_bytes(seed: int, n: int) -> bytes:
    words = splitmix64_words(seed, (n + 7) // 8)
    return words.astype("<u8").tobytes()[:n]


def splitmix64_block(seed: int, g: int) -> bytes:
    """Global 64 KiB block g of the stream (what xs_fill_blocks_dev writes for block g)."""
    return splitmix64_words(seed, 8192, first=g * 8192).astype("<u8").tobytes()
