"""Multi-GPU partitioning of crypt blocks (one process per GPU, torch.distributed).

Blocks are independent (block i of an object is a pure function of key, nonce0 + i and its
plaintext, cipher.go:665-678), so an object set shards with no data-path exchange: rank r of
W owns the blocks b with b % W == r (round-robin, BASELINE config 4).  Each rank seals its
blocks through the descriptor entry point (per-block nonce = nonce0 + b), laid out
contiguously in its own HBM.  The only collective is one all-reduce of a few int64 counters
(blocks, bytes, tag failures) -- RCCL over xGMI with backend "nccl", gloo on CPU.
"""
import math

import numpy as np

from ._lib import XsBlockDesc

BLOCK_DATA = 65536
BLOCK_SIZE = 65552


def owned_blocks(total_blocks: int, world: int, rank: int) -> np.ndarray:
    """Global indices of the blocks rank `rank` owns (round-robin)."""
    if not (0 <= rank < world):
        raise ValueError("bad rank")
    return np.arange(rank, total_blocks, world, dtype=np.int64)


def nonce_plus(nonce0: bytes, idx: np.ndarray) -> np.ndarray:
    """nonce0 + idx as 24-byte little-endian numbers (nonce.add, cipher.go:665) -> (n, 24) u8.
    Vectorised: 64-bit add of the low word, carries into bytes 8.. handled per carrying row."""
    idx = np.asarray(idx, dtype=np.uint64)
    n0 = bytes(nonce0)
    lo0 = np.uint64(int.from_bytes(n0[:8], "little"))
    out = np.empty((len(idx), 24), dtype=np.uint8)
    with np.errstate(over="ignore"):
        lo = idx + lo0
    out[:, :8] = lo.astype("<u8").view(np.uint8).reshape(-1, 8)
    out[:, 8:] = np.frombuffer(n0[8:], dtype=np.uint8)
    carry = np.flatnonzero(lo < lo0)
    if len(carry):
        hi = int.from_bytes(n0[8:], "little")
        up = np.frombuffer(((hi + 1) % (1 << 128)).to_bytes(16, "little"), dtype=np.uint8)
        out[carry, 8:] = up
    return out


def seal_descriptors(nonce0: bytes, global_idx: np.ndarray, block_len: int = BLOCK_DATA,
                     open_mode: bool = False) -> np.ndarray:
    """Descriptors for the given global blocks, packed contiguously in local buffers:
    seal: plaintext at i*65536 -> wire block at i*65552; open: the reverse."""
    n = len(global_idx)
    d = np.zeros(n, dtype=np.dtype([("src", "<u8"), ("dst", "<u8"), ("len", "<u4"), ("res", "<u4"),
                                    ("nonce", "u1", (24,))]))
    assert d.dtype.itemsize == 48 and XsBlockDesc
    i = np.arange(n, dtype=np.uint64)
    if open_mode:
        d["src"] = i * BLOCK_SIZE
        d["dst"] = i * BLOCK_DATA
    else:
        d["src"] = i * BLOCK_DATA
        d["dst"] = i * BLOCK_SIZE
    d["len"] = block_len
    d["nonce"] = nonce_plus(nonce0, global_idx)
    return d


DESC_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("len", "<u4"), ("res", "<u4"), ("nonce", "u1", (24,))])


def _align16(x):
    return (x + 15) & ~15


def mixed_object_layout(total, rng, min_size=4096, max_size=8 << 20):
    """BASELINE configs[2] object set: sizes log-uniform in [min_size, max_size] until `total`
    plaintext bytes, random 24-byte nonces (every ~len/5-th about to carry out of byte 7,
    cipher.go:665), each object's plaintext and wire body (crypt file minus its 32-byte
    header, cipher.go:1121) 16-byte aligned in one plaintext image and one wire image.
    Returns (sizes, nonces, pstart, wstart, plain_len, wire_len, desc, obj) with one seal
    descriptor per 64 KiB block (plain -> wire; swap src/dst for open) and obj[i] = the
    object of descriptor i."""
    lo, hi = math.log(min_size), math.log(max_size)
    sizes = []
    acc = 0
    while acc < total:
        sz = int(math.exp(rng.uniform(lo, hi)))
        sizes.append(sz)
        acc += sz
    nonces = [bytes(rng.integers(0, 256, 24, dtype=np.uint8)) for _ in sizes]
    for o in range(0, len(sizes), max(1, len(sizes) // 5)):
        nonces[o] = b"\xfe" + b"\xff" * 7 + nonces[o][8:]
    pstart, wstart, p, w = [], [], 0, 0
    nblk = [(sz + BLOCK_DATA - 1) // BLOCK_DATA for sz in sizes]
    for sz, nb in zip(sizes, nblk):
        pstart.append(p)
        wstart.append(w)
        p = _align16(p + sz)
        w = _align16(w + sz + 16 * nb)
    d = np.zeros(sum(nblk), dtype=DESC_DTYPE)
    obj = np.zeros(len(d), dtype=np.int64)
    k = 0
    for o, sz in enumerate(sizes):
        n = nblk[o]
        i = np.arange(n, dtype=np.uint64)
        sl = slice(k, k + n)
        d["src"][sl] = pstart[o] + i * BLOCK_DATA
        d["dst"][sl] = wstart[o] + i * BLOCK_SIZE
        d["len"][sl] = np.minimum(BLOCK_DATA, sz - i.astype(np.int64) * BLOCK_DATA)
        d["nonce"][sl] = nonce_plus(nonces[o], np.arange(n))
        obj[sl] = o
        k += n
    return sizes, nonces, pstart, wstart, p, w, d, obj


def reduce_counters(counters, dist=None, group=None):
    """Sum a small int64 tensor of counters over all ranks (the only collective)."""
    if dist is not None and dist.is_initialized():
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters
