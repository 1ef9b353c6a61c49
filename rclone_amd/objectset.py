"""Synthetic object-set runner (BASELINE configs[3]: "1 TiB synthetic object set, blocks
round-robin across GPUs").

One logical object of `total_blocks` 64 KiB blocks (block g sealed with nonce0 + g, the
nonce.add contract of cipher.go:665 / :737) is split round-robin over `world` ranks; a rank
processes its share in rounds of `round_blocks` resident blocks: the plaintext of global
block g is generated in HBM from (seed, g) (xs_fill_blocks_dev), sealed, opened + verified.
Per rank counters -- blocks, bytes, tag failures, round-trip mismatched words and an
order-independent digest of every tag (sum of the two 64-bit halves, mod 2^64) -- are summed
over ranks with one all-reduce, so the digest of a sharded run equals the single-GPU digest
of the same object set (tests/test_objectset_gpu.py checks exactly that at 1 TiB).

This is measurement/test harness code around the product kernels; it never falls back to the
CPU (every kernel call goes through librclone_crypt.so).
"""
import ctypes
import json
import os

import numpy as np
import torch

from . import _lib, device, shard

BLOCK_DATA = 65536
BLOCK_SIZE = 65552
DESC = np.dtype([("src", "<u8"), ("dst", "<u8"), ("len", "<u4"), ("res", "<u4"), ("nonce", "u1", (24,))])
N_COUNTERS = 6  # blocks, bytes, tag failures, round-trip mismatched words, tag digest lo, tag digest hi

# BASELINE configs[3]'s object set, as bench.py's objectset leg and tests/test_objectset_gpu.py
# both run it: their tag digests are the same number for any world size
CONFIG3_BLOCKS = 1 << 24  # 1 TiB of 64 KiB blocks
CONFIG3_KEY = bytes(range(100, 132))
CONFIG3_NONCE0 = b"\xf0" + b"\xff" * 7 + bytes(range(16))  # the set's nonces carry across byte 8
CONFIG3_SEED = 0x1417
CONFIG3_ROUND_BLOCKS = 100_000
# Oracle pins of the full-size synthetic workloads (data, not code): computed on the CPU by
# tests/golden/make_fullsize.py, which regenerates every block's plaintext and seals it with the
# oracle (oracle/xsalsa_simd.c), so a GPU run is held to numbers the GPU never produced.
FULLSIZE_PINS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "fullsize.json")


def fullsize_pins() -> dict:
    with open(FULLSIZE_PINS) as f:
        return json.load(f)


def _config3_digest() -> str:
    c3 = fullsize_pins()["config3"]
    if (c3["blocks"], c3["seed"], c3["key"], c3["nonce0"]) != (CONFIG3_BLOCKS, CONFIG3_SEED, CONFIG3_KEY.hex(),
                                                                CONFIG3_NONCE0.hex()):
        raise RuntimeError("tests/golden/fullsize.json pins another configs[3] set: rerun make_fullsize.py")
    return c3["tag_digest"]


# the order-independent tag digest of one pass over that set (hi || lo, hex): the CPU oracle's,
# the same for any world size (tests/test_objectset_gpu.py, bench.py's objectset leg)
CONFIG3_TAG_DIGEST = _config3_digest()


def _descriptors(nonce0: bytes, gidx: np.ndarray, round_blocks: int, open_mode: bool) -> np.ndarray:
    d = np.zeros(len(gidx), dtype=DESC)
    local = (np.arange(len(gidx), dtype=np.uint64) % np.uint64(round_blocks))
    a, b = local * np.uint64(BLOCK_DATA), local * np.uint64(BLOCK_SIZE)
    d["src"], d["dst"] = (b, a) if open_mode else (a, b)
    d["len"] = BLOCK_DATA
    d["nonce"] = shard.nonce_plus(nonce0, gidx)
    return d


def tag_digest(body: torch.Tensor, nb: int) -> torch.Tensor:
    """Sum (mod 2^64) of the two 64-bit halves of every tag of nb wire blocks -> int64[2]."""
    tags = body[:nb * BLOCK_SIZE].view(nb, BLOCK_SIZE)[:, :16].contiguous().view(torch.int64).view(nb, 2)
    return tags.sum(dim=0)


class RankRunner:
    """This rank's share of the object set, resident buffers sized for one round."""

    def __init__(self, key: bytes, nonce0: bytes, total_blocks: int, world: int, rank: int,
                 round_blocks: int, seed: int, dev):
        self.key, self.nonce0, self.world, self.rank, self.seed = bytes(key), bytes(nonce0), world, rank, seed
        self.dev = torch.device(dev)
        self.gidx = shard.owned_blocks(total_blocks, world, rank)
        self.n = len(self.gidx)
        self.B = max(1, min(round_blocks, self.n))
        self.rounds = (self.n + self.B - 1) // self.B
        self.d_seal = torch.from_numpy(_descriptors(self.nonce0, self.gidx, self.B, False).view(np.uint8)).to(self.dev)
        self.d_open = torch.from_numpy(_descriptors(self.nonce0, self.gidx, self.B, True).view(np.uint8)).to(self.dev)
        B = self.B
        self.plain = torch.empty(B * BLOCK_DATA, dtype=torch.uint8, device=self.dev)
        self.body = torch.empty(B * BLOCK_SIZE, dtype=torch.uint8, device=self.dev)
        self.out = torch.empty(B * BLOCK_DATA, dtype=torch.uint8, device=self.dev)
        self.ok = torch.empty(B, dtype=torch.uint8, device=self.dev)
        self.ws_seal = device.workspace(B, self.dev)
        self.ws_open = device.workspace(B, self.dev)
        self.counters = torch.zeros(N_COUNTERS, dtype=torch.int64, device=self.dev)
        self.kernel_events = []  # (seal?, start, end) around every crypt launch when timing

    def run_round(self, k: int, record: bool = False):
        L = _lib.lib()
        stream = torch.cuda.current_stream(self.dev)
        sp = ctypes.c_void_p(stream.cuda_stream)
        lo = k * self.B
        nb = min(self.B, self.n - lo)
        plen, blen = nb * BLOCK_DATA, nb * BLOCK_SIZE
        # global blocks gidx[lo:lo+nb] = rank + world*(lo..): first gidx[lo], stride world
        device.fill_blocks(self.plain[:plen], int(self.gidx[lo]), self.world, self.seed)
        ds = self.d_seal[lo * 48:(lo + nb) * 48]
        do = self.d_open[lo * 48:(lo + nb) * 48]
        _lib.check(L.xs_keygen_batch_dev(1, self.key, ds.data_ptr(), nb, self.plain.data_ptr(), plen,
                                         self.body.data_ptr(), blen, self.ws_seal.data_ptr(), sp), "keygen")
        ev = self._ev(record, stream)
        _lib.check(L.xs_crypt_dev(1, self.ws_seal.data_ptr(), nb, self.plain.data_ptr(), self.body.data_ptr(),
                                  None, sp), "seal")
        self._ev_end(ev, True, stream)
        _lib.check(L.xs_keygen_batch_dev(0, self.key, do.data_ptr(), nb, self.body.data_ptr(), blen,
                                         self.out.data_ptr(), plen, self.ws_open.data_ptr(), sp), "keygen")
        ev = self._ev(record, stream)
        _lib.check(L.xs_crypt_dev(0, self.ws_open.data_ptr(), nb, self.body.data_ptr(), self.out.data_ptr(),
                                  self.ok.data_ptr(), sp), "open")
        self._ev_end(ev, False, stream)
        c = self.counters
        c[0] += nb
        c[1] += plen
        c[2] += nb - self.ok[:nb].sum(dtype=torch.int64)
        # opened plaintext vs the generator's stream, recomputed (the kept plaintext is not re-read)
        device.verify_blocks(self.out[:plen], int(self.gidx[lo]), self.world, self.seed, c[3:4])
        c[4:6] += tag_digest(self.body, nb)

    def _ev(self, record, stream):
        if not record:
            return None
        a = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        return a

    def _ev_end(self, a, seal, stream):
        if a is None:
            return
        b = torch.cuda.Event(enable_timing=True)
        b.record(stream)
        self.kernel_events.append((seal, a, b))

    def run_all(self, record: bool = False):
        """One pass over the rank's share.  Blocks, bytes, failures and mismatches accumulate over
        passes; the tag digest (counters 4:6) is the latest pass's, so it is comparable across runs
        of any length (one 16-byte clear per pass)."""
        self.counters[4:6].zero_()
        for k in range(self.rounds):
            self.run_round(k, record)
        return self.counters

    def block(self, g: int):
        """(plaintext, wire) of global block g if it is in the most recent round (for checks)."""
        pos = int(np.searchsorted(self.gidx, g))
        if pos >= self.n or self.gidx[pos] != g:
            raise KeyError(g)
        k, j = divmod(pos, self.B)
        if k != self.rounds - 1:
            raise KeyError(g)
        p = self.plain[j * BLOCK_DATA:(j + 1) * BLOCK_DATA].cpu().numpy().tobytes()
        w = self.body[j * BLOCK_SIZE:(j + 1) * BLOCK_SIZE].cpu().numpy().tobytes()
        return p, w


def digest_to_u64(counters) -> tuple:
    c = [int(x) for x in counters.tolist()]
    return tuple(x & 0xFFFFFFFFFFFFFFFF for x in c)
