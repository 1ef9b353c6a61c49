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
# the order-independent tag digest of one pass over that set (hi || lo, hex), measured on the GPU by
# tests/test_objectset_gpu.py at world 1, 2 and 8 (equal for all three; each rank's last block is
# checked against the CPU oracle there): a regression anchor for the test and the bench leg
CONFIG3_TAG_DIGEST = "26763293cb7e88a920e9c78b28f3f58d"


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
        self._pipe = None  # second buffer set + streams of run_all_pipelined, made on first use

    def _span(self, k: int):
        lo = k * self.B
        nb = min(self.B, self.n - lo)
        return lo, nb, nb * BLOCK_DATA, nb * BLOCK_SIZE

    def _fill(self, k: int, plain: torch.Tensor):
        # global blocks gidx[lo:lo+nb] = rank + world*(lo..): first gidx[lo], stride world
        lo, _, plen, _ = self._span(k)
        device.fill_blocks(plain[:plen], int(self.gidx[lo]), self.world, self.seed)

    def _verify(self, k: int, out: torch.Tensor, mismatch: torch.Tensor):
        # opened plaintext vs the generator's stream, recomputed (the kept plaintext is not re-read)
        lo, _, plen, _ = self._span(k)
        device.verify_blocks(out[:plen], int(self.gidx[lo]), self.world, self.seed, mismatch)

    def _crypt(self, k: int, bufs, stream, record: bool):
        """Key schedules, seal, open, verdict count and tag digest of round k on `stream`."""
        plain, body, out, ok, ws_seal, ws_open = bufs
        L = _lib.lib()
        sp = ctypes.c_void_p(stream.cuda_stream)
        lo, nb, plen, blen = self._span(k)
        ds = self.d_seal[lo * 48:(lo + nb) * 48]
        do = self.d_open[lo * 48:(lo + nb) * 48]
        _lib.check(L.xs_keygen_batch_dev(1, self.key, ds.data_ptr(), nb, plain.data_ptr(), plen,
                                         body.data_ptr(), blen, ws_seal.data_ptr(), sp), "keygen")
        ev = self._ev(record, stream)
        _lib.check(L.xs_crypt_dev(1, ws_seal.data_ptr(), nb, plain.data_ptr(), body.data_ptr(), None, sp), "seal")
        self._ev_end(ev, True, stream)
        _lib.check(L.xs_keygen_batch_dev(0, self.key, do.data_ptr(), nb, body.data_ptr(), blen,
                                         out.data_ptr(), plen, ws_open.data_ptr(), sp), "keygen")
        ev = self._ev(record, stream)
        _lib.check(L.xs_crypt_dev(0, ws_open.data_ptr(), nb, body.data_ptr(), out.data_ptr(), ok.data_ptr(), sp),
                   "open")
        self._ev_end(ev, False, stream)
        with torch.cuda.stream(stream):
            c = self.counters
            c[0] += nb
            c[1] += plen
            c[2] += nb - ok[:nb].sum(dtype=torch.int64)
            c[4:6] += tag_digest(body, nb)

    def run_round(self, k: int, record: bool = False):
        """Round k in stream order on the current stream: generate, seal, open, verify."""
        stream = torch.cuda.current_stream(self.dev)
        bufs = (self.plain, self.body, self.out, self.ok, self.ws_seal, self.ws_open)
        self._fill(k, self.plain)
        self._crypt(k, bufs, stream, record)
        self._verify(k, self.out, self.counters[3:4])

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

    def prepare_pipeline(self):
        """Allocate run_all_pipelined's second buffer set and its two streams (once)."""
        if self._pipe is None:
            B = self.B
            second = (torch.empty(B * BLOCK_DATA, dtype=torch.uint8, device=self.dev),
                      torch.empty(B * BLOCK_SIZE, dtype=torch.uint8, device=self.dev),
                      torch.empty(B * BLOCK_DATA, dtype=torch.uint8, device=self.dev),
                      torch.empty(B, dtype=torch.uint8, device=self.dev),
                      device.workspace(B, self.dev), device.workspace(B, self.dev))
            self._pipe = {"bufs": [(self.plain, self.body, self.out, self.ok, self.ws_seal, self.ws_open), second],
                          "crypt": torch.cuda.Stream(self.dev), "data": torch.cuda.Stream(self.dev),
                          "mismatch": torch.zeros(1, dtype=torch.int64, device=self.dev)}

    def run_all_pipelined(self, record: bool = False):
        """The same pass, with the memory-bound generate / verify kernels of neighbouring rounds
        overlapped with the VALU-bound seal / open kernels: two buffer sets, the crypt work of
        round k on one stream while another generates round k+1 (or k+2) and verifies round k-1.
        Same bytes, counters and digest as run_all (tests/test_objectset_gpu.py); the caller's
        current stream is joined on entry and waits for both streams on exit."""
        self.prepare_pipeline()
        P = self._pipe
        s_c, s_d, bufs, mism = P["crypt"], P["data"], P["bufs"], P["mismatch"]
        cur = torch.cuda.current_stream(self.dev)
        self.counters[4:6].zero_()
        mism.zero_()
        s_c.wait_stream(cur)
        s_d.wait_stream(cur)
        R = self.rounds
        ev_fill, ev_crypt, ev_ver = [None] * R, [None] * R, [None] * R

        def mark(stream):
            e = torch.cuda.Event()
            e.record(stream)
            return e

        def fill(k):
            with torch.cuda.stream(s_d):
                if k >= 2:
                    s_d.wait_event(ev_crypt[k - 2])  # round k-2's seal has read this plaintext buffer
                self._fill(k, bufs[k % 2][0])
                ev_fill[k] = mark(s_d)

        fill(0)
        if R > 1:
            fill(1)
        for k in range(R):
            s_c.wait_event(ev_fill[k])
            if k >= 2:
                s_c.wait_event(ev_ver[k - 2])  # round k-2's output buffer has been verified
            self._crypt(k, bufs[k % 2], s_c, record)
            ev_crypt[k] = mark(s_c)
            with torch.cuda.stream(s_d):
                s_d.wait_event(ev_crypt[k])
                self._verify(k, bufs[k % 2][2], mism)
                ev_ver[k] = mark(s_d)
            if k + 2 < R:
                fill(k + 2)
        cur.wait_stream(s_c)
        cur.wait_stream(s_d)
        self.counters[3:4] += mism
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
