"""BASELINE configs[3] at full size: a 1 TiB synthetic object (2^24 blocks of 64 KiB, block g
sealed with nonce0 + g, cipher.go:665/:737) processed in 100k-block rounds, round-robin over
1, 2 and 8 simulated ranks on one GPU (the ranks run one after another; no collective is
needed to sum their counters here).  Size-independent properties:

* every block round-trips and every tag verifies (counters);
* the order-independent tag digest (sum of tag halves mod 2^64) is the same for every world
  size, i.e. the sharded ciphertext is the single-GPU ciphertext, and at full size it equals
  the CPU oracle's digest of all 2^24 blocks (tests/golden/fullsize.json, computed by
  tests/golden/make_fullsize.py; the contract is cipher.go:665-678 nonce.add, :737 Seal);
* the last block of every rank is bit-exact against the CPU oracle.

RCLONE_AMD_OBJECTSET_BLOCKS overrides 2^24 for a quick run.
"""
import os

import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_block

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from rclone_amd.objectset import (CONFIG3_BLOCKS, CONFIG3_KEY, CONFIG3_NONCE0, CONFIG3_SEED,  # noqa: E402
                                  CONFIG3_TAG_DIGEST)

TOTAL = int(os.environ.get("RCLONE_AMD_OBJECTSET_BLOCKS", CONFIG3_BLOCKS))
SEED = CONFIG3_SEED
KEY = CONFIG3_KEY
NONCE0 = CONFIG3_NONCE0  # the set's nonces carry across byte 8


def test_objectset_digest_independent_of_world():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rclone_amd.objectset import RankRunner, digest_to_u64
    res = {}
    for world in (1, 2, 8):
        tot = None
        for rank in range(world):
            r = RankRunner(KEY, NONCE0, TOTAL, world, rank, 100_000, SEED, "cuda")
            c = r.run_all().clone()
            tot = c if tot is None else tot + c
            g = int(r.gidx[-1])
            p, w = r.block(g)
            assert p == splitmix64_block(SEED, g)
            assert w == orc.seal(p, orc.nonce_add(NONCE0, g), KEY), (world, rank, g)
            del r
            torch.cuda.empty_cache()
        blocks, nbytes, fails, mism, d0, d1 = digest_to_u64(tot)
        assert (blocks, nbytes, fails, mism) == (TOTAL, TOTAL * 65536, 0, 0), world
        res[world] = (d0, d1)
        # the same string bench.py's objectset leg reports (counters.tag_digest)
        print(f"configs[3] world {world}: {TOTAL} blocks, tag_digest {d1:016x}{d0:016x}")
    assert res[1] == res[2] == res[8]
    if TOTAL == CONFIG3_BLOCKS:  # the oracle's digest, which bench.py's objectset leg is held to too
        d0, d1 = res[1]
        assert f"{d1:016x}{d0:016x}" == CONFIG3_TAG_DIGEST
    else:  # a quick run: the oracle digests the same prefix here
        s, _ = orc.seal_gen(TOTAL, 0, 1, SEED, NONCE0, KEY)
        assert res[1] == s


def test_verify_blocks_counts_mismatched_words():
    # the object set's round-trip check (xs_verify_blocks_dev) recomputes the generator's stream:
    # zero on the generated blocks (any first_block / stride), and exactly the flipped words
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rclone_amd import device
    nb, first, stride = 37, 5, 3
    t = torch.empty(nb * 65536, dtype=torch.uint8, device="cuda")
    device.fill_blocks(t, first, stride, SEED)
    assert t[65536 * 2:65536 * 3].cpu().numpy().tobytes() == splitmix64_block(SEED, first + 2 * stride)
    m = torch.zeros(1, dtype=torch.int64, device="cuda")
    device.verify_blocks(t, first, stride, SEED, m)
    assert int(m) == 0
    device.verify_blocks(t, first, stride + 1, SEED, m)  # another layout: almost every word differs
    assert int(m) >= (nb - 1) * 8192
    m.zero_()
    for off in (0, 8 * 8191, 65536 * 17 + 8 * 100, nb * 65536 - 8):
        t[off + 3] ^= 0x40  # one byte in each of four words (block 0 start / end, middle, last word)
    device.verify_blocks(t, first, stride, SEED, m)
    assert int(m) == 4
