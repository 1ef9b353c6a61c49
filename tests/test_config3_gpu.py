"""BASELINE configs[2] (SURVEY §8(d) "Config 3"): decrypt+verify of 10 GiB of mixed
4 KiB-8 MiB objects chunked to 64 KiB, with tag-fail injection caught.

Objects (sizes log-uniform in [4 KiB, 8 MiB], seeded) are sealed block by block on the CPU
oracle -- the reference's role, cipher.go:737 with nonce = nonce0 + i -- then opened on the
GPU in ONE descriptor batch (xs_open_batch_dev, cipher.go:880 per block).  ~0.1% of the
blocks get one byte flipped (tag bytes, first/last ciphertext byte or a random byte); the
test expects exactly those blocks' ok flags to be 0, their plaintext zero-filled and every
other byte equal to the original, and -- through the cipher.go mirror -- the decrypter of an
object to return ErrorEncryptedBadBlock exactly at its first failing block
(cipher.go:885-893), or to pass zero-filled blocks with pass_bad_blocks.

RCLONE_AMD_CONFIG3_BYTES overrides the 10 GiB total (e.g. for a quick local run).
"""
import os

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.shard import mixed_object_layout

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOTAL = int(os.environ.get("RCLONE_AMD_CONFIG3_BYTES", 10 << 30))
SEED = 0xC0F3
BLOCK_DATA, BLOCK_SIZE = 65536, 65552
MAGIC = b"RCLONE\x00\x00"


def make_layout(total, rng):
    """Object sizes, nonces and the per-block descriptor table (plain <-> wire offsets)."""
    return mixed_object_layout(total, rng)


@pytest.fixture(scope="module")
def config3():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rclone_amd import device
    rng = np.random.default_rng(SEED)
    key = bytes(32)  # crypt with an empty password: all-zero data key (cipher.go:231-236)
    sizes, nonces, pstart, wstart, ptot, wtot, d, obj = make_layout(TOTAL, rng)
    plain_dev = torch.zeros(ptot, dtype=torch.uint8, device="cuda")
    device.fill_random(plain_dev, SEED)
    for o, s in enumerate(sizes):  # alignment gaps are zero in both plaintext images
        end = pstart[o] + s
        nxt = pstart[o + 1] if o + 1 < len(sizes) else ptot
        if nxt > end:
            plain_dev[end:nxt] = 0
    plain_host = plain_dev.cpu().numpy()
    wire = np.zeros(wtot, dtype=np.uint8)
    orc.seal_desc(wire, plain_host, d, key)  # CPU reference seal
    # tag-fail injection in ~0.1% of the blocks
    nbad = max(3, len(d) // 1000)
    bad = np.sort(rng.choice(len(d), nbad, replace=False))
    flips = []
    for j, b in enumerate(bad.tolist()):
        blen = 16 + int(d["len"][b])
        pos = [0, 15, 16, blen - 1, int(rng.integers(0, blen))][j % 5]
        flips.append(int(d["dst"][b]) + pos)
        wire[flips[-1]] ^= 0x40
    od = d.copy()
    od["src"], od["dst"] = d["dst"], d["src"]
    return dict(device=device, key=key, sizes=sizes, nonces=nonces, pstart=pstart, wstart=wstart, d=d, od=od,
                obj=obj, bad=bad, flips=flips, plain_dev=plain_dev, plain_host=plain_host, wire=wire)


def test_config3_open_batch_flags_and_bytes(config3):
    c = config3
    device = c["device"]
    wire_dev = torch.from_numpy(c["wire"]).cuda()
    out = torch.zeros_like(c["plain_dev"])
    ok = device.open_batch(c["key"], c["od"], wire_dev, out)
    torch.cuda.synchronize()
    ok = ok.cpu().numpy()
    assert len(ok) == len(c["d"])
    assert np.array_equal(np.flatnonzero(ok == 0), c["bad"])   # exactly the injected blocks
    expect = c["plain_dev"].clone()
    for b in c["bad"].tolist():
        s, n = int(c["d"]["src"][b]), int(c["d"]["len"][b])
        assert int(out[s:s + n].count_nonzero()) == 0          # failed block zero-filled
        expect[s:s + n] = 0
    assert bool(torch.equal(out, expect))


def _file(c, o):
    w0 = c["wstart"][o]
    s = c["sizes"][o]
    nb = (s + BLOCK_DATA - 1) // BLOCK_DATA
    return MAGIC + c["nonces"][o] + c["wire"][w0:w0 + s + 16 * nb].tobytes()


def test_config3_stream_error_at_first_bad_block(config3):
    # the Go layer: decrypter.Read returns the good blocks, then ErrorEncryptedBadBlock
    from rclone_amd import crypt
    from tests.go_readers import Buffer, read_all
    c = config3
    nblk = [(s + BLOCK_DATA - 1) // BLOCK_DATA for s in c["sizes"]]
    first = np.concatenate([[0], np.cumsum(nblk)[:-1]])
    bad_rel = {}  # object -> failing block indices within the object
    for b in c["bad"].tolist():
        o = int(c["obj"][b])
        bad_rel.setdefault(o, []).append(b - int(first[o]))
    bad_objs = sorted(bad_rel)
    later = [o for o in bad_objs if bad_rel[o][0] > 0]   # good blocks precede the failure
    picks = sorted(set(bad_objs[:2] + later[:2]))
    clean = next(o for o in range(len(c["sizes"])) if o not in bad_rel)
    cip = crypt.Cipher("", "")
    for o in picks:
        blocks = bad_rel[o]
        p0, s = c["pstart"][o], c["sizes"][o]
        plain = c["plain_host"][p0:p0 + s].tobytes()
        data, err = read_all(cip.decrypt_data(Buffer(_file(c, o))))
        assert isinstance(err, crypt.ErrorEncryptedBadBlock), (o, err)
        assert data == plain[:blocks[0] * BLOCK_DATA]
        # pass_bad_blocks: every byte delivered, failing blocks as zeros (cipher.go:885-893)
        pb = crypt.Cipher("", "", pass_bad_blocks=True)
        data, err = read_all(pb.decrypt_data(Buffer(_file(c, o))))
        assert err is None
        exp = bytearray(plain)
        for b in blocks:
            exp[b * BLOCK_DATA:min(s, (b + 1) * BLOCK_DATA)] = bytes(min(s, (b + 1) * BLOCK_DATA) - b * BLOCK_DATA)
        assert data == bytes(exp)
    p0, s = c["pstart"][clean], c["sizes"][clean]
    data, err = read_all(cip.decrypt_data(Buffer(_file(c, clean))))
    assert err is None and data == c["plain_host"][p0:p0 + s].tobytes()


def test_config3_oracle_agrees_on_flags(config3):
    # the CPU checker itself sees the same failing set (guards the fixture, not the GPU)
    c = config3
    sample = np.unique(np.concatenate([c["bad"], np.arange(0, len(c["d"]), max(1, len(c["d"]) // 2000))]))
    od = c["od"][sample].copy()
    n = od["len"].astype(np.int64)
    off = np.concatenate([[0], np.cumsum(n)[:-1]])
    od["dst"] = off
    out = np.zeros(int(n.sum()), dtype=np.uint8)
    ok = np.zeros(len(od), dtype=np.uint8)
    orc.open_desc(out, ok, c["wire"], od, c["key"])
    assert np.array_equal(sample[ok == 0], c["bad"])


def test_config3_gpu_seal_equals_the_oracle(config3):
    # the other direction at full size: the same 10 GiB object set (partial last blocks, nonces
    # that carry out of byte 7) sealed on the GPU in one descriptor batch (xs_seal_batch_dev,
    # cipher.go:737 per block) equals the CPU oracle's wire image byte for byte -- the fixture's,
    # with the injected flips undone
    c = config3
    body = torch.zeros(len(c["wire"]), dtype=torch.uint8, device="cuda")
    c["device"].seal_batch(c["key"], c["d"], c["plain_dev"], body)
    want = torch.from_numpy(c["wire"]).cuda()
    want[torch.tensor(c["flips"], dtype=torch.int64, device="cuda")] ^= 0x40
    torch.cuda.synchronize()
    assert bool(torch.equal(body, want))
    del body, want
    torch.cuda.empty_cache()
