"""GPU parity: the HIP path (through the C ABI) against the oracle and the committed
golden fixtures (libsodium + reference KATs).  Bit-exact is the bar.
"""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import pattern_bytes, random_source, splitmix64_bytes

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MAGIC = b"RCLONE\x00\x00"


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rclone_amd import device
    return device


def to_dev(b: bytes):
    a = np.frombuffer(b, dtype=np.uint8).copy() if len(b) else np.zeros(0, dtype=np.uint8)
    return torch.from_numpy(a).cuda()


def to_bytes(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().tobytes()


def _plain(entry):
    if entry["plain"] == "random_source":
        return random_source(entry["size"])
    if entry["plain"] == "pattern":
        return pattern_bytes(entry["size"])
    return splitmix64_bytes(entry["plain_seed"], entry["size"])


def test_reference_golden_files(dev, ref_kat):
    zkey, n0 = bytes(32), bytes(range(1, 25))
    for name, plain in (("file1", b"\x01"), ("file16", bytes(range(1, 17)))):
        body = dev.seal_object(zkey, n0, to_dev(plain))
        assert (MAGIC + n0 + to_bytes(body)).hex() == ref_kat[name]
        out, ok = dev.open_object(zkey, n0, body)
        assert to_bytes(out) == plain and to_bytes(ok) == b"\x01"


def test_single_boxes(dev, sodium_vectors):
    key = bytes.fromhex(sodium_vectors["key"])
    nonce = bytes.fromhex(sodium_vectors["nonce"])
    for v in sodium_vectors["single"]:
        msg = splitmix64_bytes(v["msg_seed"], v["len"])
        body = to_bytes(dev.seal_object(key, nonce, to_dev(msg)))
        assert hashlib.sha256(body).hexdigest() == v["sha256"], v["len"]
        out, ok = dev.open_object(key, nonce, to_dev(body))
        assert to_bytes(out) == msg and to_bytes(ok) == b"\x01", v["len"]


def test_crypt_files(dev, sodium_vectors):
    key = bytes.fromhex(sodium_vectors["key"])
    for f in sodium_vectors["files"]:
        plain = _plain(f)
        if not plain:
            continue
        n0 = bytes.fromhex(f["nonce0"])
        body = to_bytes(dev.seal_object(key, n0, to_dev(plain)))
        ct = MAGIC + n0 + body
        assert len(ct) == f["enc_size"]
        assert hashlib.sha256(ct).hexdigest() == f["sha256"], (f["size"], f["plain"], f["nonce0"])
        out, ok = dev.open_object(key, n0, to_dev(body))
        assert to_bytes(out) == plain
        assert set(to_bytes(ok)) == {1}


def test_many_blocks_vs_oracle(dev):
    key = splitmix64_bytes(11, 32)
    n0 = bytes([0xF0] + [0xFF] * 23)  # wraps the 192-bit nonce inside the object
    plain = splitmix64_bytes(12, 300 * 65536 + 777)
    want = orc.encrypt_file(plain, n0, key)
    body = to_bytes(dev.seal_object(key, n0, to_dev(plain)))
    assert MAGIC + n0 + body == want
    out, ok = dev.open_object(key, n0, to_dev(body))
    assert to_bytes(out) == plain and set(to_bytes(ok)) == {1}


def test_first_block_offset(dev):
    # sealing blocks 5.. of an object equals the tail of sealing the whole object
    key = splitmix64_bytes(21, 32)
    n0 = splitmix64_bytes(22, 24)
    plain = splitmix64_bytes(23, 9 * 65536 + 5)
    whole = to_bytes(dev.seal_object(key, n0, to_dev(plain)))
    tail = to_bytes(dev.seal_object(key, n0, to_dev(plain[5 * 65536:]), first_block=5))
    assert tail == whole[5 * 65552:]


def test_tag_fail_injection(dev):
    key = splitmix64_bytes(31, 32)
    n0 = splitmix64_bytes(32, 24)
    nb = 64
    plain = splitmix64_bytes(33, nb * 65536 - 100)
    body = bytearray(to_bytes(dev.seal_object(key, n0, to_dev(plain))))
    rng = np.random.default_rng(5)
    bad = sorted(set(int(x) for x in rng.choice(nb, 9, replace=False)))
    for b in bad:
        blen = min(65552, len(body) - b * 65552)
        pos = [0, 15, 16, blen - 1, int(rng.integers(0, blen))][b % 5]   # tag bytes, first/last ct byte
        body[b * 65552 + pos] ^= 0x5A
    out, ok = dev.open_object(key, n0, to_dev(bytes(body)))
    ok = to_bytes(ok)
    out = to_bytes(out)
    assert [i for i in range(nb) if ok[i] == 0] == bad
    for b in range(nb):
        seg = slice(b * 65536, min((b + 1) * 65536, len(plain)))
        if b in bad:
            assert out[seg] == bytes(len(out[seg]))   # zero-filled (pass_bad_blocks contract)
        else:
            assert out[seg] == plain[seg]


def device_sha256(t, chunk=1 << 28):
    """SHA-256 of a device tensor's bytes, streamed to the host in 256 MiB pieces."""
    h = hashlib.sha256()
    flat = t.view(-1)
    for lo in range(0, flat.numel(), chunk):
        h.update(flat[lo:lo + chunk].cpu().numpy().data)
    return h.hexdigest()


def test_full_size_round_trip(dev, fullsize):
    # configs[1] size: 100k x 64 KiB device-resident.  The whole wire body must hash to the CPU
    # oracle's SHA-256 of the same 100k blocks (tests/golden/make_fullsize.py: every block
    # regenerated and sealed on the CPU), plus round trip and sampled blocks against the oracle
    p = fullsize["config1_object"]
    nb = p["blocks"]
    key = bytes.fromhex(p["key"])
    n0 = bytes.fromhex(p["nonce0"])
    assert (key, n0, nb) == (splitmix64_bytes(41, 32), splitmix64_bytes(42, 24), 100_000)
    plain = torch.empty(nb * 65536, dtype=torch.uint8, device="cuda")
    dev.fill_random(plain, p["seed"])
    body = dev.seal_object(key, n0, plain)
    torch.cuda.synchronize()
    assert device_sha256(body) == p["wire_sha256"]
    from rclone_amd.objectset import tag_digest
    d0, d1 = [int(x) & (2**64 - 1) for x in tag_digest(body, nb).tolist()]
    assert f"{d1:016x}{d0:016x}" == p["tag_digest"]
    out, ok = dev.open_object(key, n0, body)
    assert bool(torch.equal(out, plain))
    assert int(ok.sum()) == nb
    # sampled blocks bit-exact against the oracle
    host_plain = plain.view(nb, 65536)
    host_body = body.view(nb, 65552)
    for b in [0, 1, 777, 65535, 65536, nb - 1]:
        pb = host_plain[b].cpu().numpy().tobytes()
        want = orc.seal(pb, orc.nonce_add(n0, b), key)
        assert host_body[b].cpu().numpy().tobytes() == want, b
    # the device generator matches the host SplitMix64 generator
    assert host_plain[0, :4096].cpu().numpy().tobytes() == splitmix64_bytes(p["seed"], 4096)


def test_full_size_independent_objects(dev, fullsize):
    # config 2's other form: 100k one-block objects, each with its own random
    # nonce (every 97th about to carry out of byte 7), through descriptor mode; the whole wire
    # body against the CPU oracle's SHA-256 (tests/golden/make_fullsize.py), every tag verified,
    # tampered objects flagged and zero-filled, sampled objects against the oracle
    from rclone_amd import shard
    p = fullsize["config1_independent"]
    nb = p["blocks"]
    key = bytes.fromhex(p["key"])
    assert (key, nb, p["nonce_seed"], p["carry_every"]) == (splitmix64_bytes(51, 32), 100_000, 52, 97)
    nonces = np.frombuffer(splitmix64_bytes(p["nonce_seed"], nb * 24), dtype=np.uint8).reshape(nb, 24).copy()
    nonces[::p["carry_every"], :8] = 0xFF
    d = np.zeros(nb, dtype=shard.DESC_DTYPE)
    i = np.arange(nb, dtype=np.uint64)
    d["src"], d["dst"], d["len"], d["nonce"] = i * 65536, i * 65552, 65536, nonces
    dopen = d.copy()
    dopen["src"], dopen["dst"] = i * 65552, i * 65536
    plain = torch.empty(nb * 65536, dtype=torch.uint8, device="cuda")
    dev.fill_random(plain, p["seed"])
    body = torch.empty(nb * 65552, dtype=torch.uint8, device="cuda")
    dev.seal_batch(key, d, plain, body)
    torch.cuda.synchronize()
    assert device_sha256(body) == p["wire_sha256"]
    bad = [3, 97 * 5, nb // 2 + 1, nb - 1]
    tampered = body.clone().view(nb, 65552)
    for k, b in enumerate(bad):
        tampered[b, [2, 16, 40000, 65551][k]] ^= 0x21
    out = torch.empty_like(plain)
    ok = dev.open_batch(key, dopen, tampered.view(-1), out)
    okh = ok.cpu().numpy()
    assert [int(x) for x in np.nonzero(okh == 0)[0]] == bad
    o2 = out.view(nb, 65536)
    p2 = plain.view(nb, 65536)
    good = torch.ones(nb, dtype=torch.bool, device="cuda")
    good[bad] = False
    assert bool(torch.equal(o2[good], p2[good]))
    assert int(o2[~good].sum()) == 0  # zero-filled (pass_bad_blocks contract)
    hb = body.view(nb, 65552)
    for b in [0, 1, 97, 65535, nb // 2, nb - 1]:
        want = orc.seal(p2[b].cpu().numpy().tobytes(), bytes(nonces[b]), key)
        assert hb[b].cpu().numpy().tobytes() == want, b


def test_split_and_wave_paths_agree():
    # batches of <= XS_SPLIT_MAX (256) blocks run four waves per block (xs_seal_split /
    # xs_open_split), larger ones one wave per block: same bytes, tags and verdicts
    import torch
    from rclone_amd import device
    from rclone_amd.testdata import splitmix64_bytes
    from oracle import pyoracle as orc
    key = splitmix64_bytes(31, 32)
    nonce0 = bytes([0xFE] + [0xFF] * 7 + list(splitmix64_bytes(32, 16)))  # carries from block 2
    nbig = 300
    plain = splitmix64_bytes(33, nbig * 65536 + 777)
    tb = torch.from_numpy(np.frombuffer(plain, dtype=np.uint8).copy()).cuda()
    body_big = device.seal_object(key, nonce0, tb)                      # 301 blocks: wave path
    small = 200 * 65536
    body_small = device.seal_object(key, nonce0, tb[:small].clone())    # 200 blocks: split path
    one = device.seal_object(key, nonce0, tb[:65536].clone())           # 1 block: split path
    torch.cuda.synchronize()
    bb, bs = body_big.cpu().numpy().tobytes(), body_small.cpu().numpy().tobytes()
    assert bs == bb[:200 * 65552]
    assert one.cpu().numpy().tobytes() == bb[:65552]
    assert bs[:3 * 65552] == orc.encrypt_file(plain[:3 * 65536], nonce0, key)[32:]
    # open both ways, with a tampered block in each
    for nb, body in ((200, body_small.clone()), (301, body_big.clone())):
        body[65552 * 7 + 16 + 5] ^= 1
        out, ok = device.open_object(key, nonce0, body)
        torch.cuda.synchronize()
        okn = ok.cpu().numpy()[:nb]
        assert list(np.nonzero(okn == 0)[0]) == [7], nb
        o = out.cpu().numpy().tobytes()
        assert o[7 * 65536:8 * 65536] == bytes(65536)
        assert o[:7 * 65536] == plain[:7 * 65536] and o[8 * 65536:nb * 65536 - 65536] == plain[8 * 65536:nb * 65536 - 65536]


def test_wide_and_narrow_keygen_agree(dev):
    # batches of <= XS_KEYGEN_WIDE_MAX (16) blocks build their key schedules with one wave per
    # block (xs_keygen_wide: table entries by square-and-multiply), larger ones with one lane per
    # block (the multiply chains): the sealed bytes and verdicts must not depend on which.
    # Tail lengths cover the partial-block tables, the ks1024 words (len > 65504) and a full block.
    key = splitmix64_bytes(41, 32)
    n0 = bytes([0xFD] + [0xFF] * 15 + list(splitmix64_bytes(42, 8)))  # nonce carries at block 3
    big = 300
    for tail in (1, 31, 32, 33, 4096, 65503, 65504, 65505, 65535, 65536):
        plain = splitmix64_bytes(43 + tail, big * 65536 + tail)
        whole = to_bytes(dev.seal_object(key, n0, to_dev(plain)))          # 301 blocks: narrow
        part = dev.seal_object(key, n0, to_dev(plain[big * 65536:]), first_block=big)  # 1 block: wide
        pb = to_bytes(part)
        assert pb == whole[big * 65552:], tail
        two = to_bytes(dev.seal_object(key, n0, to_dev(plain[(big - 1) * 65536:]), first_block=big - 1))
        assert two == whole[(big - 1) * 65552:], tail
        if tail in (33, 65505, 65536):
            bad = to_dev(pb)
            bad[16 + tail // 2] ^= 0x40
            out, ok = dev.open_object(key, n0, bad, first_block=big)
            assert to_bytes(ok)[:1] == b"\x00" and to_bytes(out) == bytes(tail), tail
            out, ok = dev.open_object(key, n0, part, first_block=big)
            assert to_bytes(out) == plain[big * 65536:] and to_bytes(ok)[:1] == b"\x01", tail
