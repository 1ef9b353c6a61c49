"""The CPU oracle's pins of the full-size workloads (tests/golden/fullsize.json, written by
tests/golden/make_fullsize.py) are what the GPU tests and bench.py hold the GPU to.  Here, on the
CPU: the file's parameters are the ones the GPU runs use, the generator + sealer it was made with
agrees with the scalar oracle and the Python generator, and one pin is recomputed end to end (the
bench headline set at one rank: 100 000 blocks regenerated and sealed, tag digest summed).
Contract: /root/reference/backend/crypt/cipher.go:665-678 (nonce.add), :737 (secretbox.Seal)."""
import importlib.util
import os

import numpy as np

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_block, splitmix64_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod(name, path):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_pins_match_the_runs_parameters(fullsize):
    from rclone_amd import objectset
    bench = _mod("bench_pins", "bench.py")
    c3 = fullsize["config3"]
    assert (c3["blocks"], c3["seed"], bytes.fromhex(c3["key"]), bytes.fromhex(c3["nonce0"])) == (
        objectset.CONFIG3_BLOCKS, objectset.CONFIG3_SEED, objectset.CONFIG3_KEY, objectset.CONFIG3_NONCE0)
    assert objectset.CONFIG3_TAG_DIGEST == c3["tag_digest"] and len(c3["tag_digest"]) == 32
    hl = fullsize["bench_headline"]
    assert (hl["blocks_per_rank"], hl["seed"], bytes.fromhex(hl["key"]), bytes.fromhex(hl["nonce0"])) == (
        100_000, bench.HEADLINE_SEED, bench.HEADLINE_KEY, bench.HEADLINE_NONCE0)
    assert sorted(hl["tag_digest"]) == ["1", "2", "4", "8"]
    assert len(set(hl["tag_digest"].values())) == 4
    for k in ("config1_object", "config1_independent"):
        assert len(fullsize[k]["wire_sha256"]) == 64 and fullsize[k]["blocks"] == 100_000


def test_generator_and_sealer_agree_with_the_scalar_oracle():
    gen = _mod("make_fullsize", "tests/golden/make_fullsize.py")
    gen.self_check()
    # per-block nonces (the independent-object form) and a stride
    key, seed = splitmix64_bytes(7, 32), 99
    nonces = np.frombuffer(splitmix64_bytes(8, 5 * 24), dtype=np.uint8).reshape(5, 24).copy()
    nonces[0, :8] = 0xFF
    out = np.empty(5 * 65552, dtype=np.uint8)
    s, _ = orc.seal_gen(5, 11, 4, seed, bytes(24), key, out=out, nonces=nonces)
    tot = [0, 0]
    for j in range(5):
        want = orc.seal(splitmix64_block(seed, 11 + 4 * j), bytes(nonces[j]), key)
        assert out[j * 65552:(j + 1) * 65552].tobytes() == want
        tot[0] += int.from_bytes(want[:8], "little")
        tot[1] += int.from_bytes(want[8:16], "little")
    assert s == (tot[0] % 2**64, tot[1] % 2**64)


def test_headline_world1_pin_recomputed(fullsize):
    bench = _mod("bench_pins2", "bench.py")
    gen = _mod("make_fullsize2", "tests/golden/make_fullsize.py")
    s = gen.digest_range(0, 100_000, bench.HEADLINE_SEED, bench.HEADLINE_NONCE0, bench.HEADLINE_KEY)
    assert gen.hexdigest(s) == fullsize["bench_headline"]["tag_digest"]["1"]
