#!/usr/bin/env python3
"""Oracle pins for the full-size synthetic workloads -> tests/golden/fullsize.json.

TEST INFRASTRUCTURE, run in the build container (CPU only, a few minutes on 8 cores):

    python tests/golden/make_fullsize.py [--quick]

The GPU runs generate their plaintext in HBM (xs_fill_blocks_dev: SplitMix64 keyed by the global
block id, rclone_amd/testdata.py) and seal block g with nonce0 + g (nonce.add + secretbox.Seal,
/root/reference/backend/crypt/cipher.go:665-678, :737).  Here the CPU oracle regenerates the same
plaintext and seals every block (oracle/xsalsa_simd.c orc_simd_seal_gen, itself checked against
the scalar oracle oracle/xsalsa_oracle.c by tests/test_oracle_simd.py, which the reference's own
vectors pin: tests/test_oracle.py), so the GPU's full-size outputs are compared with numbers the
GPU never produced:

* configs[3]: the 2^24-block (1 TiB) object of rclone_amd.objectset (CONFIG3_*): the
  order-independent tag digest (sum mod 2^64 of each tag's two 64-bit halves) that
  tests/test_objectset_gpu.py and bench.py's objectset leg report for any world size;
* configs[1], one object: tests/test_gpu_parity.py::test_full_size_round_trip's 100 000 blocks:
  SHA-256 of the whole wire body (100 000 x 65 552 bytes) and its tag digest;
* configs[1], independent objects: test_full_size_independent_objects' 100 000 one-block
  objects, each with its own nonce: SHA-256 of the wire body and tag digest;
* the bench headline: bench.py's resident set at --blocks 100000 for 1, 2, 4 and 8 ranks (the
  ranks' shares of one 100000*N-block object): the tag digest summed over ranks.

The parameters of every workload are written beside its pins; the tests read them from the file.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as orc  # noqa: E402
from rclone_amd.objectset import CONFIG3_BLOCKS, CONFIG3_KEY, CONFIG3_NONCE0, CONFIG3_SEED  # noqa: E402
from rclone_amd.testdata import splitmix64_block, splitmix64_bytes  # noqa: E402

BLOCK_SIZE = 65552
OUT = os.path.join(HERE, "fullsize.json")

# tests/test_gpu_parity.py's configs[1] workloads
C1_BLOCKS = 100_000
C1_OBJECT = {"blocks": C1_BLOCKS, "seed": 0x5EED, "key": splitmix64_bytes(41, 32).hex(),
             "nonce0": splitmix64_bytes(42, 24).hex()}
C1_INDEP = {"blocks": C1_BLOCKS, "seed": 0x0B1EC7, "key": splitmix64_bytes(51, 32).hex(),
            "nonce_seed": 52, "carry_every": 97}


def indep_nonces(p):
    """Nonce j = bytes 24j..24j+23 of SplitMix64(nonce_seed); every carry_every-th one has its low
    8 bytes set to 0xFF (about to carry out of byte 7)."""
    nb = p["blocks"]
    n = np.frombuffer(splitmix64_bytes(p["nonce_seed"], nb * 24), dtype=np.uint8).reshape(nb, 24).copy()
    n[::p["carry_every"], :8] = 0xFF
    return n


def hexdigest(s):
    return "%016x%016x" % (s[1] & (2**64 - 1), s[0] & (2**64 - 1))


def add(a, b):
    return ((a[0] + b[0]) & (2**64 - 1), (a[1] + b[1]) & (2**64 - 1))


def sealed_sha256(nb, seed, key, nonce0=bytes(24), nonces=None, chunk=2048):
    """SHA-256 of the wire body of blocks 0..nb-1 (contiguous stream of seed) and its tag digest."""
    h = hashlib.sha256()
    tot = (0, 0)
    buf = np.empty(chunk * BLOCK_SIZE, dtype=np.uint8)
    for lo in range(0, nb, chunk):
        n = min(chunk, nb - lo)
        s, _ = orc.seal_gen(n, lo, 1, seed, nonce0, key, out=buf,
                            nonces=None if nonces is None else np.ascontiguousarray(nonces[lo:lo + n]))
        h.update(memoryview(buf)[:n * BLOCK_SIZE])
        tot = add(tot, s)
    return h.hexdigest(), hexdigest(tot)


def digest_range(first, nb, seed, nonce0, key, chunk=1 << 18, label=""):
    tot = (0, 0)
    t0 = time.time()
    for lo in range(0, nb, chunk):
        n = min(chunk, nb - lo)
        s, _ = orc.seal_gen(n, first + lo, 1, seed, nonce0, key)
        tot = add(tot, s)
        if label:
            done = lo + n
            print(f"  {label}: {done}/{nb} blocks, {done * 65536 / 2**30 / (time.time() - t0):.2f} GiB/s",
                  flush=True)
    return tot


def self_check():
    """orc_simd_seal_gen against the scalar oracle and the Python generator on sampled blocks."""
    key, n0, seed = CONFIG3_KEY, CONFIG3_NONCE0, CONFIG3_SEED
    buf = np.empty(3 * BLOCK_SIZE, dtype=np.uint8)
    first, stride = (1 << 24) - 7, 3
    orc.seal_gen(3, first, stride, seed, n0, key, out=buf)
    for j in range(3):
        g = first + j * stride
        assert orc.gen_block(seed, g) == splitmix64_block(seed, g)
        want = orc.seal(splitmix64_block(seed, g), orc.nonce_add(n0, g), key)
        assert buf[j * BLOCK_SIZE:(j + 1) * BLOCK_SIZE].tobytes() == want, g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="skip the 1 TiB configs[3] digest (keeps the old value)")
    args = ap.parse_args()
    import bench  # the headline workload's constants
    self_check()
    old = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            old = json.load(f)
    res = {"generator": "tests/golden/make_fullsize.py (oracle/xsalsa_simd.c orc_simd_seal_gen, CPU)",
           "contract": "/root/reference/backend/crypt/cipher.go:665-678 (nonce.add), :737 (secretbox.Seal)",
           "tag_digest": "hex(hi || lo): sum mod 2^64 over every block of the tag's low and high "
                         "little-endian 64-bit halves (rclone_amd/objectset.py tag_digest)"}
    t0 = time.time()
    # bench headline, worlds 1/2/4/8: blocks 0..100000*N-1 of one object
    nb = 100_000
    hl = {"blocks_per_rank": nb, "seed": bench.HEADLINE_SEED, "key": bench.HEADLINE_KEY.hex(),
          "nonce0": bench.HEADLINE_NONCE0.hex(), "tag_digest": {}}
    tot, done = (0, 0), 0
    for world in (1, 2, 4, 8):
        tot = add(tot, digest_range(done, world * nb - done, bench.HEADLINE_SEED, bench.HEADLINE_NONCE0,
                                    bench.HEADLINE_KEY))
        done = world * nb
        hl["tag_digest"][str(world)] = hexdigest(tot)
    res["bench_headline"] = hl
    print(f"headline digests in {time.time() - t0:.0f} s", flush=True)
    # configs[1] one object
    p = dict(C1_OBJECT)
    p["wire_sha256"], p["tag_digest"] = sealed_sha256(p["blocks"], p["seed"], bytes.fromhex(p["key"]),
                                                      bytes.fromhex(p["nonce0"]))
    res["config1_object"] = p
    # configs[1] independent objects
    q = dict(C1_INDEP)
    q["wire_sha256"], q["tag_digest"] = sealed_sha256(q["blocks"], q["seed"], bytes.fromhex(q["key"]),
                                                      nonces=indep_nonces(q))
    res["config1_independent"] = q
    print(f"configs[1] pins in {time.time() - t0:.0f} s", flush=True)
    c3 = {"blocks": CONFIG3_BLOCKS, "seed": CONFIG3_SEED, "key": CONFIG3_KEY.hex(), "nonce0": CONFIG3_NONCE0.hex()}
    if args.quick:
        c3["tag_digest"] = old.get("config3", {}).get("tag_digest")
    else:
        t1 = time.time()
        c3["tag_digest"] = hexdigest(digest_range(0, CONFIG3_BLOCKS, CONFIG3_SEED, CONFIG3_NONCE0, CONFIG3_KEY,
                                                  label="configs[3]"))
        c3["cpu_seconds"] = round(time.time() - t1, 1)
    res["config3"] = c3
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1)
        f.write("\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
