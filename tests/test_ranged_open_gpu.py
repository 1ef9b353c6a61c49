"""xs_engine_open_range: a ranged read decrypts only the 4 KiB groups its reads can reach.

The decrypter opens the block a RangeSeek lands in (cipher.go:972-1034) knowing that Reads will
serve plaintext bytes [discard, discard + limit) of it at most.  Through xs_engine_open_range the
fused kernel (xs_crypt_fused2) then runs the keystream over the 4 KiB groups covering that range
only, while the Poly1305 tag is still computed over the whole block.  Checked against the oracle,
with XS_FUSED_MAX=0 (no fused kernel: every byte written) as the control: bytes inside the range
and every verdict equal the oracle's, a tampered block is zero-filled whole, and -- for the fused
kernel on full blocks -- groups outside the window keep the caller's sentinel bytes (the window
was honoured, not just tolerated).
"""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import ctypes, json, random, sys
sys.path.insert(0, %(root)r)
from rclone_amd import _lib
from rclone_amd.testdata import splitmix64_bytes
from oracle import pyoracle as orc

L = _lib.lib()
e = L.xs_engine_create(0, 64, 3)
assert e
fused = %(fused)d
rng = random.Random(0x5EED)
key = splitmix64_bytes(91, 32)
bad, cases, skipped_groups = [], 0, 0
G = 4096
for nblk, tail in ((1, 0), (2, 0), (3, 1000), (5, 0), (16, 0), (1, 40000), (2, 65535)):
    n = (nblk - 1) * 65536 + (tail if tail else 65536)
    plain = splitmix64_bytes(7000 + nblk + tail, n)
    nonce0 = splitmix64_bytes(8000 + nblk + tail, 24)
    first = nblk %% 3
    want = b"".join(orc.seal(plain[j:j + 65536], orc.nonce_add(nonce0, first + j // 65536), key)
                    for j in range(0, n, 65536))
    ranges = [(0, n), (0, 0), (n, n + 5), (0, 1), (n - 1, n), (4095, 4097), (8192, 12288), (65000, 70000),
              (123, 123 + 4096), (65536 * (nblk - 1) + 17, n)]
    for _ in range(12):
        lo = rng.randrange(0, n)
        ranges.append((lo, lo + rng.choice((1, 100, 4096, 8191, 20000, 70000))))
    for lo, hi in ranges:
        for tamper in (None, "tag", "ct"):
            wire = bytearray(want)
            hit = None
            if tamper == "tag":
                hit = rng.randrange(nblk)
                wire[hit * 65552 + 7] ^= 0x10
            elif tamper == "ct":
                hit = rng.randrange(nblk)
                blen = min(65552, len(wire) - hit * 65552)
                wire[hit * 65552 + 16 + rng.randrange(blen - 16)] ^= 0x02
            win = L.xs_host_alloc(len(wire))
            out = L.xs_host_alloc(n)
            ctypes.memmove(win, bytes(wire), len(wire))
            ctypes.memset(out, 0xEE, n)
            ok = (ctypes.c_uint8 * nblk)()
            rc = L.xs_engine_open_range(e, key, nonce0, first, win, len(wire), out, ok, lo, hi)
            got = ctypes.string_at(out, n)
            L.xs_host_free(win)
            L.xs_host_free(out)
            cases += 1
            if rc != 0:
                bad.append(("rc", nblk, tail, lo, hi, tamper)); continue
            fails = [j for j in range(nblk) if not ok[j]]
            if fails != ([] if hit is None else [hit]):
                bad.append(("verdict", nblk, tail, lo, hi, tamper, fails)); continue
            for j in range(nblk):
                b0, b1 = j * 65536, min(n, (j + 1) * 65536)
                if j == hit:
                    if got[b0:b1] != bytes(b1 - b0):
                        bad.append(("zero-fill", nblk, tail, lo, hi, tamper, j))
                    continue
                a, z = max(lo, b0), min(hi, b1)
                if a < z and got[a:z] != plain[a:z]:
                    bad.append(("bytes", nblk, tail, lo, hi, tamper, j))
                if fused and b1 - b0 == 65536:  # full block on the fused path: the window is honoured
                    for g in range(16):
                        # group g = keystream blocks 64g..64g+63 = plaintext [4096g - 32, 4096g + 4064)
                        g0, g1 = b0 + max(0, g * G - 32), b0 + (g + 1) * G - 32
                        if g1 <= lo or g0 >= hi:
                            if got[g0:g1] != b"\xee" * (g1 - g0):
                                bad.append(("outside written", nblk, tail, lo, hi, tamper, j, g)); break
                            skipped_groups += 1
L.xs_engine_destroy(e)
print(json.dumps({"bad": bad[:10], "nbad": len(bad), "cases": cases, "skipped_groups": skipped_groups}))
"""


def _run(fused_max, knobs=None):
    env = dict(os.environ, XS_FUSED_MAX=str(fused_max), XS_ENGINE_ZERO_COPY="1", **(knobs or {}))
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT, "fused": 1 if fused_max else 0}],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("fused_max,knobs", [(16, None), (0, None), (16, {"XS_KEY_PRE_MAX": "0"}),
                                             (0, {"XS_SPLIT_MAX": "0"})],
                         ids=["fused", "two_launch", "fused_no_host_key", "two_launch_no_split"])
def test_ranged_open_matches_oracle(fused_max, knobs):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    v = _run(fused_max, knobs)
    assert v["bad"] == [], (v["nbad"], v["bad"])
    assert v["cases"] > 400
    if fused_max:
        assert v["skipped_groups"] > 1000  # the fused kernel really skipped groups outside the windows
