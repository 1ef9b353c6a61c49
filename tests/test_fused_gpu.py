"""The fused small-batch kernels (ranged reads: keygen + crypt in one launch).

Tiny zero-copy engine batches (one key, one direction, <= XS_FUSED_MAX blocks) run one launch
(xs_crypt_fused2: eight crypt waves overlap the keystream with the key-schedule wave and run the
matrix-core Poly1305 over the LDS-resident ciphertext afterwards).  With XS_FUSED_MAX=0 the same
batches take two launches instead (keygen, then the four-wave split crypt).  Both must give the
oracle's bytes, tags and verdicts for every tail length, carry nonces, first_block offsets,
multi-block batches and tampered tags / ciphertext / nonces, and the same digest.  Each setting
runs in its own process (the threshold is read once per process).
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
import ctypes, hashlib, json, sys
sys.path.insert(0, %(root)r)
from rclone_amd import _lib
from rclone_amd.testdata import splitmix64_bytes
from oracle import pyoracle as orc

L = _lib.lib()
e = L.xs_engine_create(0, 64, 3)
assert e

class Pinned:
    def __init__(self, data_or_len):
        n = data_or_len if isinstance(data_or_len, int) else len(data_or_len)
        self.n, self.p = n, L.xs_host_alloc(max(n, 1))
        if not isinstance(data_or_len, int):
            ctypes.memmove(self.p, bytes(data_or_len), n)
    def raw(self):
        return ctypes.string_at(self.p, self.n)

def expected(plain, nonce0, first, key):
    return b"".join(orc.seal(plain[j:j + 65536], orc.nonce_add(nonce0, first + j // 65536), key)
                    for j in range(0, len(plain), 65536))

h = hashlib.sha256()
bad = []
cases = 0
key = splitmix64_bytes(71, 32)
for nblk in (1, 2, 5, 16):
    for tail in (0, 1, 15, 16, 17, 31, 32, 33, 4096, 65503, 65504, 65505, 65535):
        n = (nblk - 1) * 65536 + (tail if tail else 65536)
        if n <= 0:
            continue
        plain = splitmix64_bytes(1000 * nblk + tail, n)
        nonce0 = (b"\xfe" + b"\xff" * 15 + splitmix64_bytes(nblk + tail, 8)) if tail %% 2 else splitmix64_bytes(3 + tail, 24)
        first = (tail * 7) %% 5
        src, body = Pinned(plain), Pinned(n + 16 * nblk)
        if L.xs_engine_seal(e, key, nonce0, first, src.p, n, body.p) != 0:
            bad.append(("seal rc", nblk, tail)); continue
        want = expected(plain, nonce0, first, key)
        got = body.raw()
        if got != want:
            bad.append(("seal", nblk, tail))
        h.update(got)
        # open: clean, then tag / ciphertext tampered in one block
        for tamper in (None, "tag", "ct", "last"):
            wire = bytearray(want)
            hit = None
            if tamper == "tag":
                hit = nblk // 2
                wire[hit * 65552 + 3] ^= 0x20
            elif tamper == "ct":
                hit = 0
                wire[16 + (len(wire) - 17) %% 60000] ^= 0x01
            elif tamper == "last":
                hit = nblk - 1
                wire[-1] ^= 0x80
            win, out = Pinned(wire), Pinned(n)
            ok = (ctypes.c_uint8 * nblk)()
            if L.xs_engine_open(e, key, nonce0, first, win.p, len(wire), out.p, ok) != 0:
                bad.append(("open rc", nblk, tail, tamper)); continue
            exp = bytearray(plain)
            if hit is not None:
                exp[hit * 65536:(hit + 1) * 65536] = bytes(len(exp[hit * 65536:(hit + 1) * 65536]))
            fails = [j for j in range(nblk) if not ok[j]]
            if fails != ([] if hit is None else [hit]) or out.raw() != bytes(exp):
                bad.append(("open", nblk, tail, tamper, fails))
            h.update(out.raw() + bytes(ok))
            cases += 1
# concurrent single-block opens (ranged reads of many readers): coalesced into multi-request fused
# batches of one key and direction; every caller's bytes and verdict checked.  The objects sit
# 16 MiB apart in one 3 GiB pinned arena, so a batch's buffer offsets from its lowest address
# reach past 2 GiB (bit 31 of the low word set)
import threading
errs = []
objs = []
ARENA = 3 << 30
arena = L.xs_host_alloc(ARENA)
assert arena
class View:
    def __init__(self, off, data_or_len):
        n = data_or_len if isinstance(data_or_len, int) else len(data_or_len)
        assert off + n <= ARENA
        self.n, self.p = n, arena + off
        if not isinstance(data_or_len, int):
            ctypes.memmove(self.p, bytes(data_or_len), n)
    def raw(self):
        return ctypes.string_at(self.p, self.n)
for t in range(16):
    for k in range(12):
        n = 65536 if (t + k) %% 3 else 1000 + 37 * t
        plain = splitmix64_bytes(50000 + 100 * t + k, n)
        nonce0 = splitmix64_bytes(60000 + 100 * t + k, 24)
        wire = bytearray(expected(plain, nonce0, k, key))
        if k %% 5 == 0:
            wire[16 + n // 2] ^= 4
        slot = (t * 12 + k) * (16 << 20)  # each reader its own 192 MiB: concurrent readers far apart
        objs.append((t, k, n, plain, nonce0, View(slot, wire), View(slot + (8 << 20), n), (ctypes.c_uint8 * 1)()))
def reader(t):
    for (tt, k, n, plain, nonce0, win, out, ok) in objs:
        if tt != t:
            continue
        for rep in range(4):
            if L.xs_engine_open(e, key, nonce0, k, win.p, win.n, out.p, ok) != 0:
                errs.append(("open rc", t, k)); continue
            good = k %% 5 != 0
            if ok[0] != good or out.raw() != (plain if good else bytes(n)):
                o = out.raw()
                first = next((i for i in range(n) if o[i] != (plain[i] if good else 0)), -1)
                errs.append(("open", t, k, n, ok[0], first))
s0 = (ctypes.c_uint64 * 3)()
L.xs_engine_stats(e, s0)
th = [threading.Thread(target=reader, args=(t,)) for t in range(16)]
[x.start() for x in th]
[x.join() for x in th]
s1 = (ctypes.c_uint64 * 3)()
L.xs_engine_stats(e, s1)
conc = {"batches": s1[0] - s0[0], "requests": s1[1] - s0[1]}
bad += errs
L.xs_host_free(arena)
st = (ctypes.c_uint64 * 3)()
L.xs_engine_stats(e, st)
L.xs_engine_destroy(e)
print(json.dumps({"bad": bad[:10], "nbad": len(bad), "cases": cases, "digest": h.hexdigest(), "concurrent": conc}))
"""


def _run(fused_max, **knobs):
    # the leader holds new requests while a batch is in flight and express lanes are off, so the
    # concurrent phase forms multi-request fused batches (the path this test is about)
    env = dict(os.environ, XS_FUSED_MAX=str(fused_max), XS_ENGINE_ZERO_COPY="1", XS_ENGINE_COALESCE="1",
               XS_ENGINE_OVERLAP="0", XS_EXPRESS_MAX="0", **{k: str(v) for k, v in knobs.items()})
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT}], capture_output=True, text=True, timeout=240,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(600)
def test_fused_and_two_launch_paths_agree_with_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    # the launch path's operator knobs: the defaults, no fused kernel, the fused
    # kernel without the host key setup (XS_KEY_PRE_MAX=0), and two launches with the one-wave
    # crypt kernels even for the smallest batches (XS_SPLIT_MAX=0): the same bytes and verdicts
    fused, split = _run(16), _run(0)
    nopre, nosplit = _run(16, XS_KEY_PRE_MAX=0), _run(0, XS_SPLIT_MAX=0)
    for v in (fused, split, nopre, nosplit):
        assert v["bad"] == [], (v["nbad"], v["bad"])
    assert fused["concurrent"]["batches"] < fused["concurrent"]["requests"]  # the concurrent opens did coalesce
    assert fused["cases"] == split["cases"] == nopre["cases"] == nosplit["cases"] > 150
    assert fused["digest"] == split["digest"] == nopre["digest"] == nosplit["digest"]


def test_first_fused_open_on_fresh_engines_reports_tampering():
    # the pinned completion word must start cleared on every new engine, or the first
    # fused batch could be taken as done before its kernel ran (stale verdicts).  Engines are
    # created and destroyed repeatedly (pinned memory is recycled between them, after being
    # filled with the first sequence number), and the very first operation on each is a
    # tampered one-block open.
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes

    from oracle import pyoracle as orc
    from rclone_amd import _lib
    from rclone_amd.testdata import splitmix64_bytes
    L = _lib.lib()
    key, nonce = splitmix64_bytes(81, 32), splitmix64_bytes(82, 24)
    plain = splitmix64_bytes(83, 65536)
    good = orc.seal(plain, nonce, key)
    bad = bytearray(good)
    bad[5] ^= 0x40  # the tag
    win = L.xs_host_alloc(len(good))
    out = L.xs_host_alloc(65536)
    try:
        for rep in range(6):
            junk = L.xs_host_alloc(1 << 16)  # recycled pinned memory holding the value 1
            ctypes.memset(junk, 1, 1 << 16)
            L.xs_host_free(junk)
            e = L.xs_engine_create(0, 64, 3)
            assert e
            try:
                ok = (ctypes.c_uint8 * 1)(1)
                ctypes.memmove(win, bytes(bad), len(bad))
                ctypes.memset(out, 0x5A, 65536)
                assert L.xs_engine_open(e, key, nonce, 0, win, len(bad), out, ok) == 0
                assert ok[0] == 0, rep
                assert ctypes.string_at(out, 65536) == bytes(65536), rep  # zero-filled
                ctypes.memmove(win, good, len(good))
                assert L.xs_engine_open(e, key, nonce, 0, win, len(good), out, ok) == 0
                assert ok[0] == 1 and ctypes.string_at(out, 65536) == plain, rep
            finally:
                L.xs_engine_destroy(e)
    finally:
        L.xs_host_free(win)
        L.xs_host_free(out)
