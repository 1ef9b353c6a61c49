"""Multi-device engine pool on the product path (VERDICT r01 "missing" 1 / "next" 4).

One rclone process runs --transfers / --checkers streams at once (fs/sync/sync.go:544
startTransfers; cryptcheck's checkers, cmd/cryptcheck/cryptcheck.go:91-114) and shards its
objects over the node's GPUs.  On the one-GPU test box the pool runs N logical engines on
device 0 ("0,0,0,0"); results must be bit-identical to one engine and equal to the oracle.
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes
from tests.go_readers import Buffer

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.fixture(scope="module")
def pool4():
    from rclone_amd import crypt
    p = crypt.EnginePool([0, 0, 0, 0], batch_blocks=64)
    yield p
    p.close()


def _objects(seed, sizes):
    plains = [splitmix64_bytes(seed + i, n) for i, n in enumerate(sizes)]
    nonces = b"".join(splitmix64_bytes(seed + 1000 + i, 24) if i % 5 else b"\xff" * 8 + splitmix64_bytes(i, 16)
                      for i in range(len(sizes)))
    offs, pos = [], 0
    for n in sizes:
        offs.append(pos)
        pos += (n + 15) & ~15
    stage = bytearray(pos + 16)
    for o, p in zip(offs, plains):
        stage[o:o + len(p)] = p
    return plains, nonces, offs, stage


SIZES = [0, 1, 15, 16, 65535, 65536, 65537, 3 * 65536 + 7, 1 << 20] + [1000 * k + 3 for k in range(1, 60)]


def test_pool_put_batch_equals_one_engine_and_oracle(pool4):
    from rclone_amd import _lib
    L = _lib.lib()
    assert len(pool4) == 4
    key = splitmix64_bytes(41, 32)
    plains, nonces, offs, stage = _objects(500, SIZES)
    n = len(SIZES)
    u64s = ctypes.c_uint64 * n
    lens_c, offs_c = u64s(*SIZES), u64s(*offs)
    total = L.xs_put_body_bytes(n, lens_c)
    src = (ctypes.c_uint8 * len(stage)).from_buffer(stage)
    body_p, md5_p = (ctypes.c_uint8 * (total + 16))(), (ctypes.c_uint8 * (16 * n))()
    assert L.xs_pool_put_batch(pool4.handle, key, n, nonces, offs_c, lens_c, src, body_p, md5_p) == 0, \
        _lib.last_error()
    body_1, md5_1 = (ctypes.c_uint8 * (total + 16))(), (ctypes.c_uint8 * (16 * n))()
    e = L.xs_engine_create(0, 64, 1)
    try:
        assert L.xs_engine_put_batch(e, key, n, nonces, offs_c, lens_c, src, body_1, md5_1) == 0
    finally:
        L.xs_engine_destroy(e)
    assert bytes(body_p)[:total] == bytes(body_1)[:total] and bytes(md5_p) == bytes(md5_1)
    raw, dig, bpos = bytes(body_p), bytes(md5_p), 0
    for i, p in enumerate(plains):
        want = orc.encrypt_file(p, nonces[24 * i:24 * i + 24], key)
        assert raw[bpos:bpos + len(want) - 32] == want[32:], (i, SIZES[i])
        assert dig[16 * i:16 * i + 16] == hashlib.md5(want).digest(), (i, SIZES[i])
        bpos += (len(want) - 32 + 15) & ~15
    # seal+MD5 only (cryptcheck): the same digests
    md5_s = (ctypes.c_uint8 * (16 * n))()
    assert L.xs_pool_seal_md5(pool4.handle, key, n, nonces, offs_c, lens_c, src, md5_s) == 0
    assert bytes(md5_s) == dig
    # every engine of the pool took a range of the objects
    for i in range(4):
        st = (ctypes.c_uint64 * 3)()
        L.xs_engine_md5_stats(pool4.engine(i), st)
        assert st[2] > 0, (i, list(st))


def test_pool_streams_spread_over_engines(pool4):
    # many encrypter / decrypter streams of one cipher bound to the pool, from 8 threads: each
    # stream takes an engine round-robin; bytes equal the oracle's
    from rclone_amd import crypt
    c = crypt.Cipher("potato", "")
    c.pool = pool4
    key = c.data_key
    before = [s[1] for s in pool4.stats()]
    errors = []

    def worker(t):
        try:
            for k in range(6):
                n = 20000 * t + 70001 * k + 1
                plain = splitmix64_bytes(9000 + 10 * t + k, n)
                nonce = splitmix64_bytes(9500 + 10 * t + k, 24)
                ct = c.encrypt_data(Buffer(plain), nonce).readall()
                if ct != orc.encrypt_file(plain, nonce, key):
                    errors.append(("enc", t, k))
                if c.decrypt_data(Buffer(ct)).readall() != plain:
                    errors.append(("dec", t, k))
        except Exception as exc:  # noqa: BLE001
            errors.append(repr(exc))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    after = [s[1] for s in pool4.stats()]
    assert all(a > b for a, b in zip(after, before)), (before, after)
    # cryptcheck batch through the same pool
    items, want = [], []
    for i, n in enumerate([0, 5, 65536, 200000, 1 << 20]):
        plain = splitmix64_bytes(777 + i, n)
        nonce = splitmix64_bytes(888 + i, 24)
        items.append((nonce, Buffer(plain)))
        want.append(hashlib.md5(orc.encrypt_file(plain, nonce, key)).digest())
    assert c.hash_batch_with_nonce(items) == want
    c.pool = None


def test_process_pool_from_env():
    # the process-wide pool follows RCLONE_AMD_DEVICES: three engines on device 0, streams and
    # names through the default (unbound) cipher
    code = r"""
import json, sys
sys.path.insert(0, %r)
from rclone_amd import _lib, crypt
from rclone_amd.testdata import splitmix64_bytes
from oracle import pyoracle as orc
from tests.go_readers import Buffer
L = _lib.lib()
c = crypt.Cipher("potato", "")
outs = []
for i in range(7):
    p = splitmix64_bytes(i, 70000 * i + 3)
    n = splitmix64_bytes(100 + i, 24)
    outs.append(c.encrypt_data(Buffer(p), n).readall() == orc.encrypt_file(p, n, c.data_key))
pool = L.rc_default_pool()
sizes = [L.xs_pool_size(pool)]
names = c.encrypt_file_names(["a/b", "c"])
print(json.dumps({"ok": all(outs), "pool": sizes[0], "names": c.decrypt_file_name(names[1]) == "c"}))
""" % ROOT
    env = dict(os.environ, RCLONE_AMD_DEVICES="0,0,0")
    env.pop("RCLONE_AMD_DEVICE", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res == {"ok": True, "pool": 3, "names": True}
