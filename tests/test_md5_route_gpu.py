"""Long objects off the GPU MD5 lanes (VERDICT r01 "missing" 2 / "next" 5).

The ciphertext MD5 that Fs.put tees (backend/crypt/crypt.go:516-533) and cryptcheck recomputes
(crypt.go:784-806) is one dependency chain per object: on the GPU one lane per object (~70 MB/s),
so a group of objects lasts as long as its longest one.  The engine hashes the longest objects of
a group on host cores instead (one core ~10x a lane), over the wire body the GPU sealed, while the
other objects keep their lanes.  Digests must equal hashlib.md5 over the oracle's crypt files.
"""
import ctypes
import hashlib
import time

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

LANE_BPS = 70e6  # one GPU MD5 lane


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _stage(sizes, seed):
    rng = np.random.default_rng(seed)
    offs, pos = [], 0
    for n in sizes:
        offs.append(pos)
        pos += (n + 15) & ~15
    stage = np.empty(pos + 16, dtype=np.uint8)
    stage[:] = rng.integers(0, 256, stage.size, dtype=np.uint8)
    nonces = rng.integers(0, 256, 24 * len(sizes), dtype=np.uint8).tobytes()
    return stage, offs, nonces


def _want(stage, offs, sizes, nonces, key, idx):
    out = {}
    for i in idx:
        p = stage[offs[i]:offs[i] + sizes[i]].tobytes()
        out[i] = hashlib.md5(orc.encrypt_file(p, nonces[24 * i:24 * i + 24], key)).digest()
    return out


def _run(L, e, fn, key, sizes, offs, nonces, stage, body=None):
    n = len(sizes)
    u64s = ctypes.c_uint64 * n
    lens_c, offs_c = u64s(*sizes), u64s(*offs)
    md5 = (ctypes.c_uint8 * (16 * n))()
    src = ctypes.c_void_p(stage.ctypes.data)
    t0 = time.perf_counter()
    if body is None:
        rc = fn(e, key, n, nonces, offs_c, lens_c, src, md5)
    else:
        rc = fn(e, key, n, nonces, offs_c, lens_c, src, body, md5)
    dt = time.perf_counter() - t0
    assert rc == 0
    return bytes(md5), dt


def test_512mib_object_among_10k_small():
    from rclone_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.integers(1, 65536 * 2, 10_000)]
    big = 5_000
    sizes[big] = 512 << 20
    sizes[17] = 0
    stage, offs, nonces = _stage(sizes, 11)
    key = splitmix64_bytes(12, 32)
    e = L.xs_engine_create(0, 256, 1)
    assert e
    try:
        L.xs_engine_seal_md5(e, key, 1, nonces, (ctypes.c_uint64 * 1)(0), (ctypes.c_uint64 * 1)(4096),
                             ctypes.c_void_p(stage.ctypes.data), (ctypes.c_uint8 * 16)())  # warm-up
        dig, dt = _run(L, e, L.xs_engine_seal_md5, key, sizes, offs, nonces, stage)
        st = (ctypes.c_uint64 * 3)()
        L.xs_engine_md5_stats(e, st)
        # put_batch: the bodies come back, the long object is hashed from them
        total = L.xs_put_body_bytes(len(sizes), (ctypes.c_uint64 * len(sizes))(*sizes))
        body = np.empty(total + 16, dtype=np.uint8)
        dig2, dt2 = _run(L, e, L.xs_engine_put_batch, key, sizes, offs, nonces, stage,
                         ctypes.c_void_p(body.ctypes.data))
    finally:
        L.xs_engine_destroy(e)
    assert st[0] >= 1 and st[1] >= (512 << 20), list(st)  # the long object went to the host
    lane_time = (512 << 20) / LANE_BPS
    print(f"seal_md5 {dt:.2f} s, put_batch {dt2:.2f} s, one GPU lane would take {lane_time:.1f} s")
    assert dt < lane_time / 2 and dt2 < lane_time / 2
    check = sorted({0, 1, 17, big - 1, big, big + 1, len(sizes) - 1} | set(range(0, len(sizes), 997)))
    want = _want(stage, offs, sizes, nonces, key, check)
    for i in check:
        assert dig[16 * i:16 * i + 16] == want[i], i
        assert dig2[16 * i:16 * i + 16] == want[i], i
    assert dig == dig2
    # the packed body of the long object is the oracle's ciphertext
    bpos = sum(((n + 16 * ((n + 65535) // 65536)) + 15) & ~15 for n in sizes[:big])
    ct = orc.encrypt_file(stage[offs[big]:offs[big] + sizes[big]].tobytes(), nonces[24 * big:24 * big + 24], key)
    assert body[bpos:bpos + len(ct) - 32].tobytes() == ct[32:]


def test_host_routing_shortens_the_group():
    # the same group with every object on the GPU lanes (threads = 0) vs routed: identical
    # digests, and the routed group no longer waits for the 64 MiB object's lane
    from rclone_amd import _lib
    L = _lib.lib()
    sizes = [64 << 20] + [4096 + 37 * k for k in range(2000)]
    stage, offs, nonces = _stage(sizes, 21)
    key = splitmix64_bytes(22, 32)
    e = L.xs_engine_create(0, 256, 1)
    try:
        _run(L, e, L.xs_engine_seal_md5, key, sizes[1:50], offs[1:50], nonces[24:24 * 50], stage)  # warm-up
        L.xs_engine_set_host_md5(e, 0)
        lane, t_lane = _run(L, e, L.xs_engine_seal_md5, key, sizes, offs, nonces, stage)
        L.xs_engine_set_host_md5(e, 4)
        routed, t_routed = _run(L, e, L.xs_engine_seal_md5, key, sizes, offs, nonces, stage)
    finally:
        L.xs_engine_destroy(e)
    print(f"all on GPU lanes {t_lane:.3f} s, long object on the host {t_routed:.3f} s")
    assert lane == routed
    want = _want(stage, offs, sizes, nonces, key, [0, 1, 1000, 2000])
    for i, w in want.items():
        assert routed[16 * i:16 * i + 16] == w
    assert t_routed < t_lane / 2
