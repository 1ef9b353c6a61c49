"""A failing combined batch reaches every caller it carried.

The engine packs concurrent callers' requests into one combined batch and hands the batch's
result to every request in it (rclone_amd/csrc/xs_api.cpp engine_submit).  The reference returns
a failing refill's error to the stream that made it and keeps it sticky (cipher.go:748-758,
:1042-1052); here the stream layer gets that error from the engine, so every follower of a failed
batch must see it, and nobody else.  librclone_crypt_testhooks.so (xs_api.cpp under
-DXS_TEST_HOOKS; test-only, rclone_amd/build.py) fails the first combined batch of >= 2 requests
before any launch, as a HIP error would.  Twelve threads seal and open through one engine; the
test checks that the failed calls are exactly the batch's requests (XS_ERR_HIP each), that every
other call equals the CPU oracle, and that the engine keeps working afterwards.  Both the staged
(H2D/D2H) and the zero-copy batch forms are run.  The stream-level half (RC_ERR_GPU at the exact
refill, no byte of the failed batch served, sticky error, clean close) runs on the CPU under
ASan/TSan with the stub engine's failure knob (tests/native/sanitize_main.cpp test_engine_failure).
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
import ctypes, json, sys, threading
sys.path.insert(0, %(root)r)
from oracle import pyoracle as orc
from rclone_amd import _lib
from rclone_amd.testdata import splitmix64_bytes
L = _lib.hooks_lib()
e = L.xs_engine_create(0, 64, 2)
assert e, _lib.last_error()
key = splitmix64_bytes(91, 32)
T, R = 12, 12
calls = []  # (thread, rep, op, rc, good)
lock = threading.Lock()
bar = threading.Barrier(T)

def worker(t):
    n = 1 + t %% 3
    size = n * 65536 - 100 * t
    nb = (size + 65535) // 65536
    inp, wire, out, ok = (L.xs_host_alloc(size), L.xs_host_alloc(size + 16 * nb), L.xs_host_alloc(size),
                          L.xs_host_alloc(nb))
    bar.wait()
    for r in range(R):
        plain = splitmix64_bytes(1000 * t + r, size)
        nonce = splitmix64_bytes(5000 * t + r, 24)
        ctypes.memmove(inp, plain, size)
        rc = L.xs_engine_seal(e, key, nonce, 0, inp, size, wire)
        want = orc.encrypt_file(plain, nonce, key)[32:]
        good = rc == 0 and ctypes.string_at(wire, len(want)) == want
        with lock:
            calls.append((t, r, "seal", rc, good))
        if rc != 0:
            ctypes.memmove(wire, want, len(want))  # open the oracle's body instead
        ctypes.memset(out, 0xEE, size)
        rc = L.xs_engine_open(e, key, nonce, 0, wire, len(want), out, ok)
        good = rc == 0 and ctypes.string_at(out, size) == plain and ctypes.string_at(ok, nb) == b"\1" * nb
        with lock:
            calls.append((t, r, "open", rc, good))
    for p in (inp, wire, out, ok):
        L.xs_host_free(p)

# armed once; a round of the threads in which no batch of >= 2 requests formed (unlikely: they start
# together at a barrier) leaves it armed and every call succeeding, and another round is run
L.xs_test_fail_batch(2)
for attempt in range(5):
    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    [x.start() for x in th]
    [x.join() for x in th]
    failed_reqs = L.xs_test_failed_requests()
    if failed_reqs:
        break
    bar.reset()
R_done = attempt + 1
# the engine still works after the failure
plain = splitmix64_bytes(7, 3 * 65536)
buf, body = L.xs_host_alloc(len(plain)), L.xs_host_alloc(len(plain) + 48)
ctypes.memmove(buf, plain, len(plain))
after = L.xs_engine_seal(e, key, bytes(24), 0, buf, len(plain), body) == 0 and \
    ctypes.string_at(body, len(plain) + 48) == orc.encrypt_file(plain, bytes(24), key)[32:]
st = (ctypes.c_uint64 * 3)()
L.xs_engine_stats(e, st)
L.xs_engine_destroy(e)
fails = [c for c in calls if c[3] != 0]
print(json.dumps({"calls": len(calls), "rounds": R_done, "failed_reqs": failed_reqs, "fail_rcs": sorted({c[3] for c in fails}),
                  "nfail": len(fails), "fail_ops": sorted({c[2] for c in fails}),
                  "bad_success": [c[:3] for c in calls if c[3] == 0 and not c[4]][:10],
                  "after_ok": after, "batches": st[0], "requests": st[1]}))
"""


@pytest.mark.timeout(600)
@pytest.mark.parametrize("zero_copy", ["0", "1"], ids=["staged", "zero_copy"])
def test_failed_combined_batch_reaches_every_follower(zero_copy):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    # express lanes off and no issuing while a batch is in flight: concurrent requests queue behind
    # the leader and form multi-request combined batches
    env = dict(os.environ, XS_ENGINE_ZERO_COPY=zero_copy, XS_ENGINE_COALESCE="1", XS_ENGINE_OVERLAP="0",
               XS_EXPRESS_MAX="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT}], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    v = json.loads(r.stdout.strip().splitlines()[-1])
    print(v)
    assert v["calls"] == 12 * 12 * 2 * v["rounds"]
    assert v["batches"] < v["requests"]  # requests did combine
    assert v["failed_reqs"] >= 2, v  # the hook fired on a combined batch
    assert v["nfail"] == v["failed_reqs"] and v["fail_rcs"] == [-2], v  # exactly its requests, XS_ERR_HIP
    assert v["bad_success"] == [], v
    assert v["after_ok"]
