#!/usr/bin/env python3
"""Host-memory path: pinned host plaintext -> H2D -> keygen+seal -> D2H -> pinned host wire
blocks (and the reverse for open), through xs_engine (per-slot streams; copies of one batch
overlap the kernels of the next).  Reports GiB/s of plaintext, PCIe-inclusive.  This is the
DESIGN.md "host path" number; it is never bench.py's value."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--batch", type=int, default=256, help="blocks per engine slot")
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from rclone_amd import _lib
    L = _lib.lib()
    nb = int(a.gib * 2**30) // 65536
    plain_len, body_len = nb * 65536, nb * 65552
    hp = L.xs_host_alloc(plain_len)
    hb = L.xs_host_alloc(body_len)
    ho = L.xs_host_alloc(plain_len)
    ok = L.xs_host_alloc(nb)
    assert hp and hb and ho and ok, _lib.last_error()
    ctypes.memset(hp, 0x5A, plain_len)
    eng = L.xs_engine_create(0, a.batch, a.slots)
    assert eng, _lib.last_error()
    key, n0 = bytes(range(32)), bytes(24)
    res = {}
    for name, fn in (("seal", lambda: L.xs_engine_seal(eng, key, n0, 0, hp, plain_len, hb)),
                     ("open", lambda: L.xs_engine_open(eng, key, n0, 0, hb, body_len, ho, ok))):
        _lib.check(fn(), name)
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            _lib.check(fn(), name)
            best = min(best, time.perf_counter() - t0)
        res[name + "_GiB_s"] = round(plain_len / 2**30 / best, 2)
    assert ctypes.string_at(ho, 4096) == ctypes.string_at(hp, 4096)
    assert ctypes.string_at(ok, nb) == b"\x01" * nb
    res.update({"gib": a.gib, "batch_blocks": a.batch, "slots": a.slots, "pinned": True})
    print(json.dumps(res))
    L.xs_engine_destroy(eng)
    for p in (hp, hb, ho, ok):
        L.xs_host_free(p)


if __name__ == "__main__":
    main()
