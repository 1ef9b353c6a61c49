#!/usr/bin/env python3
"""GPU MD5 of crypt files (one lane per object) vs the host: device-resident kernel rate for
N objects of one sealed 64 KiB block each (65 584-byte crypt files), and the end-to-end
batched cryptcheck call (host plaintext -> GPU seal -> GPU MD5 -> 16 B/object back) for
BASELINE configs[0]'s 1000 x 64 KiB.  CPU reference: hashlib.md5 on one core.  (The oracle is
test infrastructure and is not used here; the digests' parity is tests/test_md5_gpu.py.)"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rclone_amd import crypt, device  # noqa: E402
from rclone_amd.testdata import splitmix64_bytes  # noqa: E402

MD5_DESC = np.dtype([("off", "<u8"), ("len", "<u8"), ("prefix", "u1", (32,)), ("prefix_len", "<u4"),
                     ("res", "<u4", (3,))])


def kernel_rate(nobj, reps=5):
    flen = 65552  # wire body of one full block; +32 header in the prefix
    stride = (flen + 15) & ~15
    src = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
    device.fill_random(src, 1)
    d = np.zeros(nobj, dtype=MD5_DESC)
    d["off"] = np.arange(nobj, dtype=np.uint64) * stride
    d["len"] = flen
    d["prefix_len"] = 32
    dt = torch.from_numpy(np.frombuffer(d.tobytes(), dtype=np.uint8).copy()).cuda()
    device.md5_batch(dt, src)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        device.md5_batch(dt, src)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ms = sorted(ts)[len(ts) // 2]
    return {"objects": nobj, "ms": round(ms, 3), "GB_s": round(nobj * (flen + 32) / (ms * 1e-3) / 1e9, 2)}


def main():
    res = {"kernel": [kernel_rate(n) for n in (1000, 10000, 100000)]}
    # host single-core MD5 rate
    blob = splitmix64_bytes(2, 64 << 20)
    t0 = time.perf_counter()
    hashlib.md5(blob).digest()
    res["hashlib_md5_1core_GB_s"] = round(len(blob) / (time.perf_counter() - t0) / 1e9, 3)
    # end-to-end batched cryptcheck of configs[0]: 1000 x 64 KiB
    from tests.go_readers import Buffer
    c = crypt.Cipher("potato", "")
    plains = [splitmix64_bytes(1000 + i, 65536) for i in range(1000)]
    nonces = [splitmix64_bytes(5000 + i, 24) for i in range(1000)]
    c.hash_batch_with_nonce([(nonces[0], Buffer(plains[0]))])  # warm engine
    t0 = time.perf_counter()
    got = c.hash_batch_with_nonce([(nonces[i], Buffer(plains[i])) for i in range(1000)])
    el = time.perf_counter() - t0
    res["cryptcheck_1000x64KiB_gpu"] = {"s": round(el, 4), "GiB_s": round(1000 * 65536 / 2**30 / el, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
