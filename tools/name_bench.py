#!/usr/bin/env python3
"""File-name cipher throughput (batched listings of many names).

For a batch of N synthetic names (lowercase ASCII, lengths uniform in [lo, hi]) under a
scrypt-derived key, times on the GPU box:
  * kernel: the EME-AES-256 launch alone (HIP events inside rc_names_run), names/s and
    algorithmic GB/s (bytes read + written of the padded names);
  * end to end: rc_names_run for whole segments (host pkcs7 + pack, H2D, kernel, D2H,
    encoding) -- EncryptFileName/DecryptFileName of single-segment names;
  * cpu: the oracle's EME (oracle/eme_oracle.c, one core, a bounded sample) -- a baseline
    only, the reference's Go AES would use AES-NI and be faster per core.
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rclone_amd import crypt, names  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--names", type=int, default=1_000_000)
    ap.add_argument("--lo", type=int, default=8)
    ap.add_argument("--hi", type=int, default=64)
    ap.add_argument("--enc", default="base32")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    rng = np.random.default_rng(42)
    lens = rng.integers(a.lo, a.hi + 1, a.names)
    pool = rng.integers(ord("a"), ord("z") + 1, int(lens.sum()), dtype=np.uint8).tobytes()
    segs, p = [], 0
    for ln in lens:
        segs.append(pool[p:p + ln])
        p += ln
    padded = int(((lens // 16) + 1).sum()) * 16
    c = crypt.new_cipher(names.NAME_ENCRYPTION_STANDARD, "potato", "", True, names.new_name_encoding(a.enc))
    res = {"names": a.names, "name_len": [a.lo, a.hi], "encoding": a.enc, "padded_bytes": padded}
    for label, op, inp in (("encrypt", names.OP_ENCRYPT_SEGMENT, segs), ("decrypt", names.OP_DECRYPT_SEGMENT, None)):
        if inp is None:
            inp = enc_out
        c.names_run(op, inp[:1000], as_bytes=True)  # warm-up
        ks, ws = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r = c.names_run(op, inp, as_bytes=True)
            ws.append(time.perf_counter() - t0)
            ks.append(r.kernel_ms)
        if label == "encrypt":
            enc_out = r.values
        else:
            assert r.values == segs, "round trip failed"
        kms = float(np.median(ks))
        w = float(np.median(ws))
        res[label] = {"kernel_ms": round(kms, 4), "kernel_names_per_s": round(a.names / (kms / 1e3)),
                      "kernel_GB_s": round(2 * padded / (kms / 1e3) / 1e9, 2),
                      "end_to_end_s": round(w, 4), "end_to_end_names_per_s": round(a.names / w)}
    from oracle import pyoracle as orc  # baseline only
    key, tweak = c.name_key, c.name_tweak
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 5.0:
        orc.eme_transform(key, tweak, orc.pkcs7_pad(segs[k % len(segs)]), True)
        k += 1
    dt = time.perf_counter() - t0
    res["cpu_baseline"] = {"names_per_s": round(k / dt), "cores": 1, "kind": "port",
                           "sample": f"{k} names through oracle/eme_oracle.c (ctypes per call) in {dt:.1f} s"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
