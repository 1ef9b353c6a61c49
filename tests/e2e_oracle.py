"""TEST INFRASTRUCTURE: the CPU oracle's crypt-file MD5 of every object of an e2e_sync tree
(tools/e2e_sync.cpp --tee-all FILE), to check the tee MD5 the harness recorded for each stored
object.  crypt.put already compared that tee MD5 with the MD5 of the bytes the remote stored
(crypt.go:542-560, put_hash_mismatches == 0), so equality here pins every stored byte of the tree
to the oracle (oracle/xsalsa_simd.c orc_simd_encrypt_gen_file: the SplitMix64(seed) plaintext,
sealed block by block with nonce + j, cipher.go:694-758)."""
import hashlib
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from oracle import pyoracle as orc


def read_tee_all(path):
    rows = []
    with open(path) as f:
        for line in f:
            i, size, seed, nonce, md5 = line.split()
            rows.append((int(i), int(size), int(seed), bytes.fromhex(nonce), md5))
    return rows


def verify_tee_all(path, key, threads=None):
    """-> (objects, plaintext bytes, [indices whose tee MD5 differs from the oracle's])."""
    rows = read_tee_all(path)
    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
    local = threading.local()
    cap = max([orc.encrypted_size(r[1]) for r in rows] + [1])

    def one(r):
        buf = getattr(local, "buf", None)
        if buf is None:
            buf = local.buf = np.empty(cap, dtype=np.uint8)
        n = orc.encrypt_gen_file_into(buf, r[2], r[1], r[3], key)  # ctypes: the GIL is released
        return r[0] if hashlib.md5(memoryview(buf)[:n]).hexdigest() != r[4] else None

    with ThreadPoolExecutor(threads) as ex:
        bad = [i for i in ex.map(one, rows, chunksize=64) if i is not None]
    return len(rows), sum(r[1] for r in rows), bad
