"""Per-object hashing in the shape unchanged callers use (crypt.go:497-563 put, :784-806
computeHashWithNonce; cmd/cryptcheck/cryptcheck.go:91-114).

* rc_compute_hash_with_nonce from 8 concurrent threads (cryptcheck's --checkers 8) over a mixed
  tree of >= 1 GiB (log-uniform 4 KiB .. 8 MiB plus the edge sizes): every digest equals hashlib's
  MD5 of the CPU oracle's crypt file for the same plaintext and nonce.
* the encrypter's own tee hash (rc_encrypter_set_md5) for whole streams and for consumers that
  stop anywhere, including inside the header and inside a batch being hashed.
* reader and close errors come back as the reference returns them (io.Copy + fs.CheckClose).
"""
import hashlib
import math
import threading

import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes, splitmix64_words
from tests.go_readers import Buffer

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _tree(total_bytes, seed=0x7EE):
    """Object sizes: the edge sizes, then log-uniform in [4 KiB, 8 MiB] up to total_bytes."""
    sizes = [0, 1, 65535, 65536, 65537, 16 * 65536, 16 * 65536 + 1]
    lo, hi = math.log(4096), math.log(8 << 20)
    words = iter(int(w) for w in splitmix64_words(seed, 1 << 16))
    while sum(sizes) < total_bytes:
        u = (next(words) >> 11) / float(1 << 53)
        sizes.append(int(math.exp(lo + u * (hi - lo))))
    return sizes


class _Closing(Buffer):
    def __init__(self, data):
        super().__init__(data)
        self.closes = 0

    def close(self):
        self.closes += 1


def test_eight_checkers_per_object_hashes_1gib():
    from rclone_amd import crypt
    c = crypt.Cipher("potato", "")
    pool = crypt.EnginePool([0])
    c.pool = pool
    key = c.data_key
    sizes = _tree(1 << 30)
    total = sum(sizes)
    nonces = [splitmix64_bytes(0xA0000 + i, 24) for i in range(len(sizes))]
    nonces[3] = b"\xff" * 8 + nonces[3][8:]  # block adds carry out of nonce byte 7
    bad, done, lock = [], [0], threading.Lock()
    it = iter(range(len(sizes)))

    def checker():
        while True:
            with lock:
                i = next(it, None)
            if i is None:
                return
            plain = splitmix64_bytes(0xB0000 + i, sizes[i])
            src = _Closing(plain)
            got = c.compute_hash_with_nonce(nonces[i], src)
            want = hashlib.md5(orc.encrypt_file(plain, nonces[i], key)).hexdigest()
            with lock:
                done[0] += 1
                if got != want or src.closes != 1:
                    bad.append((i, sizes[i], got, want, src.closes))

    th = [threading.Thread(target=checker) for _ in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    stats = pool.stats()[0]
    print(f"{len(sizes)} objects, {total / 2**30:.2f} GiB; engine batches/requests/blocks {stats}")
    assert done[0] == len(sizes) and total >= 1 << 30
    assert not bad, bad[:5]
    assert stats[1] >= stats[0] > 0


def test_encrypter_tee_md5_any_stop_point():
    from rclone_amd import crypt
    c = crypt.Cipher("potato", "")
    key = c.data_key
    for size in (0, 1, 65536, 65537, 5 * 1048576 + 3, 12 * 1048576):
        plain = splitmix64_bytes(size + 5, size)
        nonce = splitmix64_bytes(size + 6, 24)
        ct = orc.encrypt_file(plain, nonce, key)
        for stop in sorted({0, 5, 32, 33, 32 + 65552, len(ct) // 3, len(ct) - 1, len(ct)}):
            if stop > len(ct):
                continue
            e = c.encrypt_data(Buffer(plain), nonce)
            e.set_md5(True)
            got = b""
            while len(got) < stop:
                data, err = e.read_go(min(1 << 20, stop - len(got)))
                got += data
                if err is not None:
                    break
            if stop == len(ct):
                data, err = e.read_go(1)
                assert data == b"" and err is crypt.EOF
            assert got == ct[:stop]
            assert e.md5() == hashlib.md5(ct[:stop]).digest(), (size, stop)


def test_hash_errors_and_close():
    from rclone_amd import crypt

    class Boom(Exception):
        pass

    class Failing(_Closing):
        def __init__(self, data, at):
            super().__init__(data)
            self.at = at

        def read_go(self, n):
            if self.pos >= self.at:
                return b"", Boom("read failed")
            return super().read_go(min(n, self.at - self.pos))

    class BadClose(_Closing):
        def close(self):
            super().close()
            raise Boom("close failed")

    c = crypt.Cipher("potato", "")
    plain = splitmix64_bytes(77, 3 * 1048576 + 9)
    nonce = splitmix64_bytes(78, 24)
    for at in (0, 1, 65536, 2 * 1048576 + 5):
        src = Failing(plain, at)
        with pytest.raises(Boom, match="read failed"):
            c.compute_hash_with_nonce(nonce, src)
        assert src.closes == 1
    src = BadClose(plain)
    with pytest.raises(Boom, match="close failed"):
        c.compute_hash_with_nonce(nonce, src)
    assert src.closes == 1
    want = hashlib.md5(orc.encrypt_file(plain, nonce, c.data_key)).hexdigest()
    assert c.compute_hash_with_nonce(nonce, _Closing(plain)) == want


def _child_hash_tree(total, checkers):
    """Run in a child process whose MD5 tiers are sized from its environment: per-object hashes
    from `checkers` threads over a mixed tree, each checked against the oracle.  Prints one JSON
    line (objects, mismatches, the CPU budget seen)."""
    import json

    from rclone_amd import _lib, crypt
    c = crypt.Cipher("potato", "")
    key = c.data_key
    sizes = _tree(total, seed=0x1A9E)
    bad, lock = [0], threading.Lock()
    it = iter(range(len(sizes)))

    def checker():
        while True:
            with lock:
                i = next(it, None)
            if i is None:
                return
            plain = splitmix64_bytes(0xC0000 + i, sizes[i])
            nonce = splitmix64_bytes(0xD0000 + i, 24)
            got = c.compute_hash_with_nonce(nonce, _Closing(plain))
            if got != hashlib.md5(orc.encrypt_file(plain, nonce, key)).hexdigest():
                with lock:
                    bad[0] += 1

    th = [threading.Thread(target=checker) for _ in range(checkers)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    print(json.dumps({"objects": len(sizes), "mismatches": bad[0], "cpus": _lib.lib().xs_effective_cpus()}))


def test_per_object_hashes_through_engine_lanes():
    # a CPU budget of 2 and one worker: most streams' MD5 runs in the 16-lane AVX-512 engine
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RCLONE_AMD_CPUS="2", XS_MD5_WORKERS="1", XS_MD5_SCALAR_BUDGET="1",
               RCLONE_AMD_PHASES="1", PYTHONPATH=root)
    code = "import tests.test_hash_stream_gpu as t; t._child_hash_tree(256 << 20, 16)"
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    phases = [json.loads(x)["rclone_amd_phases"] for x in r.stderr.splitlines() if x.startswith('{"rclone_amd_phases"')]
    print(res, phases)
    assert res["mismatches"] == 0 and res["objects"] > 200 and res["cpus"] == 2
    assert phases and phases[-1]["md5_jobs_lanes"] > 0 or not _avx512()


def _avx512():
    try:
        return "avx512f" in open("/proc/cpuinfo").read()
    except OSError:
        return False
