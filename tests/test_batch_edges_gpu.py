"""Edge cases of the descriptor-batch ABI and of concurrent handle use.

* xs_seal_batch_dev / xs_open_batch_dev must skip -- write nothing for, and report ok = 0 --
  every descriptor that is out of bounds, misaligned or has len outside 1..65536, while every
  valid descriptor in the same batch is sealed/opened bit-exactly (oracle).
* rc_* handles are used concurrently from many OS threads (crypt's --transfers/--checkers;
  each handle serialises itself like fh.mu, cipher.go:720/:902) and share one GPU engine.
"""
import threading

import numpy as np
import pytest

from oracle import pyoracle as orc
from rclone_amd.testdata import splitmix64_bytes
from tests.go_readers import Buffer, read_all

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DESC = np.dtype([("src", "<u8"), ("dst", "<u8"), ("len", "<u4"), ("res", "<u4"), ("nonce", "u1", (24,))])


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_invalid_descriptors_are_skipped():
    from rclone_amd import device
    key = splitmix64_bytes(1, 32)
    plain = splitmix64_bytes(2, 8 * 65536)
    src = torch.from_numpy(np.frombuffer(plain, dtype=np.uint8).copy()).cuda()
    slen, dlen = 8 * 65536, 8 * 65552
    rows = [  # (src_off, dst_off, len, valid)
        (0, 0, 65536, True),
        (65536, 65552, 100, True),
        (8, 2 * 65552, 64, False),               # misaligned plaintext
        (2 * 65536, 3 * 65552 + 8, 64, False),   # misaligned ciphertext (dst + 16)
        (3 * 65536, 4 * 65552, 0, False),        # len 0
        (3 * 65536, 4 * 65552, 65537, False),    # len > blockDataSize
        (slen - 64, 5 * 65552, 128, False),      # source out of bounds
        (4 * 65536, dlen - 64, 100, False),      # destination out of bounds
        (5 * 65536, 6 * 65552, 65536, True),
        (7 * 65536, 7 * 65552, 1, True),
    ]
    d = np.zeros(len(rows), dtype=DESC)
    for i, (so, do, n, _) in enumerate(rows):
        d[i]["src"], d[i]["dst"], d[i]["len"] = so, do, n
        d[i]["nonce"] = np.frombuffer(splitmix64_bytes(100 + i, 24), dtype=np.uint8)
    dst = torch.full((dlen,), 0xAA, dtype=torch.uint8, device="cuda")
    device.seal_batch(key, d, src, dst)
    torch.cuda.synchronize()
    body = dst.cpu().numpy().tobytes()
    written = np.zeros(dlen, dtype=bool)
    for i, (so, do, n, ok) in enumerate(rows):
        if ok:
            box = orc.seal(plain[so:so + n], d[i]["nonce"].tobytes(), key)
            assert body[do:do + 16 + n] == box, i
            written[do:do + 16 + n] = True
    untouched = np.frombuffer(body, dtype=np.uint8)[~written]
    assert (untouched == 0xAA).all()
    # open the same batch (src/dst swapped): invalid -> ok 0 and nothing written
    od = d.copy()
    od["src"], od["dst"] = d["dst"], d["src"]
    out = torch.full((slen,), 0x55, dtype=torch.uint8, device="cuda")
    ok = device.open_batch(key, od, dst, out)
    torch.cuda.synchronize()
    assert ok.cpu().numpy().tolist() == [int(r[3]) for r in rows]
    got = out.cpu().numpy().tobytes()
    seen = np.zeros(slen, dtype=bool)
    for so, do, n, v in rows:
        if v:
            assert got[so:so + n] == plain[so:so + n]
            seen[so:so + n] = True
    assert (np.frombuffer(got, dtype=np.uint8)[~seen] == 0x55).all()


def test_concurrent_handles_from_threads():
    from rclone_amd import crypt
    errors = []

    class Nonces:
        def __init__(self, b):
            self.b = Buffer(b)

        def read_go(self, n):
            return self.b.read_go(n)

    def worker(t):
        try:
            c = crypt.Cipher("potato" if t % 2 else "", "", batch_blocks=[1, 3, 16, 64][t % 4])
            for j in range(4):
                n = [0, 1, 65536, 3 * 65536 + 17, 200000][(t + j) % 5]
                plain = splitmix64_bytes(1000 * t + j, n)
                n0 = splitmix64_bytes(5000 * t + j, 24)
                c.crypto_rand = Nonces(n0)
                ct, err = read_all(c.encrypt_data(Buffer(plain)), bufsize=[7, 4096, 1 << 20][j % 3])
                assert err is None
                assert ct == orc.encrypt_file(plain, n0, c.data_key), (t, j)
                back, err = read_all(c.decrypt_data(Buffer(ct)))
                assert err is None and back == plain
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    assert not errors, errors
