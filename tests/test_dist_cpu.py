"""N>1 path on CPU: world_size-2 gloo ranks plan their round-robin shards of one object,
"seal" them (the CPU oracle stands in for the device as the checker), and all-reduce the
counters.  Asserts: shards are disjoint and cover every block, per-rank output reassembles
into exactly the single-rank crypt body, and the counter all-reduce sums correctly."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch

    from oracle import pyoracle as orc
    from rclone_amd import shard
    from rclone_amd.testdata import splitmix64_bytes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    total = 11
    key = splitmix64_bytes(3, 32)
    nonce0 = bytes([0xFE] + [0xFF] * 7) + bytes(16)   # carries across nonce byte 8 inside the object
    plain = splitmix64_bytes(4, total * 65536)
    idx = shard.owned_blocks(total, world, rank)
    desc = shard.seal_descriptors(nonce0, idx)
    out = {}
    for j, b in enumerate(idx.tolist()):
        p = plain[b * 65536:(b + 1) * 65536]
        out[b] = orc.seal(p, bytes(desc["nonce"][j]), key)
    counters = torch.tensor([len(idx), len(idx) * 65536, 0], dtype=torch.int64)
    shard.reduce_counters(counters, dist)
    q.put((rank, out, counters.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_round_robin_two_ranks():
    from oracle import pyoracle as orc
    from rclone_amd.testdata import splitmix64_bytes
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    blocks = {}
    for rank, out, counters in res:
        assert counters == [11, 11 * 65536, 0]
        for b in out:
            assert b % world == rank and b not in blocks
        blocks.update(out)
    assert sorted(blocks) == list(range(11))
    key = splitmix64_bytes(3, 32)
    nonce0 = bytes([0xFE] + [0xFF] * 7) + bytes(16)
    whole = orc.encrypt_file(splitmix64_bytes(4, 11 * 65536), nonce0, key)[32:]
    assert b"".join(blocks[b] for b in range(11)) == whole


def test_owned_blocks_partition():
    from rclone_amd import shard
    for world in (1, 2, 4, 8):
        seen = np.concatenate([shard.owned_blocks(1001, world, r) for r in range(world)])
        assert sorted(seen.tolist()) == list(range(1001))
    with pytest.raises(ValueError):
        shard.owned_blocks(10, 2, 2)
