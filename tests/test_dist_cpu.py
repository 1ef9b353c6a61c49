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


def _bench(args, env_extra=None, timeout=180):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=timeout, cwd=root)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


def test_bench_starts_its_own_ranks():
    """`bench.py --gpus 2` with no launcher starts two ranks itself; they join one process group
    and only rank 0 prints the line, with the world size the group reports."""
    r, lines = _bench(["--gpus", "2", "--dry-run", "--steps", "3"], {"BENCH_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    res = lines[0]
    assert res["n_gpus"] == 2 and res["dry_run"] is True
    assert res["config"] == {"ranks_seen": 2, "ranks_reported": 2, "rank_sum": 1, "process_group": "gloo"}


def test_bench_starts_eight_ranks():
    """The driver's N = 8 launch, rehearsed on the CPU: `bench.py --gpus 8 --dry-run` starts eight
    ranks, they join one gloo group, the counter all-reduce sees all of them, and exactly one line
    is printed (rank 0's)."""
    r, lines = _bench(["--gpus", "8", "--dry-run", "--steps", "3"], {"BENCH_DIST_BACKEND": "gloo"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout
    res = lines[0]
    assert res["n_gpus"] == 8 and res["dry_run"] is True
    assert res["config"] == {"ranks_seen": 8, "ranks_reported": 8, "rank_sum": sum(range(8)), "process_group": "gloo"}


def test_pool_check_timeout_grows_with_devices():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    t = [bench.pool_check_timeout(n) for n in (1, 2, 8)]
    assert t[0] >= 90 and t[0] < t[1] < t[2] and t[2] >= 200


def test_bench_forced_one_rank_group():
    """BENCH_FORCE_PG=1 puts an N = 1 run through a one-rank process group (its own rendezvous on
    127.0.0.1 when no launcher set one): the collectives an N-GPU run makes, on one rank."""
    r, lines = _bench(["--dry-run", "--steps", "1"], {"BENCH_FORCE_PG": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 1
    assert lines[0]["config"] == {"ranks_seen": 1, "ranks_reported": 1, "rank_sum": 0, "process_group": "gloo"}
    r, lines = _bench(["--dry-run", "--steps", "1"])
    assert r.returncode == 0 and lines[0]["config"]["process_group"] is None


def test_bench_refuses_gpus_world_mismatch():
    r, lines = _bench(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1"})
    assert r.returncode != 0 and not lines
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_bench_rank_failure_fails_the_job():
    """A rank that cannot run (no GPU here: RCCL ranks need one device each) ends the job with a
    non-zero status and no result line."""
    r, lines = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and not lines
    assert "need 2 GPUs" in r.stderr or "exited with status" in r.stderr


def test_bench_wrong_shard_fails_the_job():
    """A rank whose shard digest is wrong (forced) makes the summed digest miss on every rank: the
    line still prints with objectset.ok false, and the job ends non-zero."""
    r, lines = _bench(["--gpus", "2", "--dry-run", "--steps", "1"],
                      {"BENCH_DIST_BACKEND": "gloo", "BENCH_FORCE_DIGEST_MISMATCH": "1"})
    assert r.returncode != 0, r.stderr[-3000:]
    assert len(lines) == 1 and lines[0]["objectset"]["ok"] is False
    assert "objectset leg failed" in r.stderr
    r, lines = _bench(["--gpus", "2", "--dry-run", "--steps", "1"], {"BENCH_DIST_BACKEND": "gloo"})
    assert r.returncode == 0 and lines[0]["objectset"]["ok"] is True


def test_fail_if_wrong_paths():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    bench.fail_if_wrong(True, "a", "a", 0, None)
    bench.fail_if_wrong(True, "a", "a", 0, True)
    for args, msg in (((False, "a", "b", 0, True), "headline tag digest a != oracle b"),
                      ((True, "a", "a", 3, True), "3 tag failures"),
                      ((True, "a", "a", 0, False), "objectset leg failed")):
        with pytest.raises(SystemExit, match=msg):
            bench.fail_if_wrong(*args)
    # the headline pins: worlds 1/2/4/8 at 100000 blocks per rank, nothing for other layouts
    assert len(bench.headline_expected_digest(1, 100_000, False)) == 32
    assert bench.headline_expected_digest(8, 100_000, False) != bench.headline_expected_digest(1, 100_000, False)
    assert bench.headline_expected_digest(3, 100_000, False) is None
    assert bench.headline_expected_digest(1, 50_000, False) is None
    # the same blocks split another way: 4 ranks x 50 000 = blocks 0..199 999 = 2 ranks x 100 000
    assert bench.headline_expected_digest(4, 50_000, False) == bench.headline_expected_digest(2, 100_000, False)
    assert bench.headline_expected_digest(1, 100_000, True) is None


def test_power_sampler_reads_hwmon(tmp_path, monkeypatch):
    """bench.py's in-process board power / clock sampler over a fake amdgpu hwmon directory: the
    mean of power1_input samples x the window, or the energy1_input difference when the counter
    exists; None (with the reason) when the GPU has no hwmon power file."""
    import importlib.util
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_pw", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    hw = tmp_path / "bus" / "pci" / "devices" / "0000:8b:00.0" / "hwmon" / "hwmon3"
    hw.mkdir(parents=True)
    (hw / "power1_input").write_text("1400000000\n")  # microwatts
    (hw / "freq1_input").write_text("1850000000\n")   # Hz
    monkeypatch.setenv("RCLONE_AMD_SYSFS_ROOT", str(tmp_path))
    p = bench.PowerSampler((0, 0x8B, 0), period=0.002)
    p.start()
    time.sleep(0.1)
    p.stop()
    w, j, ghz, info = p.result()
    assert w == 1400.0 and abs(ghz - 1.85) < 1e-9 and info["samples"] > 5
    assert abs(j - 1400.0 * info["window_s"]) < 1400.0 * 1e-4  # window_s is rounded to 0.1 ms
    assert bench.energy_per_gib([[0, 0, 0, w, j, ghz]], 2**30) == round(j, 4)
    assert bench.energy_per_gib([[0, 0, 0, w, j, ghz], [0, 0, 0, None, None, None]], 2**30) is None
    # an energy counter wins over sampled power
    (hw / "energy1_input").write_text("5000000\n")  # microjoules
    p = bench.PowerSampler((0, 0x8B, 0), period=0.002)
    p.start()
    (hw / "energy1_input").write_text("5700000\n")
    time.sleep(0.02)
    p.stop()
    assert abs(p.result()[1] - 0.7) < 1e-9
    # no such GPU in sysfs: nothing is read, the line says why
    q = bench.PowerSampler((0, 0x99, 0))
    q.start()
    q.stop()
    w, j, ghz, info = q.result()
    assert w is None and j is None and "absent" in info["source"]
