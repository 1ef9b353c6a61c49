"""The N>1 paths on the GPU box (VERDICT r03 "next" 1 and 2).

* `bench.py --gpus 2` starts its own two ranks (no launcher).  On a one-GPU box they are gloo
  ranks sharing device 0 (BENCH_DIST_BACKEND=gloo); the real N-GPU run is the same code over
  RCCL with one rank per GPU.  Each mode's result must equal the one-rank run over the same
  blocks: the tag digest is order-independent, so rank r's round-robin share b = r (mod 2) of a
  2n-block object sums to the one-rank digest of all 2n blocks (BASELINE configs[3] layout).
* One process spreads its streams over two *distinct* devices (xs_pool over [0, 1], the
  counterpart of rclone's --transfers / --checkers goroutine pool, fs/sync/sync.go:544-548):
  runs when the box shows more than one device, else skips with that reason.
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _bench(*args, gloo=True, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "BENCH_FORCE_PG")}
    # the default mode's configs[3] leg over a 400 000-block object instead of 1 TiB (one step):
    # the same code, the same cross-rank sums, seconds instead of tens of seconds
    env["BENCH_OBJECTSET_BLOCKS"] = "400000"
    if gloo:
        env["BENCH_DIST_BACKEND"] = "gloo"
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--warmup-seconds", "0", "--no-cpu", *args],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return lines[0]


def test_bench_two_ranks_default_mode_matches_one_rank():
    nb = 8192
    two = _bench("--gpus", "2", "--steps", "2", "--warmup", "1", "--blocks", str(nb), "--objectset-steps", "1")
    one = _bench("--gpus", "1", "--steps", "2", "--warmup", "1", "--blocks", str(2 * nb), "--objectset-steps", "1")
    assert two["n_gpus"] == 2 and two["config"]["ranks_seen"] == 2 and len(two["config"]["rank_gpus"]) == 2
    assert two["config"]["distinct_gpus"] == min(2, torch.cuda.device_count())
    # counters summed over the ranks: 2 ranks x 2 steps x (seal + open) x nb blocks
    assert two["counters"]["blocks"] == 2 * 2 * 2 * nb == one["counters"]["blocks"]
    assert two["counters"]["bytes"] == one["counters"]["bytes"]
    assert two["counters"]["tag_failures"] == 0 == one["counters"]["tag_failures"]
    assert two["counters"]["tag_digest"] == one["counters"]["tag_digest"]
    assert two["build_id"] == one["build_id"]
    assert two["value"] > 0 and two["scaling"] == "weak"
    # the configs[3] leg: a fixed object split over the ranks, the same digest for 1 and 2 ranks
    for k in ("blocks", "bytes", "tag_failures", "roundtrip_mismatch_words", "tag_digest"):
        assert two["objectset"]["counters"][k] == one["objectset"]["counters"][k], k
    assert two["objectset"]["ok"] and one["objectset"]["ok"] and two["objectset"]["scaling"] == "strong"
    assert two["objectset"]["counters"]["blocks"] == 400000


def test_bench_two_ranks_object_set_matches_one_rank():
    args = ["--steps", "1", "--warmup", "1", "--object-blocks", "40000", "--blocks", "8192"]
    two = _bench("--gpus", "2", *args)
    one = _bench("--gpus", "1", *args)
    assert two["n_gpus"] == 2 and two["config"]["ranks_seen"] == 2
    assert two["counters"]["blocks"] == 40000 == one["counters"]["blocks"]
    assert two["counters"]["tag_failures"] == 0 and two["counters"]["roundtrip_mismatch_words"] == 0
    assert two["counters"]["tag_digest"] == one["counters"]["tag_digest"]


def test_bench_two_ranks_names_and_mixed():
    names = _bench("--gpus", "2", "--steps", "1", "--warmup", "1", "--names", "20000")
    assert names["n_gpus"] == 2 and names["config"]["ranks_seen"] == 2 and names["value"] > 0
    mixed = _bench("--gpus", "2", "--steps", "1", "--warmup", "1", "--mixed-gib", "0.1")
    assert mixed["n_gpus"] == 2 and mixed["counters"]["verified"] is True


def test_bench_rccl_one_rank_group_matches_no_group():
    """Every RCCL call the N-GPU line makes (init with device_id, the topology gather, barriers,
    the counter SUM and the time MAX all-reduces, destroy), run for real on this box's GPU through
    a one-rank RCCL group (BENCH_FORCE_PG=1; two RCCL ranks cannot share one device), in each
    mode: the results equal the run without a group."""
    base = ["--gpus", "1", "--steps", "2", "--warmup", "1", "--objectset-steps", "1"]
    for extra in (["--blocks", "8192"], ["--object-blocks", "40000", "--blocks", "8192"], ["--names", "20000"],
                  ["--mixed-gib", "0.1"]):
        pg = _bench(*base, *extra, gloo=False, env_extra={"BENCH_FORCE_PG": "1", "BENCH_DIST_BACKEND": "nccl"})
        assert pg["config"]["process_group"] == "nccl" and pg["config"]["ranks_seen"] == 1, (extra, pg["config"])
        assert pg["n_gpus"] == 1 and pg["value"] > 0
        if "--names" in extra:
            continue
        one = _bench(*base, *extra, gloo=False)
        assert one["config"]["process_group"] is None
        if "--mixed-gib" in extra:
            assert pg["counters"]["verified"] is True
            continue
        for k in ("blocks", "bytes", "tag_failures", "tag_digest"):
            assert pg["counters"][k] == one["counters"][k], (extra, k)
        if pg.get("objectset"):  # the default mode's configs[3] leg through the RCCL group
            assert pg["objectset"]["counters"]["tag_digest"] == one["objectset"]["counters"]["tag_digest"]


def test_bench_rccl_refuses_more_ranks_than_gpus():
    n = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "BENCH_DIST_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "1",
                        "--no-cpu"], capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode != 0 and not any(ln.startswith("{") for ln in r.stdout.splitlines())
    assert f"need {n + 1} GPUs, {n} visible" in r.stderr


def test_pool_over_distinct_devices():
    """One process, engines on two distinct GPUs: a batched put splits its objects over both,
    bytes and MD5s equal the oracle's, and streams of one cipher land on both devices."""
    n_dev = torch.cuda.device_count()
    if n_dev < 2:
        pytest.skip(f"needs two HIP devices, this box shows {n_dev}: the pool over distinct devices "
                    "runs on the driver's multi-GPU node only")
    from oracle import pyoracle as orc
    from rclone_amd import _lib, crypt
    from rclone_amd.testdata import splitmix64_bytes
    from tests.go_readers import Buffer
    L = _lib.lib()
    pool = crypt.EnginePool([0, 1], batch_blocks=64)
    try:
        assert [L.xs_engine_device(pool.engine(i)) for i in range(len(pool))] == [0, 1]
        key = splitmix64_bytes(61, 32)
        sizes = [0, 1, 65536, 65537, 3 * 65536 + 7, 1 << 20] + [4096 * k + 5 for k in range(1, 40)]
        plains = [splitmix64_bytes(700 + i, n) for i, n in enumerate(sizes)]
        nonces = b"".join(splitmix64_bytes(900 + i, 24) for i in range(len(sizes)))
        offs, pos = [], 0
        for n in sizes:
            offs.append(pos)
            pos += (n + 15) & ~15
        stage = bytearray(pos + 16)
        for o, p in zip(offs, plains):
            stage[o:o + len(p)] = p
        cnt = len(sizes)
        u64s = ctypes.c_uint64 * cnt
        lens_c, offs_c = u64s(*sizes), u64s(*offs)
        total = L.xs_put_body_bytes(cnt, lens_c)
        src = (ctypes.c_uint8 * len(stage)).from_buffer(stage)
        body, md5 = (ctypes.c_uint8 * (total + 16))(), (ctypes.c_uint8 * (16 * cnt))()
        assert L.xs_pool_put_batch(pool.handle, key, cnt, nonces, offs_c, lens_c, src, body, md5) == 0, \
            _lib.last_error()
        raw, dig, bpos = bytes(body), bytes(md5), 0
        for i, p in enumerate(plains):
            want = orc.encrypt_file(p, nonces[24 * i:24 * i + 24], key)
            assert raw[bpos:bpos + len(want) - 32] == want[32:], (i, sizes[i])
            assert dig[16 * i:16 * i + 16] == hashlib.md5(want).digest(), (i, sizes[i])
            bpos += (len(want) - 32 + 15) & ~15
        for i in range(2):  # both devices took a range of the objects
            st = (ctypes.c_uint64 * 3)()
            L.xs_engine_md5_stats(pool.engine(i), st)
            assert st[2] > 0, (i, list(st))
        c = crypt.Cipher("potato", "")
        c.pool = pool
        before = [s[1] for s in pool.stats()]
        for k in range(6):
            p = splitmix64_bytes(5000 + k, 70001 * k + 3)
            nonce = splitmix64_bytes(5100 + k, 24)
            ct = c.encrypt_data(Buffer(p), nonce).readall()
            assert ct == orc.encrypt_file(p, nonce, c.data_key)
            assert c.decrypt_data(Buffer(ct)).readall() == p
        after = [s[1] for s in pool.stats()]
        assert all(a > b for a, b in zip(after, before)), (before, after)
        c.pool = None
    finally:
        pool.close()


def test_bench_pool_check_runs_its_checks():
    """bench.py's after-timing pool check (one process, engines over every visible GPU) on this
    box's device repeated: the function the multi-GPU bench line runs, checked here for real."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    res = bench.pool_check([0, 0])
    assert res["ran"] and res["ok"], res
    assert res["engine_devices"] == [0, 0] and res["objects_differing_from_oracle"] == 0
    assert all(t > 0 for t in res["engine_objects"])
    if torch.cuda.device_count() < 2:
        assert bench.pool_check() == {"devices": torch.cuda.device_count(), "ran": False}
