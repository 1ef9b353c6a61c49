#!/usr/bin/env python3
"""Benchmark: device-resident crypt block encrypt+decrypt on MI355X (BASELINE.json metric).

One step = seal (encrypt) every 64 KiB block of a resident 100k-block object set, then
open (decrypt + verify) all of them: keygen + block kernel per direction, inputs already in
HBM (BASELINE.json configs[1] "1xMI355X encrypt: 100k x 64KiB device-resident blocks", with
the decrypt pass of configs[2] on the same blocks).  value = plaintext GiB pushed through the
cipher per second, both directions counted (2 x 6.25 GiB per step per GPU), summed over
ranks (weak scaling: every rank owns its own 100k blocks = its round-robin share of a larger
object set; no payload crosses ranks).  Counters (blocks, bytes, tag failures) are summed
across ranks with one RCCL all-reduce after the timed region.

Also reported: the dominant kernel's roofline (HBM; achieved algorithmic GB/s from HIP events
around every xs_crypt launch inside the timed region), the CPU baseline (the oracle's
C restatement, OpenMP, on this host's cores, bounded sample), and -- after the headline timing,
outside it -- BASELINE configs[3] as the `objectset` key: a 1 TiB object round-robin over the N
ranks (fixed total work: strong scaling), generated, sealed, opened and verified, with a tag
digest that must equal the one-GPU digest (rclone_amd.objectset.CONFIG3_TAG_DIGEST) -- see
DESIGN.md.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--blocks B] [--no-cpu] [--objectset-steps S]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident GiB/s, 64KiB-block crypt encrypt+decrypt, 1/2/4/8 MI355X"
BLOCK_DATA = 65536
BLOCK_SIZE = 65552
# algorithmic HBM bytes per 64 KiB block per launch:
#   seal: read 65536 plaintext + write 65552 wire block
#   open: read 65552 wire block + write 65536 plaintext + 1 ok byte
# (the 960-byte per-block key schedule is this design's own intermediate, not counted)
ALG_BYTES_SEAL = 65536 + 65552
ALG_BYTES_OPEN = 65552 + 65536 + 1
READ_BYTES_SEAL, READ_BYTES_OPEN = 65536, 65552  # the read half alone (SURVEY 8(d) "HBM-read roofline")
VALU_CYC, SIMDS, CLOCK_HZ = 4, 256 * 4, 2.4e9
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# the headline resident set: global block g = SplitMix64(HEADLINE_SEED) block g, sealed with
# HEADLINE_NONCE0 + g (the nonce carries across byte 8 inside the set); its tag digest for 1/2/4/8
# ranks is pinned by the CPU oracle in tests/golden/fullsize.json (tests/golden/make_fullsize.py)
HEADLINE_KEY = bytes(range(32))
HEADLINE_NONCE0 = bytes([0xF0]) + bytes([0xFF] * 7) + bytes(16)
HEADLINE_SEED = 0x5EED


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60, help="timed steps (about 0.4 s at N=1)")
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps (at least --warmup-seconds of them)")
    ap.add_argument("--warmup-seconds", type=float, default=2.0,
                    help="minimum back-to-back warm-up time: the DVFS clock settles after >= 2 s of load "
                         "(MI355X_MICROARCH.md)")
    ap.add_argument("--blocks", type=int, default=100_000, help="64 KiB blocks per GPU")
    ap.add_argument("--independent", action="store_true",
                    help="configs[1] as independent one-block objects, each with its own random nonce "
                         "(default: the rank's share of one object, nonce0 + block index)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--object-blocks", type=int, default=0,
                    help="configs[3] mode: one logical object of this many blocks (2^24 = 1 TiB) split "
                         "round-robin over the ranks, processed in --blocks rounds with on-device "
                         "generation inside each step (0 = the default resident-set bench)")
    ap.add_argument("--objectset-steps", type=int, default=3,
                    help="after the headline timing: the configs[3] leg (the 2^24-block 1 TiB object round-robin "
                         "over the ranks, generate + seal + open + verify), this many timed steps after "
                         "--objectset-warmup untimed ones; reported as the line's `objectset` key (0 = skip)")
    ap.add_argument("--objectset-warmup", type=int, default=1)
    ap.add_argument("--mixed-gib", type=float, default=0.0,
                    help="configs[2] mode: this many GiB of 4 KiB-8 MiB objects per rank (descriptor batches, "
                         "partial last blocks, ~0.1%% of the blocks tampered); one step = seal the set + "
                         "open+verify its tampered wire image (0 = the default resident-set bench)")
    ap.add_argument("--names", type=int, default=0,
                    help="file-name mode (SURVEY 8(f) rank 4): encrypt + decrypt this many names per step "
                         "through rc_names_run (0 = the default crypt-block bench)")
    ap.add_argument("--name-paths", action="store_true", help="names mode: 3-segment paths instead of one segment")
    ap.add_argument("--no-pool-check", action="store_true",
                    help="skip the after-timing check of one process's engine pool over every visible GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch check only: start the ranks, join the process group (gloo, CPU), all-reduce a "
                         "per-rank counter and print the line with value null; no device work")
    return ap.parse_args()


def launch_ranks(args):
    """`--gpus N` (N > 1) started without a launcher: start N ranks of this same command, one
    process per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), and exit
    with the first non-zero rank status (the other ranks are then stopped by PID).  Runs before
    anything touches the GPU: the children are fresh interpreters, never an exec of this one.
    Only rank 0 prints the JSON line.

    The rendezvous store is hosted here, by the launcher, for the job's whole life (as torchrun's
    agent does): its port is bound once and never released before the ranks connect, so no other
    process can take it in between; the ranks are told to be clients of it
    (TORCHELASTIC_USE_AGENT_STORE).  The launcher never touches a GPU."""
    import signal
    import subprocess

    from torch.distributed import TCPStore
    n = args.gpus
    store = TCPStore("127.0.0.1", 0, n, is_master=True, wait_for_workers=False)
    port = store.port
    procs = []

    def die_with_parent():  # a rank never outlives the launcher (a killed launcher must not leave
        try:                # ranks waiting in a collective on the GPUs)
            ctypes.CDLL(None).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except Exception:  # noqa: BLE001
            pass
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   TORCHELASTIC_USE_AGENT_STORE="True")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      preexec_fn=die_with_parent))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            c = p.poll()
            if c is None:
                continue
            pending.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench: rank {procs.index(p)} exited with status {c}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop()
        time.sleep(0.02)
    del store
    return rc


def grouped(world):
    """Whether this run holds a process group: every N > 1 run, and an N = 1 run under
    BENCH_FORCE_PG=1, which puts the one rank through the same RCCL calls an N-GPU run makes
    (init with device_id, the topology gather, barriers, counter SUM and time MAX all-reduces):
    the RCCL path's rehearsal on a one-GPU box, where two RCCL ranks cannot share the device."""
    return world > 1 or os.environ.get("BENCH_FORCE_PG") == "1"


def pg_init_kwargs(world):
    """init_process_group arguments.  Under a launcher: env:// (nothing to add).  A one-rank group
    under BENCH_FORCE_PG with no launcher: an in-process store on a port bound once and kept
    (no bind-close-rebind window for another process to take the port)."""
    if world == 1 and "MASTER_PORT" not in os.environ:
        from torch.distributed import TCPStore
        return {"store": TCPStore("127.0.0.1", 0, 1, is_master=True, wait_for_workers=False),
                "rank": 0, "world_size": 1}
    return {}


def rank_topology(dist, world, dev):
    """What the job actually ran on: the process group's own world size and each rank's GPU
    (PCI domain:bus:device, gathered with one small all-reduce).  `distinct_gpus` < ranks means
    ranks shared a GPU (the gloo rehearsal on a one-GPU box)."""
    import torch
    p = torch.cuda.get_device_properties(dev)
    me = (p.pci_domain_id << 16) | (p.pci_bus_id << 8) | p.pci_device_id
    if not grouped(world):
        ids = [me]
        seen = 1
    else:
        seen = dist.get_world_size()
        t = torch.zeros(world, dtype=torch.int64, device=dev)
        t[dist.get_rank()] = me
        dist.all_reduce(t)
        ids = [int(x) for x in t.cpu().tolist()]
    bus = ["%04x:%02x:%02x" % (i >> 16, (i >> 8) & 0xFF, i & 0xFF) for i in ids]
    return {"ranks_seen": seen, "rank_gpus": bus, "distinct_gpus": len(set(ids)),
            "process_group": dist.get_backend() if grouped(world) else None}


def run_dry(args, world, rank, dist):
    """--dry-run: the launch and the collective without any device work (CPU test of N > 1)."""
    import torch
    seen = dist.get_world_size() if grouped(world) else 1
    # a stand-in for a shard's digest contribution (rank + 1); BENCH_FORCE_DIGEST_MISMATCH=1 makes
    # rank BENCH_FORCE_FAIL_RANK (default the last) contribute a wrong one, as a bad shard would:
    # the summed digest then misses on every rank and the run must end non-zero, as the real leg's
    forced = os.environ.get("BENCH_FORCE_DIGEST_MISMATCH") == "1" and \
        rank == int(os.environ.get("BENCH_FORCE_FAIL_RANK", world - 1))
    t = torch.tensor([1, rank, rank + 1 + int(forced)], dtype=torch.int64)
    if grouped(world):
        dist.all_reduce(t)
    objset_ok = int(t[2]) == world * (world + 1) // 2
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True,
                          "config": {"ranks_seen": seen, "ranks_reported": int(t[0]), "rank_sum": int(t[1]),
                                     "process_group": dist.get_backend() if grouped(world) else None},
                          "objectset": {"ok": objset_ok, "digest_stand_in": int(t[2])}}),
              flush=True)
    if grouped(world):
        dist.destroy_process_group()
    fail_if_wrong(True, None, None, 0, objset_ok)


def fail_if_wrong(digest_ok, digest, expect, tag_failures, objset_ok):
    """End the run non-zero (after the line is printed) when a result is wrong: the headline set's
    tag digest differs from the CPU oracle's, a headline tag failed, or the configs[3] leg failed.
    Every rank calls it with the same, already all-reduced, inputs, so every rank exits non-zero."""
    bad = [] if digest_ok else [f"headline tag digest {digest} != oracle {expect}"]
    if tag_failures:
        bad.append(f"{tag_failures} tag failures in the headline set")
    if objset_ok is False:
        bad.append("objectset leg failed (tag digest vs the oracle's, counters or tag failures)")
    if bad:
        raise SystemExit("bench: " + "; ".join(bad))


def cpu_baseline(seconds):
    """CPU restatement seal+open of a bounded sample, OpenMP over blocks: the vectorised one
    (oracle/xsalsa_simd.c: AVX-512 16-way / AVX2 8-way Salsa20, radix-2^44 Poly1305) when the host
    has AVX2, else the scalar oracle/xsalsa_oracle.c."""
    import numpy as np
    from oracle import pyoracle as orc  # checker/baseline only
    from rclone_amd.testdata import splitmix64_bytes

    lib = orc.lib()
    level = lib.orc_simd_level()
    seal, open_ = ((lib.orc_simd_seal_blocks, lib.orc_simd_open_blocks) if level > 0
                   else (lib.orc_seal_blocks, lib.orc_open_blocks))
    impl = {2: "oracle/xsalsa_simd.c AVX-512 (16-way Salsa20, radix-2^44 Poly1305)",
            1: "oracle/xsalsa_simd.c AVX2 (8-way Salsa20, radix-2^44 Poly1305)"}.get(level, "oracle/xsalsa_oracle.c scalar")
    nb = 1024  # 64 MiB sample, repeated until `seconds` elapse
    plain = np.frombuffer(splitmix64_bytes(0x5EED, nb * BLOCK_DATA), dtype=np.uint8).copy()
    body = np.empty(nb * BLOCK_SIZE, dtype=np.uint8)
    out = np.empty(nb * BLOCK_DATA, dtype=np.uint8)
    ok = np.empty(nb, dtype=np.uint8)
    key = splitmix64_bytes(1, 32)
    n0 = splitmix64_bytes(2, 24)
    vp = ctypes.c_void_p
    threads = seal(vp(body.ctypes.data), vp(plain.ctypes.data), nb, n0, key)  # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        threads = seal(vp(body.ctypes.data), vp(plain.ctypes.data), nb, n0, key)
        open_(vp(out.ctypes.data), vp(ok.ctypes.data), vp(body.ctypes.data), nb, n0, key)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    assert ok.all() and np.array_equal(out, plain)
    gib = passes * 2 * nb * BLOCK_DATA / 2**30
    return {"value": round(gib / el, 3), "unit": "GiB/s", "cores": int(threads), "kind": "port",
            "sample": f"{passes} x (seal+open of {nb} x 64KiB blocks) = {gib:.1f} GiB in {el:.1f} s, "
                      f"{impl}, OpenMP over blocks"}


def load_traffic():
    """HBM bytes and VALU instructions per xs_crypt launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/make_traffic.py), or ({}, reason) when there is none or it
    was measured on other kernel sources than the ones built here (sha256 stamp)."""
    from rclone_amd.build import kernel_sources_sha256
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return {}, "no profiles/pmc_traffic.json"
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception as exc:  # noqa: BLE001
        return {}, f"unreadable pmc_traffic.json: {exc}"
    have = kernel_sources_sha256()
    if d.get("kernel_sources_sha256") != have:
        return {}, (f"stale: counters measured on kernel sources {d.get('kernel_sources_sha256', 'unstamped')[:12]}, "
                    f"tree has {have[:12]}")
    return d, None


class ClockProbe:
    """In-window shader clock: one wave beside the crypt kernels (xs_clock_probe_dev, own stream)
    compares s_memtime with the 100 MHz s_memrealtime.  It is launched as the timed region opens
    and ends by itself after a set share of the expected window, so the closing device
    synchronize never waits for it."""

    def __init__(self, L, dev):
        import torch
        self.L, self.torch = L, torch
        self.stop = torch.zeros(1, dtype=torch.int32, device=dev)  # never raised: the probe ends by time
        self.out = torch.zeros(5, dtype=torch.int64, device=dev)
        self.stream = torch.cuda.Stream(dev)
        # its first launch pays the one-time load of the probe's code object (milliseconds):
        # never inside the timed window
        self.start(1e-4)
        self.stream.synchronize()

    def start(self, seconds):
        import ctypes as ct
        from rclone_amd import _lib
        _lib.check(self.L.xs_clock_probe_dev(self.stop.data_ptr(), self.out.data_ptr(), max(seconds, 1e-4),
                                             ct.c_void_p(self.stream.cuda_stream)), "clock probe")

    def result(self):
        self.stream.synchronize()
        t0, r0, t1, r1, n = [int(x) for x in self.out.cpu().tolist()]
        if r1 <= r0:
            return None
        return {"shader_clock_ghz": round((t1 - t0) / (r1 - r0) / 10.0, 4), "window_s": round((r1 - r0) / 1e8, 4),
                "samples": n, "source": "xs_clock_probe_dev: s_memtime / s_memrealtime (100 MHz), one wave on a side "
                                       "stream over the first 80% of the timed steps"}


class PowerSampler:
    """Board power and shader clock over the timed window, read in-process from the rank's amdgpu
    hwmon directory in sysfs (no child process, no GPU call): a thread samples power1_average
    (else power1_input; microwatts) and freq1_input (sclk, Hz) every `period` seconds between
    start() and stop().  When energy1_input (microjoules, a running counter) exists, energy is
    its difference over the window; otherwise the mean sampled power x the window.  Every figure
    is None when the directory or the file is absent (e.g. a container without the device)."""

    def __init__(self, pci, period=0.005):
        import glob
        import threading
        self.threading, self.period = threading, period
        self.dir = None
        dom, bus, dv = pci
        root = os.environ.get("RCLONE_AMD_SYSFS_ROOT") or "/sys"  # the library's sysfs root knob (tests)
        for d in sorted(glob.glob(f"{root}/bus/pci/devices/{dom:04x}:{bus:02x}:{dv:02x}.0/hwmon/hwmon*")):
            if any(os.path.exists(os.path.join(d, f)) for f in ("power1_average", "power1_input")):
                self.dir = d
                break
        self.pfile = self._file("power1_average") or self._file("power1_input")
        self.ffile = self._file("freq1_input")
        self.efile = self._file("energy1_input")
        self.p, self.f = [], []
        self.t0 = self.t1 = self.e0 = self.e1 = None
        self._stop = None

    def _file(self, name):
        if self.dir and os.path.exists(os.path.join(self.dir, name)):
            return os.path.join(self.dir, name)
        return None

    @staticmethod
    def _read(path):
        try:
            with open(path) as fh:
                return int(fh.read().strip())
        except (OSError, ValueError):
            return None

    def _loop(self):
        while not self._stop.wait(self.period):
            if self.pfile:
                v = self._read(self.pfile)
                if v is not None:
                    self.p.append(v * 1e-6)
            if self.ffile:
                v = self._read(self.ffile)
                if v is not None:
                    self.f.append(v * 1e-9)

    def start(self):
        if not self.pfile:
            return
        self.e0 = self._read(self.efile) if self.efile else None
        self._stop = self.threading.Event()
        self._th = self.threading.Thread(target=self._loop, daemon=True)
        self.t0 = time.perf_counter()
        self._th.start()

    def stop(self):
        if not self._stop:
            return
        self.t1 = time.perf_counter()
        self._stop.set()
        self._th.join()
        self.e1 = self._read(self.efile) if self.efile else None

    def result(self):
        """(mean W, joules over the window, mean sclk GHz, dict for the line) or Nones."""
        if not self.p or self.t0 is None:
            return None, None, (sum(self.f) / len(self.f) if self.f else None), \
                {"source": "absent: no amdgpu hwmon power file for this GPU in sysfs"}
        w = sum(self.p) / len(self.p)
        span = self.t1 - self.t0
        if self.e0 is not None and self.e1 is not None and self.e1 > self.e0:
            joules, how = (self.e1 - self.e0) * 1e-6, "energy1_input difference"
        else:
            joules, how = w * span, f"mean of {len(self.p)} {os.path.basename(self.pfile)} samples x window"
        ghz = sum(self.f) / len(self.f) if self.f else None
        return w, joules, ghz, {"source": f"{self.dir} ({how})", "window_s": round(span, 4),
                                "samples": len(self.p), "mean_W": round(w, 1), "min_W": round(min(self.p), 1),
                                "max_W": round(max(self.p), 1),
                                "sclk_ghz_mean": round(ghz, 4) if ghz else None}


def energy_per_gib(rows, total_bytes):
    """Whole-job joules over the timed window (summed over ranks) per GiB pushed through the cipher
    (both directions counted, as `value`); None unless every rank had a power reading."""
    js = [r[4] for r in rows]
    if not js or any(j is None for j in js) or not total_bytes:
        return None
    return round(sum(js) / (total_bytes / 2**30), 4)


def headline_expected_digest(world, nb, independent):
    """The CPU oracle's tag digest of the headline set for this layout, or None when
    tests/golden/fullsize.json does not pin it (another --blocks, --independent, another N)."""
    if os.environ.get("BENCH_FORCE_DIGEST_MISMATCH") == "2":  # tests: a wrong headline digest fails the run
        return "0" * 32
    if independent:
        return None
    from rclone_amd.objectset import fullsize_pins
    hl = fullsize_pins()["bench_headline"]
    if (hl["seed"], hl["key"], hl["nonce0"]) != (HEADLINE_SEED, HEADLINE_KEY.hex(), HEADLINE_NONCE0.hex()):
        return None
    # the set is blocks 0 .. world*nb - 1 of one object whatever the split, and the digest is
    # order-independent: the pin for k ranks of blocks_per_rank covers any world*nb equal to it
    total, per = world * nb, hl["blocks_per_rank"]
    if total % per:
        return None
    return hl["tag_digest"].get(str(total // per))


def per_rank(dist, world, rank, dev, values):
    """Gather one row of floats per rank (one all-reduce of a world x k tensor; the row alone at
    N = 1) -> list of rows, rank order."""
    import torch
    t = torch.zeros((world, len(values)), dtype=torch.float64, device=dev)
    t[rank] = torch.tensor([float("nan") if v is None else float(v) for v in values], dtype=torch.float64)
    if grouped(world):
        # NaN (a rank without a reading) would poison the SUM: carry a mask beside the values
        m = torch.isnan(t)
        t[m] = 0.0
        mask = (~m).to(torch.float64)
        dist.all_reduce(t)
        dist.all_reduce(mask)
        t[mask == 0] = float("nan")
    return [[None if x != x else x for x in row] for row in t.cpu().tolist()]


def spread(col, nd=4):
    """min / max / list of one per-rank column (Nones skipped)."""
    xs = [x for x in col if x is not None]
    if not xs:
        return None
    return {"min": round(min(xs), nd), "max": round(max(xs), nd), "per_rank": [None if x is None else round(x, nd)
                                                                              for x in col]}


def issue_bound(valu_insts, ms, clock_hz=None, mfma_insts=None):
    """VALU roofline of a launch: integer VALU wave-instructions issued per second against the
    chip's issue peak, 256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per wave64 integer instruction
    (measured on gfx950: tools/microbench/issuebench.hip) = 614.4 G wave-instructions/s; and the
    same bound at the clock measured in the timed window.  rocprofv3's SQ_INSTS_VALU also counts
    the matrix-core Poly1305's v_mfma_i32_16x16x64_i8 (SQ_INSTS_VALU_MFMA_I8), which execute on
    the SIMD's matrix pipe: the bound counts the other VALU instructions (valu_insts - mfma_insts)
    and reports the MFMAs beside it.  Without an MFMA count (older PMC stamps) every instruction
    is counted."""
    if not valu_insts:
        return None
    vector = valu_insts - (mfma_insts or 0)
    peak = SIMDS * CLOCK_HZ / VALU_CYC / 1e9
    achieved = vector / (ms * 1e-3) / 1e9
    res = {"bound": "valu", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "G wave-instr/s",
           "frac": round(achieved / peak, 4), "valu_wave_insts": valu_insts, "cycles_per_inst": VALU_CYC}
    if mfma_insts is not None:
        # The MFMAs' own issue cost is left out: SQ_VALU_MFMA_COEXEC_CYCLES shows vector
        # instructions issuing in about half of the matrix pipe's busy cycles, so no fixed
        # per-MFMA hold is a bound (round 3's 8-cycle hold model printed fractions above 1).
        res.update({"mfma_wave_insts": mfma_insts, "vector_wave_insts": vector,
                    "counted": "SQ_INSTS_VALU - SQ_INSTS_VALU_MFMA_I8 (MFMAs run on the matrix pipe)"})
    if clock_hz:
        peak_w = SIMDS * clock_hz / VALU_CYC / 1e9
        res.update({"window_clock_ghz": round(clock_hz / 1e9, 4), "peak_at_window_clock": round(peak_w, 1),
                    "frac_at_window_clock": round(achieved / peak_w, 4)})
    return res


def pool_check_timeout(n_devices):
    """Seconds the pool-check child may take: a base for interpreter start, torch import and the
    oracle check, plus a share per engine (device context + streams + staging)."""
    return 90 + 15 * max(1, n_devices)


def pool_check(devices=None):
    """After the timed region, rank 0 only, outside every timing: the drop-in's one-process spread
    of objects over the node's GPUs (xs_pool over every visible device, the counterpart of
    rclone's --transfers goroutine pool, fs/sync/sync.go:544-548).  A small batched put (crypt
    files of 40 objects, 0 B .. 1 MiB) is split over the devices; every wire body and MD5 must equal
    the CPU oracle's (checker only) and every device must have taken objects.  On a one-GPU box
    it reports the device count and does nothing else.  Never fails the bench: errors are reported."""
    import subprocess

    import torch
    n_dev = torch.cuda.device_count()
    if devices is None:
        if n_dev < 2:
            return {"devices": n_dev, "ran": False}
        devices = list(range(n_dev))
    # in a child process with a time limit: whatever the pool does on a node it has never run
    # on, the bench line still prints.  The limit grows with the device count (each engine opens
    # its device's context and streams; a cold context costs seconds on a fresh node).
    code = ("import json, sys; sys.path.insert(0, %r); import bench; "
            "print(json.dumps(bench._pool_check_body(%r)))" % (ROOT, list(devices)))
    limit = pool_check_timeout(len(devices))
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=limit, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return {"devices": n_dev, "ran": True, "ok": False, "error": f"timed out after {limit} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"devices": n_dev, "ran": True, "ok": False, "error": f"rc {r.returncode}: {r.stderr[-300:]}"}
    return json.loads(lines[-1])


def _pool_check_body(devices):
    import hashlib

    import torch
    n_dev = torch.cuda.device_count()
    try:
        from oracle import pyoracle as orc  # checker only, never timed
        from rclone_amd import _lib, crypt
        from rclone_amd.testdata import splitmix64_bytes
        L = _lib.lib()
        t0 = time.perf_counter()
        pool = crypt.EnginePool(list(devices), batch_blocks=64)
        try:
            engines = [L.xs_engine_device(pool.engine(i)) for i in range(len(pool))]
            key = splitmix64_bytes(0x9001, 32)
            sizes = [0, 1, 65535, 65536, 65537, 1 << 20] + [20011 * k + 3 for k in range(1, 35)]
            plains = [splitmix64_bytes(0x9100 + i, sz) for i, sz in enumerate(sizes)]
            nonces = b"".join(splitmix64_bytes(0x9200 + i, 24) for i in range(len(sizes)))
            offs, pos = [], 0
            for sz in sizes:
                offs.append(pos)
                pos += (sz + 15) & ~15
            stage = bytearray(pos + 16)
            for o, p in zip(offs, plains):
                stage[o:o + len(p)] = p
            cnt = len(sizes)
            u64s = ctypes.c_uint64 * cnt
            lens_c, offs_c = u64s(*sizes), u64s(*offs)
            total = L.xs_put_body_bytes(cnt, lens_c)
            src = (ctypes.c_uint8 * len(stage)).from_buffer(stage)
            body, md5 = (ctypes.c_uint8 * (total + 16))(), (ctypes.c_uint8 * (16 * cnt))()
            rc = L.xs_pool_put_batch(pool.handle, key, cnt, nonces, offs_c, lens_c, src, body, md5)
            if rc != 0:
                return {"devices": n_dev, "ran": True, "ok": False, "error": _lib.last_error()}
            raw, dig, bpos, bad = bytes(body), bytes(md5), 0, 0
            for i, p in enumerate(plains):
                want = orc.encrypt_file(p, nonces[24 * i:24 * i + 24], key)
                bad += raw[bpos:bpos + len(want) - 32] != want[32:] or dig[16 * i:16 * i + 16] != hashlib.md5(want).digest()
                bpos += (len(want) - 32 + 15) & ~15
            took = []
            for i in range(len(pool)):
                st = (ctypes.c_uint64 * 3)()
                L.xs_engine_md5_stats(pool.engine(i), st)
                took.append(int(st[2]))  # objects this engine hashed
        finally:
            pool.close()
        return {"devices": n_dev, "ran": True, "engine_devices": engines, "objects": cnt,
                "objects_differing_from_oracle": int(bad), "engine_objects": took,
                "ok": bad == 0 and all(t > 0 for t in took) and engines == list(devices),
                "seconds": round(time.perf_counter() - t0, 3)}
    except Exception as exc:  # noqa: BLE001 -- reported, never fatal to the bench line
        return {"devices": n_dev, "ran": True, "ok": False, "error": repr(exc)[:300]}


def time_objectset(r, steps, warm, world, dev, dist):
    """Time `steps` full passes of a RankRunner (every round: generate in HBM, seal, open, verify,
    digest) after `warm()`, bracketed by barrier + synchronize on both sides; counters summed and
    the time max-reduced over the ranks.  Returns (seconds, summed counters, kernel ms lists)."""
    import torch

    from rclone_amd import shard
    warm()
    torch.cuda.synchronize(dev)
    r.counters.zero_()
    r.kernel_events.clear()
    if grouped(world):
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        r.run_all(record=True)
    torch.cuda.synchronize(dev)
    if grouped(world):
        dist.barrier()
    el = time.perf_counter() - t0
    counters = r.counters.clone()
    tmax = torch.tensor([el], dtype=torch.float64, device=dev)
    shard.reduce_counters(counters, dist if grouped(world) else None)
    if grouped(world):
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    seal_ms = [a.elapsed_time(b) for s, a, b in r.kernel_events if s]
    open_ms = [a.elapsed_time(b) for s, a, b in r.kernel_events if not s]
    return float(tmax.item()), counters, seal_ms, open_ms


def objectset_leg(args, world, rank, dev, dist):
    """The headline run's configs[3] leg, after the headline timing and outside it: BASELINE
    configs[3]'s 1 TiB object (2^24 blocks, block g sealed with nonce0 + g, cipher.go:665-678)
    round-robin over the N ranks in 100k-block rounds, the same object set
    tests/test_objectset_gpu.py runs (rclone_amd.objectset.CONFIG3_*), so the tag digest here must
    equal the one that test prints for world 1, 2 and 8.  Fixed total work: strong scaling.
    All ranks run it; rank 0 gets the dict, the others None."""
    import torch

    from rclone_amd.objectset import (CONFIG3_BLOCKS, CONFIG3_KEY, CONFIG3_NONCE0, CONFIG3_ROUND_BLOCKS,
                                      CONFIG3_SEED, CONFIG3_TAG_DIGEST, RankRunner, digest_to_u64)
    total = int(os.environ.get("BENCH_OBJECTSET_BLOCKS", CONFIG3_BLOCKS))
    # the round size changes neither the work nor the digest; rehearsals with many ranks on one GPU
    # shrink it to fit eight ranks' buffers in one HBM
    round_blocks = int(os.environ.get("BENCH_OBJECTSET_ROUND_BLOCKS", CONFIG3_ROUND_BLOCKS))
    t_setup = time.perf_counter()
    r = RankRunner(CONFIG3_KEY, CONFIG3_NONCE0, total, world, rank, round_blocks, CONFIG3_SEED, dev)
    setup_s = time.perf_counter() - t_setup

    def warm():
        for _ in range(args.objectset_warmup):
            r.run_all()
    el, counters, seal_ms, open_ms = time_objectset(r, args.objectset_steps, warm, world, dev, dist)
    blocks, nbytes, fails, mism, d0, d1 = digest_to_u64(counters)
    digest = f"{d1:016x}{d0:016x}"  # the last pass's, summed over the ranks
    full = total == CONFIG3_BLOCKS
    expected = CONFIG3_TAG_DIGEST if full else None  # the CPU oracle's pin (full size only)
    if os.environ.get("BENCH_FORCE_DIGEST_MISMATCH") == "1":  # tests: a wrong shard must fail the run
        expected = "f" * 32
    ok = fails == 0 and mism == 0 and blocks == args.objectset_steps * total and (expected is None or digest == expected)
    seal_avg = sum(seal_ms) / max(len(seal_ms), 1)
    open_avg = sum(open_ms) / max(len(open_ms), 1)
    rows = per_rank(dist, world, rank, dev, [seal_avg, open_avg, r.n])
    del r
    torch.cuda.empty_cache()
    if rank != 0:
        return None, ok
    return {"workload": f"BASELINE configs[3]: one {total}-block object ({total * BLOCK_DATA / 2**40:.3f} TiB) "
                        f"round-robin over {world} rank(s), {round_blocks}-block rounds; one step = "
                        "generate in HBM + seal + open + verify every block",
            "value": round(2 * nbytes / 2**30 / el, 3), "unit": "GiB/s", "scaling": "strong",
            "steps": args.objectset_steps, "warmup": args.objectset_warmup,
            "ms_per_step": round(el / args.objectset_steps * 1e3, 3), "ok": ok,
            "seal_kernel_ms_avg": round(seal_avg, 4),
            "open_kernel_ms_avg": round(open_avg, 4),
            "per_rank": {"seal_kernel_ms": spread([x[0] for x in rows]), "open_kernel_ms": spread([x[1] for x in rows]),
                         "blocks_per_pass": [int(x[2]) for x in rows]},
            "setup_s": round(setup_s, 2),
            "counters": {"blocks": blocks, "bytes": nbytes, "tag_failures": fails, "roundtrip_mismatch_words": mism,
                         "tag_digest": digest,
                         "tag_digest_expected": expected,
                         "digest_source": "one pass, summed over ranks; expected = the CPU oracle's digest of all "
                                          "2^24 blocks (tests/golden/fullsize.json config3, "
                                          "tests/golden/make_fullsize.py)"}}, ok


def run_objectset(args, world, rank, dev, dist):
    """BASELINE configs[3]: the rank's round-robin share of an --object-blocks object, in
    --blocks rounds; one step = every round (generate in HBM, seal, open, verify, digest)."""
    from rclone_amd.objectset import CONFIG3_KEY, CONFIG3_NONCE0, CONFIG3_SEED, RankRunner, digest_to_u64
    r = RankRunner(CONFIG3_KEY, CONFIG3_NONCE0, args.object_blocks, world, rank, args.blocks, CONFIG3_SEED, dev)

    def warm():
        for _ in range(args.warmup):
            r.run_round(0)
    el, counters, seal_ms, open_ms = time_objectset(r, args.steps, warm, world, dev, dist)
    blocks, nbytes, fails, mism, d0, d1 = digest_to_u64(counters)
    if fails or mism or blocks != args.steps * args.object_blocks:
        raise SystemExit(f"bench: object set failed (blocks {blocks}, tag failures {fails}, mismatches {mism})")
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(2 * nbytes / 2**30 / el, 3),
            "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (SplitMix64 keyed by global block id, generated in HBM inside each step)",
            "config": {"workload": f"one {args.object_blocks}-block object ({args.object_blocks * BLOCK_DATA / 2**40:.3f} "
                                   f"TiB) round-robin over {world} rank(s), {args.blocks}-block rounds, seal then "
                                   f"open+verify (BASELINE configs[3])",
                       "object_blocks": args.object_blocks, "round_blocks": args.blocks,
                       "parallelism": f"{world} rank(s), blocks sharded, counters all-reduced", **args.topo},
            "build_id": args.build_id,
            "seal_kernel_GiB_s": round(r.n * BLOCK_DATA * args.steps / 2**30 / (sum(seal_ms) * 1e-3), 3),
            "open_kernel_GiB_s": round(r.n * BLOCK_DATA * args.steps / 2**30 / (sum(open_ms) * 1e-3), 3),
            "counters": {"blocks": blocks, "bytes": nbytes, "tag_failures": fails, "roundtrip_mismatch_words": mism,
                         "tag_digest": f"{d1:016x}{d0:016x}"},
            "roofline": None, "cpu_baseline": None,
        }
        print(json.dumps(res), flush=True)
    if grouped(world):
        dist.destroy_process_group()


def run_mixed(args, world, rank, dev, dist):
    """BASELINE configs[2]: decrypt+verify of mixed 4 KiB-8 MiB objects chunked to 64 KiB, with
    tag-fail injection.  Each rank owns its own object set (weak scaling).  The set is sealed on
    the GPU once (sampled blocks checked against the oracle on rank 0), ~0.1% of its blocks get
    one byte flipped (tag bytes, first / last / random ciphertext byte), then one step = seal the
    plaintext image into a second wire image + open+verify the tampered one, each as one
    descriptor batch (keygen + block kernel).  After the timed steps the failing set must be
    exactly the tampered blocks, zero-filled, and every other byte equal to the plaintext."""
    import numpy as np
    import torch

    from rclone_amd import _lib, device, shard
    L = _lib.lib()
    seed = 0xC0F3 + rank
    rng = np.random.default_rng(seed)
    key = bytes(32)  # crypt with an empty password: all-zero data key (cipher.go:231-236)
    sizes, nonces, pstart, wstart, ptot, wtot, d, obj = shard.mixed_object_layout(int(args.mixed_gib * 2**30), rng)
    nb = len(d)
    od = d.copy()
    od["src"], od["dst"] = d["dst"], d["src"]

    def dev_bytes(a):
        return torch.from_numpy(np.frombuffer(a.tobytes(), dtype=np.uint8).copy()).to(dev)
    d_seal, d_open = dev_bytes(d), dev_bytes(od)
    plain = torch.empty(ptot, dtype=torch.uint8, device=dev)
    device.fill_random(plain, seed)
    for o, sz in enumerate(sizes):  # alignment gaps are never written by open: keep them zero
        end = pstart[o] + sz
        nxt = pstart[o + 1] if o + 1 < len(sizes) else ptot
        if nxt > end:
            plain[end:nxt] = 0
    wire_a = torch.zeros(wtot, dtype=torch.uint8, device=dev)
    wire_b = torch.zeros(wtot, dtype=torch.uint8, device=dev)
    out = torch.zeros(ptot, dtype=torch.uint8, device=dev)
    ok = torch.empty(nb, dtype=torch.uint8, device=dev)
    ws_seal = device.workspace(nb, dev)
    ws_open = device.workspace(nb, dev)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def seal(dst, ev=None):
        _lib.check(L.xs_keygen_batch_dev(1, key, d_seal.data_ptr(), nb, plain.data_ptr(), ptot, dst.data_ptr(),
                                         wtot, ws_seal.data_ptr(), sp), "keygen")
        if ev is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
        _lib.check(L.xs_crypt_dev(1, ws_seal.data_ptr(), nb, plain.data_ptr(), dst.data_ptr(), None, sp), "seal")
        if ev is not None:
            b.record(stream)
            ev.append((True, a, b))

    def open_(ev=None):
        _lib.check(L.xs_keygen_batch_dev(0, key, d_open.data_ptr(), nb, wire_a.data_ptr(), wtot, out.data_ptr(),
                                         ptot, ws_open.data_ptr(), sp), "keygen")
        if ev is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
        _lib.check(L.xs_crypt_dev(0, ws_open.data_ptr(), nb, wire_a.data_ptr(), out.data_ptr(), ok.data_ptr(), sp),
                   "open")
        if ev is not None:
            b.record(stream)
            ev.append((False, a, b))

    seal(wire_a)
    torch.cuda.synchronize(dev)
    if rank == 0 and not args.no_cpu:  # the oracle checks sampled blocks (never timed)
        from oracle import pyoracle as orc
        partial = int(np.flatnonzero(d["len"] < BLOCK_DATA)[0])
        carry = int(np.flatnonzero(obj == 0)[-1])  # object 0's nonce carries out of byte 7
        for i in sorted({0, partial, carry, nb // 2, nb - 1}):
            s0, w0, n = int(d["src"][i]), int(d["dst"][i]), int(d["len"][i])
            p = plain[s0:s0 + n].cpu().numpy().tobytes()
            w = wire_a[w0:w0 + 16 + n].cpu().numpy().tobytes()
            if orc.seal(p, bytes(d["nonce"][i]), key) != w:
                raise SystemExit("bench: mixed block %d differs from the oracle" % i)
    nbad = max(3, nb // 1000)
    bad = np.sort(rng.choice(nb, nbad, replace=False))
    pos = []
    for j, b in enumerate(bad.tolist()):
        blen = 16 + int(d["len"][b])
        pos.append(int(d["dst"][b]) + [0, 15, 16, blen - 1, int(rng.integers(0, blen))][j % 5])
    idx = torch.tensor(pos, dtype=torch.int64, device=dev)
    wire_a[idx] ^= 0x40
    for _ in range(args.warmup):
        seal(wire_b)
        open_()
    torch.cuda.synchronize(dev)
    ev = []
    if grouped(world):
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        seal(wire_b, ev)
        open_(ev)
    torch.cuda.synchronize(dev)
    if grouped(world):
        dist.barrier()
    el = time.perf_counter() - t0
    # verification after the timed region: exactly the tampered blocks fail, are zero-filled, the
    # rest is the plaintext; the second wire image equals the first away from the flipped bytes
    fails = np.flatnonzero(ok.cpu().numpy() == 0)
    expect = plain.clone()
    for b in bad.tolist():
        s0, n = int(d["src"][b]), int(d["len"][b])
        expect[s0:s0 + n] = 0
    wire_b[idx] ^= 0x40
    good = np.array_equal(fails, bad) and bool(torch.equal(out, expect)) and bool(torch.equal(wire_a, wire_b))
    del expect
    counters = torch.tensor([args.steps * 2 * nb, args.steps * 2 * int(d["len"].sum()), len(fails),
                             0 if good else 1], dtype=torch.int64, device=dev)
    tmax = torch.tensor([el], dtype=torch.float64, device=dev)
    shard.reduce_counters(counters, dist if grouped(world) else None)
    if grouped(world):
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    el = float(tmax.item())
    if int(counters[3].item()):
        raise SystemExit("bench: mixed object set verification failed")
    seal_ms = [a.elapsed_time(b) for s_, a, b in ev if s_]
    open_ms = [a.elapsed_time(b) for s_, a, b in ev if not s_]
    seal_avg, open_avg = sum(seal_ms) / len(seal_ms), sum(open_ms) / len(open_ms)
    plain_bytes = int(d["len"].sum())
    alg_seal = 2 * plain_bytes + 16 * nb          # read len, write 16 + len per block
    alg_open = 2 * plain_bytes + 16 * nb + nb     # read 16 + len, write len + 1 ok byte
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(int(counters[1].item()) / 2**30 / el, 3),
            "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (SplitMix64 plaintext generated in HBM, seeded object sizes and nonces)",
            "config": {"workload": f"{plain_bytes / 2**30:.2f} GiB per rank of {len(sizes)} objects, sizes "
                                   f"log-uniform 4 KiB-8 MiB, {nb} blocks ({int((d['len'] < BLOCK_DATA).sum())} "
                                   f"partial), {nbad} tampered; seal + open+verify as descriptor batches "
                                   f"(BASELINE configs[2])",
                       "objects": len(sizes), "blocks": nb, "tampered_blocks": nbad,
                       "parallelism": f"{world} rank(s), one object set each, counters all-reduced", **args.topo},
            "build_id": args.build_id,
            "seal_GiB_s": round(plain_bytes / 2**30 / (seal_avg * 1e-3), 3),
            "open_GiB_s": round(plain_bytes / 2**30 / (open_avg * 1e-3), 3),
            "roofline": {"bound": "hbm", "kernel": "xs_open", "achieved": round(alg_open / (open_avg * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg_open / (open_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel_ms_avg": round(open_avg, 4), "alg_bytes_per_launch": alg_open,
                         "seal": {"kernel": "xs_seal", "kernel_ms_avg": round(seal_avg, 4),
                                  "achieved": round(alg_seal / (seal_avg * 1e-3) / 1e9, 1),
                                  "frac": round(alg_seal / (seal_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}},
            "counters": {"blocks": int(counters[0].item()), "bytes": int(counters[1].item()),
                         "tag_failures_last_step": int(counters[2].item()), "verified": True},
            "cpu_baseline": None,
        }
        print(json.dumps(res), flush=True)
    if grouped(world):
        dist.destroy_process_group()


def names_cpu_baseline(segs, key, tweak, seconds):
    """Oracle EME (oracle/eme_oracle.c) over a bounded sample, one core, C loop per name."""
    from oracle import pyoracle as orc  # checker/baseline only
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        orc.eme_transform(key, tweak, orc.pkcs7_pad(segs[k % len(segs)]), True)
        k += 1
    dt = time.perf_counter() - t0
    return {"value": round(k / dt), "unit": "names/s", "cores": 1, "kind": "port",
            "sample": f"{k} single-segment names encrypted by oracle/eme_oracle.c in {dt:.1f} s "
                      "(one ctypes call per name; EME only, no encoding)"}


def run_names(args, world, rank):
    """configs-independent secondary bench: batched file-name encryption (EME-AES-256 + pkcs7 +
    base32) and decryption of a synthetic listing, through the C ABI (rc_names_run).  One step =
    encrypt N names then decrypt them; value = names/s both directions counted, summed over ranks
    (each rank its own listing, weak scaling).  The EME kernel's own time comes from HIP events
    inside rc_names_run."""
    import numpy as np
    import torch
    from rclone_amd import _lib, crypt, names
    L = _lib.lib()
    n = args.names
    rng = np.random.default_rng(1000 + rank)
    lens = rng.integers(8, 65, n)
    pool = rng.integers(ord("a"), ord("z") + 1, int(lens.sum()), dtype=np.uint8).tobytes()
    segs, p = [], 0
    for ln in lens:
        segs.append(pool[p:p + ln])
        p += ln
    if args.name_paths:
        inp = [b"dir%03d/sub%04d/" % (i % 997, i % 7919) + s for i, s in enumerate(segs)]
    else:
        inp = segs
    c = crypt.new_cipher(names.NAME_ENCRYPTION_STANDARD, "potato", "", True, names.new_name_encoding("base32"))

    def carr(lst):
        a = (ctypes.c_char_p * n)(*lst)
        ln = (ctypes.c_uint64 * n)(*[len(x) for x in lst])
        return a, ln

    def run(op, arr, lens_):
        out = ctypes.c_void_p()
        rc = L.rc_names_run(c._h, op, n, arr, lens_, ctypes.byref(out))
        if rc != 0:
            raise SystemExit(f"rc_names_run failed: {rc} {_lib.last_error()}")
        return out

    def collect(h):
        vals = []
        ptr, ln, err, arg = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_int64()
        for i in range(n):
            L.rc_names_get(h, i, ctypes.byref(ptr), ctypes.byref(ln), ctypes.byref(err), ctypes.byref(arg))
            if err.value:
                raise SystemExit(f"name {i}: error {err.value}")
            vals.append(ctypes.string_at(ptr.value, ln.value))
        return vals

    op_e = names.OP_ENCRYPT_FILE_NAME
    op_d = names.OP_DECRYPT_FILE_NAME
    pa, pl = carr(inp)
    h = run(op_e, pa, pl)
    enc = collect(h)
    L.rc_names_free(h)
    ea, el_ = carr(enc)
    h = run(op_d, ea, el_)
    if collect(h) != inp:
        raise SystemExit("names: round trip failed")
    L.rc_names_free(h)
    for _ in range(args.warmup):
        L.rc_names_free(run(op_e, pa, pl))
        L.rc_names_free(run(op_d, ea, el_))
    if grouped(world):
        import torch.distributed as dist
        dist.barrier()
    k_e, k_d, t_e, t_d = [], [], [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        h = run(op_e, pa, pl)
        k_e.append(L.rc_names_kernel_ms(h))
        L.rc_names_free(h)
        b = time.perf_counter()
        h = run(op_d, ea, el_)
        k_d.append(L.rc_names_kernel_ms(h))
        L.rc_names_free(h)
        t_e.append(b - a)
        t_d.append(time.perf_counter() - b)
    el = time.perf_counter() - t0
    if grouped(world):
        import torch.distributed as dist
        t = torch.tensor([el], dtype=torch.float64, device="cuda")  # RCCL reduces device tensors only
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        padded = int(((lens // 16) + 1).sum()) * 16
        ke, kd = float(np.mean(k_e)), float(np.mean(k_d))
        res = {
            "metric": "file names/s, crypt EME-AES-256 name encrypt+decrypt (rc_names_run, host-resident)",
            "value": round(2 * n * args.steps * world / el), "unit": "names/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (lowercase names, 8-64 bytes)",
            "config": {"workload": f"{n} {'3-segment paths' if args.name_paths else 'names'} per rank, "
                                   "EncryptFileName then DecryptFileName, base32, standard mode",
                       "names_per_rank": n, "paths": bool(args.name_paths), **args.topo},
            "build_id": args.build_id,
            "encrypt_s": round(float(np.mean(t_e)), 4), "decrypt_s": round(float(np.mean(t_d)), 4),
            "kernel": {"encrypt_ms": round(ke, 4), "decrypt_ms": round(kd, 4),
                       "segments_per_launch": n * (3 if args.name_paths else 1),
                       "segment_bytes_padded": padded,
                       "kernel_names_per_s": round(n / (ke * 1e-3))},
            "cpu_baseline": None,
        }
        if not args.no_cpu and world == 1:  # the CPU baseline is an N=1 figure (rank 0 only)
            res["cpu_baseline"] = names_cpu_baseline(segs, c.name_key, c.name_tweak, 5.0)
        print(json.dumps(res), flush=True)
    if grouped(world):
        import torch.distributed as dist
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                         f"(--nproc-per-node {args.gpus}) or drop the launcher and let bench.py start the ranks")
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo rehearses the N>1 path on a box with fewer GPUs than ranks (ranks
    # share GPUs round-robin; counters and times go through gloo).  The real run is RCCL, one
    # rank per GPU.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if args.dry_run:
        if grouped(world):
            dist.init_process_group("gloo", **pg_init_kwargs(world))
        return run_dry(args, world, rank, dist)
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > 1 and ndev < world:
        raise SystemExit(f"bench: {world} ranks over RCCL need {world} GPUs, {ndev} visible "
                         "(BENCH_DIST_BACKEND=gloo rehearses ranks sharing GPUs)")
    gpu = local % max(ndev, 1) if backend == "gloo" else local
    # the C library's engines (rc_* handles, file names) run on this rank's GPU too
    os.environ.setdefault("RCLONE_AMD_DEVICE", str(gpu))
    if grouped(world):
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu), **pg_init_kwargs(world))
        else:
            dist.init_process_group(backend, **pg_init_kwargs(world))
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    from rclone_amd import _lib
    _lib.lib()  # refuses a library not built from this tree's sources (build id)
    args.build_id = _lib.build_id()
    args.topo = rank_topology(dist, world, dev)
    if args.topo["ranks_seen"] != args.gpus:
        raise SystemExit(f"bench: process group has {args.topo['ranks_seen']} ranks, --gpus {args.gpus}")

    if args.object_blocks:
        return run_objectset(args, world, rank, dev, dist)
    if args.names:
        return run_names(args, world, rank)
    if args.mixed_gib:
        return run_mixed(args, world, rank, dev, dist)

    import numpy as np

    from rclone_amd import _lib, device, shard
    L = _lib.lib()
    nb = args.blocks
    plain_len = nb * BLOCK_DATA
    body_len = nb * BLOCK_SIZE
    key, nonce0 = HEADLINE_KEY, HEADLINE_NONCE0
    # this rank's round-robin share of one logical object of world*nb blocks (BASELINE config 4
    # layout); per-block nonces via descriptors, blocks packed contiguously in local HBM
    gidx = shard.owned_blocks(world * nb, world, rank)
    ds, do = shard.seal_descriptors(nonce0, gidx), shard.seal_descriptors(nonce0, gidx, open_mode=True)
    if args.independent:  # object g = global block g, nonce from a seeded stream (same for any world size)
        allnon = np.random.default_rng(0x0B1EC7).integers(0, 256, size=(world * nb, 24), dtype=np.uint8)
        ds["nonce"] = do["nonce"] = allnon[gidx]
    block_nonce = [bytes(x) for x in ds["nonce"][[0, 1, nb // 2, nb - 1]]]
    d_seal = torch.from_numpy(ds.view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(do.view(np.uint8).copy()).to(dev)
    plain = torch.empty(plain_len, dtype=torch.uint8, device=dev)
    device.fill_blocks(plain, rank, world, HEADLINE_SEED)  # global block g = rank + world*i, keyed by g
    body = torch.empty(body_len, dtype=torch.uint8, device=dev)
    out = torch.empty(plain_len, dtype=torch.uint8, device=dev)
    ok = torch.empty(nb, dtype=torch.uint8, device=dev)
    ws_seal = device.workspace(nb, dev)
    ws_open = device.workspace(nb, dev)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    ev = []  # (seal?, start, end) around every xs_crypt launch

    def step(record):
        _lib.check(L.xs_keygen_batch_dev(1, key, d_seal.data_ptr(), nb, plain.data_ptr(), plain_len,
                                         body.data_ptr(), body_len, ws_seal.data_ptr(), sp), "keygen")
        if record:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
        _lib.check(L.xs_crypt_dev(1, ws_seal.data_ptr(), nb, plain.data_ptr(), body.data_ptr(), None, sp), "seal")
        if record:
            b.record(stream)
            ev.append((True, a, b))
        _lib.check(L.xs_keygen_batch_dev(0, key, d_open.data_ptr(), nb, body.data_ptr(), body_len,
                                         out.data_ptr(), plain_len, ws_open.data_ptr(), sp), "keygen")
        if record:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
        _lib.check(L.xs_crypt_dev(0, ws_open.data_ptr(), nb, body.data_ptr(), out.data_ptr(), ok.data_ptr(), sp),
                   "open")
        if record:
            b.record(stream)
            ev.append((False, a, b))

    # correctness gate first, on one step: round trip + every tag verified + sampled blocks bit-exact
    # against the oracle (rank 0 only; the oracle is the checker, never timed).  The warm-up then
    # runs straight into the timed region, so the clock and the board power are settled when it
    # starts (a host-side check between the two would let the GPU idle and cool)
    step(False)
    torch.cuda.synchronize(dev)
    if not (torch.equal(out, plain) and int(ok.sum()) == nb):
        raise SystemExit("bench: round trip failed on rank %d" % rank)
    if rank == 0 and not args.no_cpu:
        from oracle import pyoracle as orc
        for j, i in enumerate([0, 1, nb // 2, nb - 1]):
            p = plain[i * BLOCK_DATA:(i + 1) * BLOCK_DATA].cpu().numpy().tobytes()
            w = body[i * BLOCK_SIZE:(i + 1) * BLOCK_SIZE].cpu().numpy().tobytes()
            if orc.seal(p, block_nonce[j], key) != w:
                raise SystemExit("bench: block %d differs from the oracle" % i)
    # the clock probe runs at N=1 only (RCCL's own streams could share its hardware queue)
    probe = ClockProbe(L, dev) if world == 1 else None
    props = torch.cuda.get_device_properties(dev)
    power = PowerSampler((props.pci_domain_id, props.pci_bus_id, props.pci_device_id))
    if grouped(world):
        dist.barrier()
    tw = time.perf_counter()
    nwarm, tail = 0, []
    while nwarm < args.warmup or time.perf_counter() - tw < args.warmup_seconds:
        ts = time.perf_counter()
        for _ in range(4):
            step(False)
        torch.cuda.synchronize(dev)  # keep the host within a few steps of the device
        tail = (tail + [(time.perf_counter() - ts) / 4])[-4:]
        nwarm += 4
    warm_s = time.perf_counter() - tw
    step_s = sorted(tail)[len(tail) // 2]  # settled per-step time: sizes the clock probe's window
    if grouped(world):
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if probe:
        probe.start(0.8 * args.steps * step_s)
    power.start()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    power.stop()
    el_rank = time.perf_counter() - t0  # this rank's own steps (the straggler view)
    if grouped(world):
        dist.barrier()
    el = time.perf_counter() - t0
    clock = probe.result() if probe else None
    if clock and el > 1.5 * args.steps * step_s:  # the probe must never have held the steps back
        clock["warning"] = f"timed region {el:.4f} s vs {args.steps * step_s:.4f} s expected"
    if not torch.equal(out, plain):  # the last timed step's round trip (after the timing)
        raise SystemExit("bench: round trip failed after the timed steps on rank %d" % rank)
    # counters and max time over ranks (RCCL, small tensors only)
    from rclone_amd.objectset import tag_digest
    counters = torch.tensor([args.steps * 2 * nb, args.steps * 2 * plain_len, int(nb - int(ok.sum())), 0, 0],
                            dtype=torch.int64, device=dev)
    counters[3:5] = tag_digest(body, nb)  # order-independent: the same for any world size
    tmax = torch.tensor([el], dtype=torch.float64, device=dev)
    shard.reduce_counters(counters, dist if grouped(world) else None)
    if grouped(world):
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    el = float(tmax.item())
    seal_ms = [a.elapsed_time(b) for s, a, b in ev if s]
    open_ms = [a.elapsed_time(b) for s, a, b in ev if not s]
    seal_avg = sum(seal_ms) / len(seal_ms)
    open_avg = sum(open_ms) / len(open_ms)
    watts, joules, sclk, power_info = power.result()
    rows = per_rank(dist, world, rank, dev, [el_rank, seal_avg, open_avg, watts, joules, sclk])
    # the headline set's tag digest against the CPU oracle's (tests/golden/fullsize.json), for the
    # layouts it pins: --blocks 100000 at 1/2/4/8 ranks, one object (not --independent)
    digest = "%016x%016x" % (int(counters[4].item()) & (2**64 - 1), int(counters[3].item()) & (2**64 - 1))
    expect = headline_expected_digest(world, nb, args.independent)
    digest_ok = expect is None or digest == expect
    # configs[3] leg: every rank, after the headline's timing and reduction (never inside them)
    objset, objset_ok = objectset_leg(args, world, rank, dev, dist) if args.objectset_steps > 0 else (None, None)
    if os.environ.get("BENCH_TRACE"):
        print("seal_ms", [round(x, 3) for x in seal_ms], "\nopen_ms", [round(x, 3) for x in open_ms],
              file=sys.stderr)
    total_bytes = int(counters[1].item())
    value = total_bytes / 2**30 / el
    if rank == 0:
        ach_seal = ALG_BYTES_SEAL * nb / (seal_avg * 1e-3) / 1e9
        ach_open = ALG_BYTES_OPEN * nb / (open_avg * 1e-3) / 1e9
        tr, stale = load_traffic()
        # PMC figures are per launch of the default workload; scale if nb differs
        pmc_nb = tr.get("blocks_per_launch", nb)
        scale = nb / pmc_nb if pmc_nb else 1.0
        clk_hz = clock["shader_clock_ghz"] * 1e9 if clock else None

        def per(key):
            v = tr.get(key)
            return round(v * scale) if v else None
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SplitMix64 plaintext generated in HBM)",
            "config": {"workload": (f"{nb} x 64KiB device-resident one-block objects per GPU, each with its own "
                                    f"random nonce" if args.independent else
                                    f"{nb} x 64KiB device-resident blocks per GPU (round-robin share of "
                                    f"one {world * nb}-block object)") +
                                   ", seal then open+verify (BASELINE configs[1]+[2] shape)",
                       "blocks_per_gpu": nb, "block_bytes": BLOCK_DATA,
                       "parallelism": f"{world} rank(s), blocks sharded, no data-path collective", **args.topo},
            "build_id": args.build_id,
            "seal_GiB_s": round(nb * BLOCK_DATA / 2**30 / (seal_avg * 1e-3), 3),
            "open_GiB_s": round(nb * BLOCK_DATA / 2**30 / (open_avg * 1e-3), 3),
            "roofline": {"bound": "hbm", "kernel": "xs_seal",
                         "achieved": round(ach_seal, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach_seal / HBM_PEAK_GBS, 4),
                         "traffic": per("seal_bytes_per_launch"),
                         "kernel_ms_avg": round(seal_avg, 4),
                         "alg_bytes_per_launch": ALG_BYTES_SEAL * nb,
                         # SURVEY 8(d)'s HBM-read roofline: the bytes the kernel must read (65536
                         # plaintext per block) per second against the same 8 TB/s
                         "read_achieved": round(READ_BYTES_SEAL * nb / (seal_avg * 1e-3) / 1e9, 1),
                         "read_frac": round(READ_BYTES_SEAL * nb / (seal_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic_source": tr.get("source") if tr else stale,
                         "traffic_git_head": tr.get("git_head"),
                         "valu": issue_bound(per("seal_valu_wave_insts_per_launch"), seal_avg, clk_hz,
                                             per("seal_mfma_wave_insts_per_launch")),
                         "open": {"kernel": "xs_open", "achieved": round(ach_open, 1),
                                  "frac": round(ach_open / HBM_PEAK_GBS, 4), "kernel_ms_avg": round(open_avg, 4),
                                  "read_achieved": round(READ_BYTES_OPEN * nb / (open_avg * 1e-3) / 1e9, 1),
                                  "read_frac": round(READ_BYTES_OPEN * nb / (open_avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                                     4),
                                  "traffic": per("open_bytes_per_launch"),
                                  "valu": issue_bound(per("open_valu_wave_insts_per_launch"), open_avg, clk_hz,
                                                      per("open_mfma_wave_insts_per_launch"))}},
            "clock": clock,
            "energy_J_per_GiB": energy_per_gib(rows, total_bytes),
            "power": power_info,
            "per_rank": {"step_ms": spread([r[0] * 1e3 / args.steps for r in rows], 3),
                         "seal_kernel_ms": spread([r[1] for r in rows]),
                         "open_kernel_ms": spread([r[2] for r in rows]),
                         "power_W": spread([r[3] for r in rows], 1),
                         "sclk_ghz": spread([r[5] for r in rows])},
            "warmup_s": round(warm_s, 3), "warmup_steps": nwarm,
            "counters": {"blocks": int(counters[0].item()), "bytes": total_bytes,
                         "tag_failures": int(counters[2].item()),
                         "tag_digest": digest, "tag_digest_expected": expect, "tag_digest_ok": digest_ok,
                         "digest_source": "summed over ranks; expected = CPU oracle, tests/golden/fullsize.json "
                                          "bench_headline (tests/golden/make_fullsize.py)"},
            "cpu_baseline": None,
            "objectset": objset,
        }
    # the group is torn down before rank 0's after-timing checks: the other ranks leave (and free
    # their GPUs) instead of waiting in the group while the pool check opens every device
    if grouped(world):
        dist.destroy_process_group()
    if rank == 0:
        if not args.no_cpu and world == 1:  # the CPU baseline is an N=1 figure (rank 0 only)
            res["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        if not args.no_pool_check:
            res["pool_check"] = pool_check()
        print(json.dumps(res), flush=True)
    fail_if_wrong(digest_ok, digest, expect, int(counters[2].item()), objset_ok)


if __name__ == "__main__":
    main()
