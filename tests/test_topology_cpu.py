"""Node topology of the multi-GPU host path, CPU only: the device list
parser (RCLONE_AMD_DEVICES, repeats allowed) and the sysfs mapping PCI bus id -> NUMA node ->
CPU list that places each engine's pinned staging and host threads, against a fake sysfs root
(RCLONE_AMD_SYSFS_ROOT).  Thread pinning and the scoped memory policy are checked inside the
sanitizer harness (tests/native/sanitize_main.cpp test_topology).  Unmeasured on a multi-socket
node: the development box has one GPU.
"""
import ctypes

import pytest

from rclone_amd import _lib


def _devices(s):
    out = (ctypes.c_int * 16)()
    n = _lib.lib().xs_parse_device_list(s.encode(), out, 16)
    return list(out[:min(n, 16)])


def test_device_list_parsing():
    assert _devices("0,1,1,2") == [0, 1, 1, 2]  # repeats: several engines on one device
    assert _devices("3, 4") == [3, 4]
    assert _devices("0,x,2") == [0]
    assert _devices("") == [] and _devices("x") == []
    assert _devices(",7,,") == [7]


@pytest.fixture
def fake_sysfs(tmp_path, monkeypatch):
    def put(rel, text):
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)
    # an 8-GPU, two-socket node: GPUs 0-3 on node 0, 4-7 on node 1
    for g, bus in enumerate(["05", "15", "65", "75", "85", "95", "e5", "f5"]):
        put(f"bus/pci/devices/0000:{bus}:00.0/numa_node", "%d\n" % (0 if g < 4 else 1))
    put("bus/pci/devices/0000:aa:00.0/numa_node", "-1\n")  # single-node kernels report -1
    put("devices/system/node/node0/cpulist", "0-47,96-143\n")
    put("devices/system/node/node1/cpulist", "48-95,144-191\n")
    put("devices/system/node/node2/cpulist", "garbage\n")
    monkeypatch.setenv("RCLONE_AMD_SYSFS_ROOT", str(tmp_path))
    return tmp_path


def test_pci_bus_id_to_node(fake_sysfs):
    lib = _lib.lib()
    assert lib.xs_pci_numa_node(b"0000:05:00.0") == 0
    assert lib.xs_pci_numa_node(b"0000:E5:00.0") == 1  # hipDeviceGetPCIBusId may use upper case
    assert lib.xs_pci_numa_node(b"0000:aa:00.0") == -1
    assert lib.xs_pci_numa_node(b"0000:00:00.0") == -1  # no such function
    assert lib.xs_pci_numa_node(b"") == -1


def test_node_cpu_lists(fake_sysfs):
    lib = _lib.lib()
    buf = (ctypes.c_int * 256)()
    n = lib.xs_numa_node_cpus(1, buf, 256)
    assert n == 96 and list(buf[:n]) == list(range(48, 96)) + list(range(144, 192))
    assert lib.xs_numa_node_cpus(0, buf, 4) == 96 and list(buf[:4]) == [0, 1, 2, 3]  # count past cap
    assert lib.xs_numa_node_cpus(2, buf, 256) == 0  # malformed
    assert lib.xs_numa_node_cpus(5, buf, 256) == 0  # absent
    assert lib.xs_numa_node_cpus(-1, buf, 256) == 0


def test_device_numa_node_without_device():
    # no HIP device here: unknown, never an error
    assert _lib.lib().xs_device_numa_node(0) == -1
    assert _lib.lib().xs_engine_numa_node(None) == -1


def test_effective_cpus_follows_the_cgroup_quota(fake_sysfs, monkeypatch):
    lib = _lib.lib()
    aff = len(__import__("os").sched_getaffinity(0))
    cg = fake_sysfs / "fs" / "cgroup"
    cg.mkdir(parents=True)
    (cg / "cpu.max").write_text("max 100000\n")  # no quota: the affinity mask
    assert lib.xs_effective_cpus() == aff
    (cg / "cpu.max").write_text("150000 100000\n")  # 1.5 CPUs of quota -> 2
    assert lib.xs_effective_cpus() == min(aff, 2)
    monkeypatch.setenv("RCLONE_AMD_CPUS", "5")
    assert lib.xs_effective_cpus() == 5


def test_effective_cpus_nested_cgroup_quota(fake_sysfs, tmp_path, monkeypatch):
    """A process in a nested cgroup v2 group without a namespace (a systemd slice with
    CPUQuota): the quota is the smallest cpu.max on the path from /proc/self/cgroup's group up to
    the mount root, not only the root's file."""
    import os
    lib = _lib.lib()
    aff = len(os.sched_getaffinity(0))
    proc = tmp_path / "proc"
    (proc / "self").mkdir(parents=True)
    (proc / "self" / "cgroup").write_text("1:cpu:/\n0::/system.slice/rclone.service\n")
    monkeypatch.setenv("RCLONE_AMD_PROC_ROOT", str(proc))
    cg = fake_sysfs / "fs" / "cgroup"
    (cg / "system.slice" / "rclone.service").mkdir(parents=True)
    (cg / "system.slice" / "rclone.service" / "cpu.max").write_text("max 100000\n")
    (cg / "system.slice" / "cpu.max").write_text("300000 100000\n")  # the slice: 3 CPUs
    assert lib.xs_effective_cpus() == min(aff, 3)
    (cg / "system.slice" / "rclone.service" / "cpu.max").write_text("100000 100000\n")  # tighter below
    assert lib.xs_effective_cpus() == 1
    (cg / "cpu.max").write_text("200000 100000\n")  # root looser than the group: the group wins
    assert lib.xs_effective_cpus() == 1
    (proc / "self" / "cgroup").write_text("0::/\n")  # a namespace: the root file only
    assert lib.xs_effective_cpus() == min(aff, 2)
    (proc / "self" / "cgroup").write_text("0::/../escape\n")  # never leaves the mount
    assert lib.xs_effective_cpus() == min(aff, 2)
