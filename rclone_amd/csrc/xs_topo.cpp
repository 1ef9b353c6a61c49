// xs_topo.cpp -- node topology for the multi-GPU host path.
//
// One rclone process spreads its --transfers / --checkers streams over the node's GPUs
// (fs/sync/sync.go:544 startTransfers hands objects to a goroutine pool; xs_pool hands each stream
// an engine).  On a two-socket 8-GPU node half of the GPUs hang off each socket, so an engine's
// host-side resources -- its pinned staging, the handles' staging buffers and the host threads
// that hash or feed its objects -- belong on the NUMA node of the engine's GPU, or every byte
// crosses the socket link twice.  This file holds the host-only part: the sysfs lookups (PCI bus
// id -> NUMA node -> CPU list), the device-list parser, thread pinning and a scoped memory policy
// for pinned allocations.  The HIP part (device -> PCI bus id) is in xs_api.cpp.
//
// The sysfs root is RCLONE_AMD_SYSFS_ROOT (default /sys) so tests can point it at a fake tree.
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rc_internal.h"

namespace xs {

static std::string sysfs_root() {
  const char* r = getenv("RCLONE_AMD_SYSFS_ROOT");
  return r && *r ? std::string(r) : std::string("/sys");
}

static bool read_line(const std::string& path, std::string* out) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  const bool ok = fgets(buf, sizeof buf, f) != nullptr;
  fclose(f);
  if (!ok) return false;
  out->assign(buf);
  while (!out->empty() && isspace((unsigned char)out->back())) out->pop_back();
  return true;
}

// "0000:C1:00.0" -> NUMA node from <root>/bus/pci/devices/0000:c1:00.0/numa_node; -1 if unknown
// (no such file, or the kernel reports -1 on a single-node machine)
int pci_numa_node(const char* busid) {
  if (!busid || !*busid) return -1;
  std::string id(busid);
  for (auto& ch : id) ch = (char)tolower((unsigned char)ch);
  std::string v;
  if (!read_line(sysfs_root() + "/bus/pci/devices/" + id + "/numa_node", &v) || v.empty()) return -1;
  char* end = nullptr;
  const long n = strtol(v.c_str(), &end, 10);
  if (end == v.c_str() || n < 0 || n > 4095) return -1;
  return (int)n;
}

// Linux cpulist format: "0-15,32-47" (ranges and single ids, comma separated); false if malformed
bool parse_cpulist(const char* s, std::vector<int>* out) {
  out->clear();
  if (!s) return false;
  const char* p = s;
  while (*p) {
    while (*p == ' ' || *p == ',') p++;
    if (!*p || *p == '\n') break;
    char* end = nullptr;
    const long a = strtol(p, &end, 10);
    if (end == p || a < 0) return false;
    long b = a;
    p = end;
    if (*p == '-') {
      p++;
      b = strtol(p, &end, 10);
      if (end == p || b < a) return false;
      p = end;
    }
    if (b - a > 65536) return false;
    for (long c = a; c <= b; c++) out->push_back((int)c);
    if (*p && *p != ',' && *p != '\n' && *p != ' ') return false;
  }
  return true;
}

bool node_cpus(int node, std::vector<int>* cpus) {
  cpus->clear();
  if (node < 0) return false;
  std::string v;
  if (!read_line(sysfs_root() + "/devices/system/node/node" + std::to_string(node) + "/cpulist", &v)) return false;
  return parse_cpulist(v.c_str(), cpus) && !cpus->empty();
}

// "0,1,1,2" -> {0,1,1,2} (repeats allowed: several engines on one device); stops at the first
// entry that is not a number.  Returns the count.
int parse_device_list(const char* s, std::vector<int>* out) {
  out->clear();
  if (!s) return 0;
  const char* p = s;
  while (*p) {
    while (*p == ',' || *p == ' ') p++;
    if (!*p) break;
    char* end = nullptr;
    const long d = strtol(p, &end, 10);
    if (end == p || d < 0) break;
    out->push_back((int)d);
    p = end;
  }
  return (int)out->size();
}

// The process's cgroup v2 path ("/a/b" from "0::/a/b" in /proc/self/cgroup; "" when unknown)
static std::string self_cgroup() {
  const char* proc = getenv("RCLONE_AMD_PROC_ROOT");
  std::string self;
  FILE* f = fopen(((proc && *proc ? std::string(proc) : std::string("/proc")) + "/self/cgroup").c_str(), "r");
  if (f) {
    char buf[4096];
    while (fgets(buf, sizeof buf, f)) {
      if (strncmp(buf, "0::", 3) == 0) {
        self.assign(buf + 3);
        while (!self.empty() && isspace((unsigned char)self.back())) self.pop_back();
        break;
      }
    }
    fclose(f);
  }
  if (self == "/" || self.find("..") != std::string::npos) self.clear();
  return self;
}

// The CPUs the process's cgroup allows (cgroup v2 cpuset.cpus.effective of its own group, else of
// the mount root); false when no such file is readable.  This is what `docker --cpuset-cpus`, a
// systemd AllowedCPUs= or a cpuset update after load set for the whole process.
static bool cgroup_cpuset(cpu_set_t* set) {
  const std::string base = sysfs_root() + "/fs/cgroup";
  std::string v;
  const std::string self = self_cgroup();
  if (!(!self.empty() && read_line(base + self + "/cpuset.cpus.effective", &v)) &&
      !read_line(base + "/cpuset.cpus.effective", &v))
    return false;
  std::vector<int> cpus;
  if (!parse_cpulist(v.c_str(), &cpus) || cpus.empty()) return false;
  CPU_ZERO(set);
  for (int c : cpus)
    if (c < CPU_SETSIZE) CPU_SET(c, set);
  return CPU_COUNT(set) > 0;
}

// The process's CPU affinity, read again whenever the library sizes a pool or pins one of its
// threads.  Its first source is the main thread's mask (read by pid, not by the calling thread, so
// a thread the library has already pinned to one node does not shrink it): what the operator gave
// the process with taskset / numactl / the container.  That mask can also be narrowed by the host
// program itself -- OMP_PROC_BIND binding the initial thread, an embedding runtime pinning its main
// thread -- which says nothing about the CPUs the process may use.  So when it is
// narrower than the mask captured at load, the union of the two counts, cut to the cgroup's cpuset
// when one is readable (a cpuset narrowed after load is the operator's, and is honoured), and the
// library says so once on stderr.  The mask at load is the fallback when the main thread cannot be
// queried.
static cpu_set_t g_process_cpus;
static bool g_process_cpus_ok = false;
static std::atomic<bool> g_narrow_logged{false};

void capture_process_affinity() {
  CPU_ZERO(&g_process_cpus);
  g_process_cpus_ok = sched_getaffinity(0, sizeof g_process_cpus, &g_process_cpus) == 0 && CPU_COUNT(&g_process_cpus) > 0;
}

[[maybe_unused]] static const bool g_captured_at_load = (capture_process_affinity(), true);

static bool process_cpus(cpu_set_t* set) {
  CPU_ZERO(set);
  cpu_set_t cur;
  CPU_ZERO(&cur);
  if (!(sched_getaffinity(getpid(), sizeof cur, &cur) == 0 && CPU_COUNT(&cur) > 0)) {
    if (!g_process_cpus_ok) return false;
    *set = g_process_cpus;
    return true;
  }
  *set = cur;
  if (!g_process_cpus_ok || CPU_COUNT(&cur) >= CPU_COUNT(&g_process_cpus)) return true;
  cpu_set_t u, cs;
  CPU_OR(&u, &cur, &g_process_cpus);
  if (cgroup_cpuset(&cs)) {
    cpu_set_t in;
    CPU_AND(&in, &u, &cs);
    if (CPU_COUNT(&in) > 0) u = in;
  }
  *set = u;
  if (!g_narrow_logged.exchange(true))
    fprintf(stderr,
            "rclone_amd: the main thread's CPU mask (%d CPUs) is narrower than the process's at load (%d); "
            "pool sizing and thread pinning use %d CPUs (load-time mask%s)\n",
            CPU_COUNT(&cur), CPU_COUNT(&g_process_cpus), CPU_COUNT(&u),
            CPU_COUNT(&u) < CPU_COUNT(&g_process_cpus) ? " cut to the cgroup cpuset" : "");
  return true;
}

// cgroup v2: the quota that binds this process is the smallest cpu.max on the path from its own
// group (/proc/self/cgroup "0::/a/b") up to the mount root, so a nested group (a systemd slice
// with CPUQuota, no cgroup namespace) is honoured as well as a container's root-level file.
static double cgroup_v2_quota(const std::string& root) {
  double quota = -1;
  auto consider = [&](const std::string& dir) {
    std::string v;
    if (!read_line(dir + "/cpu.max", &v)) return false;  // "max 100000" or "1600000 100000"
    long long q = 0, per = 0;
    if (sscanf(v.c_str(), "%lld %lld", &q, &per) == 2 && q > 0 && per > 0) {
      const double f = (double)q / (double)per;
      if (quota < 0 || f < quota) quota = f;
    }
    return true;
  };
  std::string self = self_cgroup();
  const std::string base = root + "/fs/cgroup";
  // walk /a/b -> /a -> "" (the mount root); a path that does not resolve under this mount (a
  // cgroup namespace shows "/") simply finds no files below the root
  while (!self.empty() && self != "/" && self.find("..") == std::string::npos) {
    consider(base + self);
    const size_t cut = self.find_last_of('/');
    if (cut == std::string::npos) break;
    self.resize(cut);
  }
  if (!consider(base) && quota < 0) return -2;  // no v2 file at the root either: try v1
  return quota;
}

// CPUs this process can use: its affinity mask (as it is now), capped by the cgroup CPU quota (v2
// cpu.max along the process's own group path, or v1 cpu.cfs_quota_us / cpu.cfs_period_us under
// the sysfs root); RCLONE_AMD_CPUS overrides.  A GPU box share of 16 cores on a 256-CPU machine
// is 16, not 256.
int effective_cpus() {
  if (const char* e = getenv("RCLONE_AMD_CPUS")) {
    const int v = atoi(e);
    if (v > 0) return v;
  }
  cpu_set_t mask;
  int n = process_cpus(&mask) ? CPU_COUNT(&mask) : (int)std::thread::hardware_concurrency();
  const std::string root = sysfs_root();
  double quota = cgroup_v2_quota(root);
  if (quota == -2) {
    quota = -1;
    std::string a, b;
    if (read_line(root + "/fs/cgroup/cpu/cpu.cfs_quota_us", &a) && read_line(root + "/fs/cgroup/cpu/cpu.cfs_period_us", &b)) {
      const long long q = atoll(a.c_str()), per = atoll(b.c_str());
      if (q > 0 && per > 0) quota = (double)q / (double)per;
    }
  }
  if (quota > 0) n = std::min(n, std::max(1, (int)(quota + 0.999)));
  return std::max(1, n);
}

// Pin the calling thread to the CPUs of `node` that the process may use (the node's CPU list
// intersected with the process affinity as it is now).  No-op when the node or its CPU list
// is unknown, the intersection is empty, or RCLONE_AMD_NUMA=0.  Only threads this library starts
// are pinned -- never a caller's thread.
void pin_thread_to_node(int node) {
  if (!numa_enabled()) return;
  std::vector<int> cpus;
  if (!node_cpus(node, &cpus)) return;
  cpu_set_t mask, set;
  const bool have_mask = process_cpus(&mask);
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c < CPU_SETSIZE && (!have_mask || CPU_ISSET(c, &mask))) CPU_SET(c, &set);
  if (CPU_COUNT(&set) == 0) return;
  (void)sched_setaffinity(0, sizeof set, &set);
}

bool numa_enabled() {
  static const bool on = [] {
    const char* v = getenv("RCLONE_AMD_NUMA");
    return v ? atoi(v) != 0 : true;
  }();
  return on;
}

// Preferred-node memory policy for the calling thread while in scope (pinned allocations made in
// it land on `node`); restores the previous policy.  No-op for node < 0.
ScopedMemPolicy::ScopedMemPolicy(int node) {
  if (node < 0 || node >= 1024 || !numa_enabled()) return;
  unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
  if (syscall(SYS_get_mempolicy, &old_mode_, old_mask_, 1024ul, nullptr, 0ul) != 0) return;
  mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
  const int kMpolPreferred = 1;
  active_ = syscall(SYS_set_mempolicy, kMpolPreferred, mask, 1024ul) == 0;
}

ScopedMemPolicy::~ScopedMemPolicy() {
  if (active_) (void)syscall(SYS_set_mempolicy, old_mode_, old_mask_, 1024ul);
}

}  // namespace xs

extern "C" int xs_pci_numa_node(const char* pci_bus_id) { return xs::pci_numa_node(pci_bus_id); }

extern "C" int xs_numa_node_cpus(int node, int* cpus, int cap) {
  std::vector<int> v;
  if (!xs::node_cpus(node, &v)) return 0;
  for (int i = 0; i < cap && i < (int)v.size(); i++) cpus[i] = v[i];
  return (int)v.size();
}

extern "C" int xs_effective_cpus(void) { return xs::effective_cpus(); }

extern "C" int xs_parse_device_list(const char* list, int* out, int cap) {
  std::vector<int> v;
  xs::parse_device_list(list, &v);
  for (int i = 0; i < cap && i < (int)v.size(); i++) out[i] = v[i];
  return (int)v.size();
}
