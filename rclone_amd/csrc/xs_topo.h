// xs_topo.h -- node topology helpers (xs_topo.cpp): NUMA placement of each engine's host-side
// resources on a multi-socket, multi-GPU node.
#pragma once
#include <vector>

namespace xs {
// ---- node topology (xs_topo.cpp): NUMA placement of each engine's host-side resources
int pci_numa_node(const char* busid);                       // sysfs; -1 when unknown
bool parse_cpulist(const char* s, std::vector<int>* out);   // "0-15,32-47"
bool node_cpus(int node, std::vector<int>* cpus);           // false when unknown / empty
int parse_device_list(const char* s, std::vector<int>* out);
bool numa_enabled();                                        // RCLONE_AMD_NUMA (default 1)
int effective_cpus();  // affinity, capped by the cgroup CPU quota (RCLONE_AMD_CPUS overrides)
void pin_thread_to_node(int node);  // library-started threads only, inside the process's mask
void capture_process_affinity();    // re-read the process mask (done at load; tests)
class ScopedMemPolicy {  // preferred-node policy of the calling thread while in scope
 public:
  explicit ScopedMemPolicy(int node);
  ~ScopedMemPolicy();
  ScopedMemPolicy(const ScopedMemPolicy&) = delete;
  ScopedMemPolicy& operator=(const ScopedMemPolicy&) = delete;

 private:
  bool active_ = false;
  int old_mode_ = 0;
  unsigned long old_mask_[1024 / (8 * sizeof(unsigned long))] = {0};
};
}  // namespace xs
