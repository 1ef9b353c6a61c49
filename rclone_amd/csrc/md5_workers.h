// md5_workers.h -- host hashing for the per-object ciphertext MD5 of the streaming paths: crypt.put's
// tee hash (backend/crypt/crypt.go:516-533) and computeHashWithNonce's io.Copy into the hasher
// (crypt.go:799-803), which unchanged callers run one object at a time per goroutine (--transfers /
// --checkers).  MD5 is one dependency chain per stream, so a stream is sped up only by
// overlapping its hashing with its other work, and many streams only by hashing them at once.
//
// Where a job (the next piece of one stream) is hashed, in order of preference:
//   1. a scalar worker thread (min(8, cores / 2) per NUMA node), when one is free and the caller
//      has other work to overlap it with (a stream's read and seal of its next batch, or the
//      consumer reading the batch) -- the fastest chain per stream (~1.1 GB/s on a Zen 5 core);
//   2. the caller's own thread, while the streams hashing on host cores stay within the
//      process's CPU budget (affinity and cgroup quota) -- same speed, no hand-off;
//   3. past that budget, a lane of the 16-stream AVX-512 engine (md5_x16.h): each lane runs at
//      about half a scalar chain (0.48 GB/s on Zen 5) but a core carries 16 of them (7.7 GB/s),
//      so many more streams than cores (a high --checkers) still progress together.
// A stream submits its jobs one at a time (it waits for job k before submitting job k+1), so its
// bytes are hashed in order whichever tier takes each job.
#pragma once
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "md5_x16.h"
#include "rc_internal.h"
#include "xs_host_md5.h"

namespace xs {

class Md5Workers;
struct Md5Job {
  HostMd5* st = nullptr;
  const uint8_t* p = nullptr;
  size_t n = 0;
  std::atomic<int> busy{0};  // 1 from submit until the bytes are hashed (2: a waiter sleeps on it)
  const Md5Workers* owner = nullptr;
  // multi-buffer engine: the whole blocks left after HostMd5::begin_blocks
  const uint8_t* blk = nullptr;
  size_t nblk = 0;
};

// Where jobs went (cumulative, all nodes): scalar workers, callers' threads, engine lanes.
struct Md5TierStats {
  std::atomic<uint64_t> worker{0}, inline_{0}, lanes{0};
  std::atomic<uint64_t> worker_ns{0}, worker_bytes{0};  // scalar workers' hashing time and bytes
};
inline Md5TierStats& md5_tier_stats() {
  static Md5TierStats* s = new Md5TierStats();
  return *s;
}

class Md5Workers {
 public:
  // max_threads scalar workers; scalar_budget scalar chains on host cores at once before streams
  // go to the engine; lane_threads engine threads at most (16 streams each).
  Md5Workers(int max_threads, int node, int scalar_budget, bool lanes, int lane_threads)
      : max_(max_threads), node_(node), budget_(std::max(1, scalar_budget)), lanes_on_(lanes && md5_x16_supported()),
        lane_threads_max_(std::max(1, lane_threads)) {}

  // Hash j->st with j->p[0:n], here or later; the caller waits with wait() before touching j->st
  // or reusing j->p.  overlap: the caller has other work to do meanwhile (else a hand-off to a
  // scalar worker only adds a wake-up).
  void submit(Md5Job* j, bool overlap = true) {
    if (max_ > 0 && overlap) {
      std::unique_lock<std::mutex> g(mu_);
      const bool spawn = (int)q_.size() >= idle_ && (int)th_.size() < max_;
      if ((int)q_.size() < idle_ || spawn) {
        j->owner = this;
        j->busy.store(1, std::memory_order_relaxed);
        q_.push_back(j);
        if (spawn)
          th_.emplace_back([this] {
            pin_thread_to_node(node_);  // the node of the engines whose streams it hashes
            run();
          });
        cv_.notify_one();
        md5_tier_stats().worker++;
        return;
      }
    }
    // scalar chains already on host cores: busy workers + callers hashing now
    const int on_cores = inline_.load(std::memory_order_relaxed) + busy_workers_.load(std::memory_order_relaxed);
    if (!lanes_on_ || on_cores < budget_) {
      inline_.fetch_add(1, std::memory_order_relaxed);
      j->st->update(j->p, j->n);
      inline_.fetch_sub(1, std::memory_order_relaxed);
      md5_tier_stats().inline_++;
      return;
    }
    // past the CPU budget: the leading partial block here, the whole blocks on an engine lane
    j->blk = j->st->begin_blocks(j->p, j->n, &j->nblk);
    if (j->nblk == 0) return;
    std::unique_lock<std::mutex> g(mu_);
    j->owner = this;
    j->busy.store(1, std::memory_order_relaxed);
    lq_.push_back(j);
    if (lane_idle_ == 0 && (int)lth_.size() < lane_threads_max_ &&
        (int)lq_.size() + lane_active_ > 16 * (int)lth_.size())
      lth_.emplace_back([this] {
        pin_thread_to_node(node_);
        run_lanes();
      });
    lcv_.notify_one();
    md5_tier_stats().lanes++;
  }

  // Each job has its own wake-up: busy is 1 while hashing, 2 once a waiter sleeps on it (a
  // private futex on the job's own word), so finishing a job wakes only that job's waiter and
  // costs no syscall when nobody sleeps -- never a broadcast to every stream's waiter.
  void wait(Md5Job* j) const {
    if (!j->busy.load(std::memory_order_acquire)) return;
    for (int k = 0; k < 64; k++) {  // a job hashes ~1 MiB (~1 ms): spin only briefly
      if (!j->busy.load(std::memory_order_acquire)) return;
      std::this_thread::yield();
    }
    for (;;) {
      int v = j->busy.load(std::memory_order_acquire);
      if (v == 0) return;
      if (v == 1 && !j->busy.compare_exchange_strong(v, 2, std::memory_order_acq_rel)) {
        if (v == 0) return;
      }
      syscall(SYS_futex, reinterpret_cast<int*>(&j->busy), FUTEX_WAIT_PRIVATE, 2, nullptr, nullptr, 0);
    }
  }

 private:
  static void finish(Md5Job* j) {
    // the private-futex wake only hashes the address: safe even if the waiter has already seen 0
    // and released the job
    if (j->busy.exchange(0, std::memory_order_acq_rel) == 2)
      syscall(SYS_futex, reinterpret_cast<int*>(&j->busy), FUTEX_WAKE_PRIVATE, INT32_MAX, nullptr, nullptr, 0);
  }

  void run() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      idle_++;
      cv_.wait(lk, [&] { return !q_.empty(); });
      idle_--;
      Md5Job* j = q_.front();
      q_.pop_front();
      busy_workers_.fetch_add(1, std::memory_order_relaxed);
      lk.unlock();
      const auto t0 = std::chrono::steady_clock::now();
      j->st->update(j->p, j->n);
      md5_tier_stats().worker_ns.fetch_add(
          (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(),
          std::memory_order_relaxed);
      md5_tier_stats().worker_bytes.fetch_add(j->n, std::memory_order_relaxed);
      lk.lock();
      busy_workers_.fetch_sub(1, std::memory_order_relaxed);
      finish(j);
    }
  }

  // One engine thread: 16 lanes, each carrying one job's whole blocks; the lanes advance together
  // up to 64 blocks at a time, so new jobs join within ~16 us.
  void run_lanes() {
    alignas(64) static const uint8_t zero_block[64] = {0};
    uint32_t st[4][16];
    const uint8_t* p[16];
    uint32_t stride[16];
    Md5Job* lane[16] = {nullptr};
    size_t rem[16] = {0};
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      int nact = 0;
      for (int i = 0; i < 16; i++) {
        if (!lane[i] && !lq_.empty()) {
          Md5Job* j = lq_.front();
          lq_.pop_front();
          lane[i] = j;
          rem[i] = j->nblk;
          p[i] = j->blk;
          const uint32_t* s = j->st->state();
          for (int w = 0; w < 4; w++) st[w][i] = s[w];
          lane_active_++;
        }
        nact += lane[i] != nullptr;
      }
      if (nact == 0) {
        lane_idle_++;
        lcv_.wait(lk, [&] { return !lq_.empty(); });
        lane_idle_--;
        continue;
      }
      size_t k = 64;
      for (int i = 0; i < 16; i++) {
        if (lane[i]) {
          k = std::min(k, rem[i]);
          stride[i] = 64;
        } else {
          p[i] = zero_block;
          stride[i] = 0;
        }
      }
      lk.unlock();
      md5_x16_blocks(st, p, stride, k);
      lk.lock();
      for (int i = 0; i < 16; i++) {
        if (!lane[i]) continue;
        rem[i] -= k;
        p[i] += 64 * k;
        if (rem[i] == 0) {
          uint32_t* s = lane[i]->st->state();
          for (int w = 0; w < 4; w++) s[w] = st[w][i];
          finish(lane[i]);
          lane[i] = nullptr;
          lane_active_--;
        }
      }
    }
  }

  const int max_, node_, budget_;
  const bool lanes_on_;
  const int lane_threads_max_;
  mutable std::mutex mu_;
  mutable std::condition_variable cv_, lcv_;
  std::deque<Md5Job*> q_, lq_;
  std::vector<std::thread> th_, lth_;
  int idle_ = 0, lane_idle_ = 0, lane_active_ = 0;
  std::atomic<int> inline_{0}, busy_workers_{0};
};

// Process-wide workers, one set per NUMA node (never destroyed: threads stay parked until exit).
// XS_MD5_WORKERS: scalar workers per node (0: none), default min(8, cores / 2); XS_MD5_LANES=0
// turns the 16-stream engine off; the CPU budget is the process's usable CPUs (affinity and the
// cgroup quota, effective_cpus()).
inline Md5Workers& md5_workers(int node) {
  constexpr int kNodes = 64;
  static std::mutex mu;
  static Md5Workers* w[kNodes + 1] = {nullptr};
  const int slot = node >= 0 && node < kNodes ? node + 1 : 0;
  std::lock_guard<std::mutex> g(mu);
  if (!w[slot]) {
    const int cpus = effective_cpus();
    int n;
    if (const char* e = getenv("XS_MD5_WORKERS")) n = std::max(0, atoi(e));
    else n = std::max(1, std::min(8, cpus / 2));
    const char* l = getenv("XS_MD5_LANES");
    // scalar chains on host cores at once (workers + callers) before streams go to engine lanes
    int budget = cpus;
    if (const char* b = getenv("XS_MD5_SCALAR_BUDGET")) budget = std::max(1, atoi(b));
    w[slot] = new Md5Workers(n, slot - 1, budget, l ? atoi(l) != 0 : true, std::max(1, cpus / 4));
  }
  return *w[slot];
}

// Wait for a job submitted to any node's workers (no-op for an idle job).
inline void md5_wait(Md5Job* j) {
  if (!j->busy.load(std::memory_order_acquire)) return;
  j->owner->wait(j);
}

}  // namespace xs
