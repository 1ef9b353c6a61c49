// md5_workers.h -- host worker threads for the per-object ciphertext MD5 of the streaming paths:
// crypt.put's tee hash (backend/crypt/crypt.go:516-533) and computeHashWithNonce's io.Copy into
// the hasher (crypt.go:799-803), which unchanged callers run one object at a time per goroutine
// (--transfers / --checkers).  MD5 is one dependency chain per stream, so a stream can only be
// sped up by overlapping its hashing with its other work: while a worker hashes batch k of a
// stream, the stream's own thread reads and seals batch k+1 (the GPU seals it) or serves it to
// the consumer.  Jobs of one stream are submitted one at a time (the stream waits for job k before
// submitting job k+1), so a stream's bytes are hashed in order.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "rc_internal.h"
#include "xs_host_md5.h"

namespace xs {

class Md5Workers;
struct Md5Job {
  HostMd5* st = nullptr;
  const uint8_t* p = nullptr;
  size_t n = 0;
  std::atomic<int> busy{0};  // 1 from submit until the worker has hashed the bytes
  const Md5Workers* owner = nullptr;
};

class Md5Workers {
 public:
  Md5Workers(int max_threads, int node) : max_(max_threads), node_(node) {}
  int max_threads() const { return max_; }
  // j->st is updated with j->p[0:n] on a worker; the caller waits with wait() before touching
  // j->st or reusing j->p.  When every worker is taken (or there are none: max_threads 0) the
  // hash runs here, on the caller's thread: a queued job would only wait for a worker, while the
  // caller can hash it now -- so with more streams than workers each stream still has a core.
  void submit(Md5Job* j) {
    if (max_ > 0) {
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
        return;
      }
    }
    j->st->update(j->p, j->n);
  }
  void wait(Md5Job* j) const {
    if (!j->busy.load(std::memory_order_acquire)) return;
    for (int k = 0; k < 64; k++) {  // a job hashes ~1 MiB (~1 ms): spin only briefly
      if (!j->busy.load(std::memory_order_acquire)) return;
      std::this_thread::yield();
    }
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return !j->busy.load(std::memory_order_acquire); });
  }

 private:
  void run() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      idle_++;
      cv_.wait(lk, [&] { return !q_.empty(); });
      idle_--;
      Md5Job* j = q_.front();
      q_.pop_front();
      lk.unlock();
      j->st->update(j->p, j->n);
      lk.lock();
      j->busy.store(0, std::memory_order_release);
      done_.notify_all();  // under mu_: a waiter checks busy under mu_ too, so no lost wake-up
    }
  }
  const int max_, node_;
  mutable std::mutex mu_;
  mutable std::condition_variable cv_, done_;
  std::deque<Md5Job*> q_;
  std::vector<std::thread> th_;
  int idle_ = 0;
};

// Process-wide workers, one set per NUMA node (never destroyed: threads stay parked until exit).
// XS_MD5_WORKERS sets their number per node (0: every stream hashes on its own thread); default
// min(8, cores / 2).
inline Md5Workers& md5_workers(int node) {
  constexpr int kNodes = 64;
  static std::mutex mu;
  static Md5Workers* w[kNodes + 1] = {nullptr};
  const int slot = node >= 0 && node < kNodes ? node + 1 : 0;
  std::lock_guard<std::mutex> g(mu);
  if (!w[slot]) {
    int n;
    if (const char* e = getenv("XS_MD5_WORKERS")) {
      n = std::max(0, atoi(e));
    } else {
      const unsigned hc = std::thread::hardware_concurrency();
      n = (int)std::max(1u, std::min(8u, hc ? hc / 2 : 1u));
    }
    w[slot] = new Md5Workers(n, slot - 1);
  }
  return *w[slot];
}

// Wait for a job submitted to any node's workers (no-op for an idle job).
inline void md5_wait(Md5Job* j) {
  if (!j->busy.load(std::memory_order_acquire)) return;
  j->owner->wait(j);
}

}  // namespace xs
