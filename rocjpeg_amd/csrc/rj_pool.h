// rj_pool.h -- a small persistent host worker pool for the per-call byte staging of a decode
// handle (rj_decoder.cpp): the bitstreams of non-resident streams are copied into pinned memory
// in chunks by the workers while the calling thread hands each finished chunk, in order, to the
// DMA engine (hipMemcpyAsync).  HIP calls stay on the calling thread.
//
// The reference copies each image's slice data into a VA buffer on the calling thread
// (src/rocjpeg_vaapi_decoder.cpp:677-689, vaCreateBuffer); here one call stages a whole batch.
#pragma once
#include <atomic>
#include <exception>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace rj {

class HostPool {
 public:
  // `threads` includes the caller: threads - 1 workers are started (lazily, on the first Run).
  explicit HostPool(int threads) : want_(threads < 1 ? 1 : threads) {}
  ~HostPool() {
    {
      std::lock_guard<std::mutex> l(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  int threads() const { return want_; }

  // Runs task(k) for k in [0, n) on the workers and the caller (only the caller when `serial`);
  // the caller also runs done(k) for every k in increasing k as soon as tasks 0..k have all
  // finished (done may be empty).  Returns after every task and every done() call.  An exception
  // thrown by a task (on any thread) or by done() is caught, every worker is let finish this job,
  // and the first one is rethrown on the calling thread (rj_api.cpp's Guard maps it to a status).
  void Run(int n, const std::function<void(int)> &task, const std::function<void(int)> &done, bool serial = false) {
    if (n <= 0) return;
    if (want_ == 1 || n == 1 || serial) {
      for (int k = 0; k < n; k++) {
        task(k);
        if (done) done(k);
      }
      return;
    }
    Start();
    first_error_ = nullptr;
    failed_.store(false, std::memory_order_relaxed);
    flags_.reset(new std::atomic<uint8_t>[n]);
    for (int k = 0; k < n; k++) flags_[k].store(0, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> l(mu_);
      task_ = &task;
      ntask_ = n;
      next_.store(0, std::memory_order_relaxed);
      active_ = int(workers_.size());
      gen_++;
    }
    cv_.notify_all();
    int flushed = 0;
    auto flush = [&] {
      while (flushed < n && flags_[flushed].load(std::memory_order_acquire)) {
        if (done && !failed_.load(std::memory_order_relaxed)) Guarded([&] { done(flushed); });
        flushed++;
      }
    };
    for (;;) {
      const int k = next_.fetch_add(1, std::memory_order_relaxed);
      if (k >= n) break;
      if (!failed_.load(std::memory_order_relaxed)) Guarded([&] { task(k); });
      flags_[k].store(1, std::memory_order_release);
      flush();
    }
    while (flushed < n) {
      flush();
      if (flushed < n) std::this_thread::yield();
    }
    {
      std::unique_lock<std::mutex> l(mu_);  // every worker has left this job (task_ stays valid until then)
      idle_cv_.wait(l, [&] { return active_ == 0; });
      task_ = nullptr;
    }
    if (failed_.load(std::memory_order_acquire)) {
      std::exception_ptr e;
      {
        std::lock_guard<std::mutex> l(mu_);
        e = first_error_;
        first_error_ = nullptr;
      }
      std::rethrow_exception(e);
    }
  }

 private:
  void Start() {
    if (!workers_.empty()) return;
    for (int t = 1; t < want_; t++) workers_.emplace_back([this] { Loop(); });
  }
  void Loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)> *task;
      int n;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
        task = task_;
        n = ntask_;
      }
      for (;;) {
        const int k = next_.fetch_add(1, std::memory_order_relaxed);
        if (k >= n) break;
        if (!failed_.load(std::memory_order_relaxed)) Guarded([&] { (*task)(k); });  // (later tasks are skipped)
        flags_[k].store(1, std::memory_order_release);
      }
      std::lock_guard<std::mutex> l(mu_);
      if (--active_ == 0) idle_cv_.notify_all();
    }
  }

  // runs f, keeping the first exception of the job (a worker must never let one escape)
  template <typename F>
  void Guarded(F &&f) {
    try {
      f();
    } catch (...) {
      std::lock_guard<std::mutex> l(mu_);
      if (!first_error_) first_error_ = std::current_exception();
      failed_.store(true, std::memory_order_release);
    }
  }

  const int want_;
  std::exception_ptr first_error_;
  std::atomic<bool> failed_{false};
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  bool quit_ = false;
  uint64_t gen_ = 0;
  const std::function<void(int)> *task_ = nullptr;
  int ntask_ = 0, active_ = 0;
  std::atomic<int> next_{0};
  std::unique_ptr<std::atomic<uint8_t>[]> flags_;
};

}  // namespace rj
