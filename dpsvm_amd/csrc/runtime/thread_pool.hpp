// Small persistent fork-join pool for the CPU solver's per-iteration loops.
// (The reference CPU path, seq.cpp, is single-threaded; spawning threads per
// SMO iteration would cost more than the work, so workers stay parked.)
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#if defined(__x86_64__) || defined(__i386__)
#include <xmmintrin.h>
#endif

namespace dpsvm {

// Flush-to-zero + denormals-are-zero on this thread's SSE unit; returns the
// previous control word (restore with set_fp_control).  Late SMO iterations
// multiply tiny alpha steps by kernel values: with denormal results every
// such multiply takes a microcode assist (x86), ~10x the time of the update.
inline unsigned flush_denormals() {
#if defined(__x86_64__) || defined(__i386__)
  const unsigned old = _mm_getcsr();
  _mm_setcsr(old | 0x8040u);  // FTZ (bit 15) | DAZ (bit 6)
  return old;
#else
  return 0u;
#endif
}
inline void set_fp_control(unsigned v) {
#if defined(__x86_64__) || defined(__i386__)
  _mm_setcsr(v);
#else
  (void)v;
#endif
}

class ThreadPool {
 public:
  // ftz: workers run with flush-to-zero / denormals-are-zero
  explicit ThreadPool(int threads, bool ftz = false) : nthreads_(threads < 1 ? 1 : threads) {
    for (int t = 1; t < nthreads_; ++t)
      workers_.emplace_back([this, t, ftz] {
        if (ftz) flush_denormals();
        loop(t);
      });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& w : workers_) w.join();
  }
  int size() const { return nthreads_; }

  // fn(thread_index, begin, end) over [0, n) split in nthreads contiguous chunks
  void run(int64_t n, const std::function<void(int, int64_t, int64_t)>& fn, int64_t min_chunk = 2048) {
    int t = nthreads_;
    if (n < min_chunk * 2 || t == 1) {
      fn(0, 0, n);
      return;
    }
    if ((int64_t)t * min_chunk > n) t = (int)(n / min_chunk);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      n_ = n;
      active_ = t;
      pending_.store(t - 1);
      ++gen_;
    }
    cv_.notify_all();
    fn(0, 0, n / t);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_.load() == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int idx) {
    uint64_t seen = 0;
    while (true) {
      const std::function<void(int, int64_t, int64_t)>* job;
      int64_t n;
      int active;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        job = job_;
        n = n_;
        active = active_;
      }
      if (job && idx < active) {
        (*job)(idx, n * idx / active, n * (idx + 1) / active);
        if (pending_.fetch_sub(1) == 1) {
          std::lock_guard<std::mutex> lk(mu_);
          done_cv_.notify_one();
        }
      }
    }
  }

  int nthreads_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int, int64_t, int64_t)>* job_ = nullptr;
  int64_t n_ = 0;
  int active_ = 0;
  std::atomic<int> pending_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace dpsvm
