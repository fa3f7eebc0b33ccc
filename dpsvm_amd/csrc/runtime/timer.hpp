// Timers (reference C9: CycleTimer.h:37-175 — rdtsc x parsed CPU GHz, result
// truncated to whole seconds when stored in an unsigned long long,
// svmTrainMain.cpp:206-208,312-314).  Here: monotonic steady_clock in double
// seconds for host regions, and hipEvent pairs for device regions on a stream.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>

namespace dpsvm {

using Clock = std::chrono::steady_clock;

inline double secs_since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// wall-clock stopwatch (double seconds, no truncation)
class Stopwatch {
 public:
  Stopwatch() : t0_(Clock::now()) {}
  void reset() { t0_ = Clock::now(); }
  double seconds() const { return secs_since(t0_); }

 private:
  Clock::time_point t0_;
};

// device-side interval on one stream: start()/stop() enqueue events, seconds()
// waits for the stop event
class EventTimer {
 public:
  EventTimer() {
    (void)hipEventCreate(&a_);
    (void)hipEventCreate(&b_);
  }
  ~EventTimer() {
    if (a_) (void)hipEventDestroy(a_);
    if (b_) (void)hipEventDestroy(b_);
  }
  EventTimer(const EventTimer&) = delete;
  EventTimer& operator=(const EventTimer&) = delete;
  void start(hipStream_t s) { (void)hipEventRecord(a_, s); }
  void stop(hipStream_t s) { (void)hipEventRecord(b_, s); }
  double seconds() const {
    float ms = 0.f;
    if (hipEventSynchronize(b_) != hipSuccess) return -1.0;
    if (hipEventElapsedTime(&ms, a_, b_) != hipSuccess) return -1.0;
    return ms * 1e-3;
  }

 private:
  hipEvent_t a_ = nullptr, b_ = nullptr;
};

}  // namespace dpsvm
