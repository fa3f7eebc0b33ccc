// HIP error checking (the reference checks almost no CUDA/cuBLAS return codes,
// SURVEY Q19).  DPSVM_SYNC_DEBUG=1 additionally synchronises and checks after
// every kernel launch.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "dpsvm/common.hpp"

#define HIP_CHECK(expr)                                                                      \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      ::dpsvm::fail(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr " [" \
                    __FILE__ ":" + std::to_string(__LINE__) + "]");                          \
  } while (0)

namespace dpsvm {
inline bool sync_debug_env() {
  static const bool v = [] {
    const char* e = std::getenv("DPSVM_SYNC_DEBUG");
    return e && e[0] == '1';
  }();
  return v;
}
// Launch-side caches that hold device pointers or per-device state are keyed by
// the calling thread's current device: svmTrain -p N runs one rank per device
// as threads of ONE process, so a process-wide cache filled by device 0 would
// hand device 0's memory to ranks 1..N-1.
constexpr int kMaxDevices = 64;
inline int current_device() {
  int d = 0;
  HIP_CHECK(hipGetDevice(&d));
  if (d < 0 || d >= kMaxDevices) fail("current_device: device id out of range");
  return d;
}
inline void post_launch(const char* what, hipStream_t s, bool force_sync = false) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e));
  if (force_sync || sync_debug_env()) {
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) fail(std::string("kernel failed (") + what + "): " + hipGetErrorString(e));
  }
}
}  // namespace dpsvm
