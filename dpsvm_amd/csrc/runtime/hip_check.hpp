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
inline void post_launch(const char* what, hipStream_t s, bool force_sync = false) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e));
  if (force_sync || sync_debug_env()) {
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) fail(std::string("kernel failed (") + what + "): " + hipGetErrorString(e));
  }
}
}  // namespace dpsvm
