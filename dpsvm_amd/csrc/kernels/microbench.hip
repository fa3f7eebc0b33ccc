// Latency floors used to judge the SMO iteration kernels (bench/iter_latency.py):
// the cost of a chain of dependent, (nearly) empty kernels replayed from a
// hipGraph — the "boundary" row of the MI355X price list — so the fused
// iteration's time can be split into launch floor vs. in-kernel latency.
#include <hip/hip_runtime.h>

#include <chrono>

#include "../runtime/hip_check.hpp"
#include "kernels.hpp"

namespace dpsvm {
namespace dev {

// each kernel reads one word written by its predecessor (a true dependency)
__global__ void chain_kernel(const int* __restrict__ in, int* __restrict__ out) {
  const int v = in[0];
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = v + 1;
}

}  // namespace dev

namespace launch {

double launch_floor_us(int blocks, int threads, int chain, int reps) {
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* buf;
  HIP_CHECK(hipMalloc(&buf, 2 * sizeof(int)));
  HIP_CHECK(hipMemsetAsync(buf, 0, 2 * sizeof(int), s));
  hipGraph_t g;
  hipGraphExec_t ge;
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  for (int i = 0; i < chain; ++i)
    dev::chain_kernel<<<dim3(blocks), threads, 0, s>>>(buf + (i & 1), buf + ((i + 1) & 1));
  HIP_CHECK(hipStreamEndCapture(s, &g));
  HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphLaunch(ge, s));  // warm
  HIP_CHECK(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) HIP_CHECK(hipGraphLaunch(ge, s));
  HIP_CHECK(hipStreamSynchronize(s));
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipFree(buf);
  (void)hipStreamDestroy(s);
  return us / ((double)reps * chain);
}

}  // namespace launch
}  // namespace dpsvm
