// Latency floors used to judge the SMO iteration kernels (bench/iter_latency.py):
// the cost of a chain of dependent, (nearly) empty kernels replayed from a
// hipGraph — the "boundary" row of the MI355X price list — so the fused
// iteration's time can be split into launch floor vs. in-kernel latency.
#include <hip/hip_runtime.h>

#include <chrono>

#include "../runtime/hip_check.hpp"
#include "device_util.hpp"
#include "kernels.hpp"

namespace dpsvm {
namespace dev {

// each kernel reads one word written by its predecessor (a true dependency)
__global__ void chain_kernel(const int* __restrict__ in, int* __restrict__ out) {
  const int v = in[0];
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = v + 1;
}

// Known-bytes stream for pinning FETCH_SIZE (bench/fetch_probe.py): every 16-B
// chunk of x read exactly once by 16-B loads (full 128-B lines per 8 lanes, the
// access shape of the wide pass 1 and of the GEMMs' LDS-DMA), four loads in
// flight per lane, a per-workgroup sum written so nothing is dead code.
__global__ __launch_bounds__(256) void stream_read_kernel(const float4* __restrict__ x, int64_t n16,
                                                          float* __restrict__ out) {
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const float4 a = x[i], b = x[i + stride], c = x[i + 2 * stride], d = x[i + 3 * stride];
    acc += (a.x + a.y + a.z + a.w) + (b.x + b.y + b.z + b.w) + (c.x + c.y + c.z + c.w) + (d.x + d.y + d.z + d.w);
  }
  for (; i < n16; i += stride) {
    const float4 a = x[i];
    acc += a.x + a.y + a.z + a.w;
  }
  acc = wave_sum(acc);
  __shared__ float s_w[4];
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

}  // namespace dev

namespace launch {

void stream_read(const void* x, int64_t bytes, float* out, int blocks, hipStream_t s) {
  DPSVM_CHECK(bytes % 16 == 0 && ((uintptr_t)x & 15) == 0, "stream_read: 16-B aligned whole chunks");
  dev::stream_read_kernel<<<dim3((unsigned)blocks), 256, 0, s>>>((const float4*)x, bytes / 16, out);
  post_launch("stream_read", s);
}

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
