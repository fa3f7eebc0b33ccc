// Setup kernels shared by every engine: |x|^2 of every row in one launch (the
// reference runs n thrust::inner_product calls with a D2H each,
// svmTrain.cu:361-364), f = -y (svmTrain.cu:380) and an int fill.
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// one wave per row, 4 rows per workgroup
__global__ __launch_bounds__(256) void row_sqnorm_kernel(const float* __restrict__ x, int64_t n,
                                                         int d, int ld, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* r = x + row * (int64_t)ld;
  float s = 0.f;
  for (int k = lane; k < d; k += 64) s += r[k] * r[k];
  s = wave_sum(s);
  if (lane == 0) out[row] = s;
}

__global__ void init_f_kernel(const float* __restrict__ y, int64_t off, int64_t nl,
                              float* __restrict__ f) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nl) f[j] = -y[off + j];  // f = -y (svmTrain.cu:380)
}

__global__ void fill_i32_kernel(int32_t* p, int64_t n, int32_t v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

}  // namespace dev

namespace launch {

void row_sqnorm(const float* x, int64_t n, int d, int ld, float* out, hipStream_t s) {
  if (n <= 0) return;
  dev::row_sqnorm_kernel<<<dim3((unsigned)((n + 3) / 4)), 256, 0, s>>>(x, n, d, ld, out);
  post_launch("row_sqnorm", s);
}

void init_f(const float* y, int64_t off, int64_t nl, float* f, hipStream_t s) {
  if (nl <= 0) return;
  dev::init_f_kernel<<<dim3((unsigned)((nl + 255) / 256)), 256, 0, s>>>(y, off, nl, f);
  post_launch("init_f", s);
}

void fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t s) {
  if (n <= 0) return;
  dev::fill_i32_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, s>>>(p, n, v);
  post_launch("fill_i32", s);
}

}  // namespace launch
}  // namespace dpsvm
