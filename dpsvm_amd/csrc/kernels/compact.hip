// Support-vector compaction and gathering (replaces the reference's
// thrust::remove_if over a 4-zip + host-side row gather, svmTrain.cu:595-631,
// K11): ballot/popcount per wave, one-workgroup scan, ordered scatter.
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// ---------------------------------------------------------------------------
// SV compaction (K11 replacement: thrust::remove_if over a 4-zip)
// ---------------------------------------------------------------------------
constexpr int kCompactBlock = 1024;

__global__ __launch_bounds__(kCompactBlock) void compact_count_kernel(const float* alpha, int64_t n,
                                                                      int32_t* counts) {
  __shared__ int32_t wc[kCompactBlock / 64];
  const int64_t i = (int64_t)blockIdx.x * kCompactBlock + threadIdx.x;
  const bool p = i < n && alpha[i] > 0.f;
  const uint64_t m = __ballot(p);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t s = 0;
    for (int w = 0; w < kCompactBlock / 64; ++w) s += wc[w];
    counts[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(1024) void compact_scan_kernel(int32_t* counts, int nb, int32_t* total) {
  // single workgroup exclusive scan (sequential chunks per thread + LDS scan)
  __shared__ int32_t part[1024];
  const int per = (nb + 1023) / 1024;
  const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
  int32_t s = 0;
  for (int b = b0; b < b1; ++b) s += counts[b];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t run = 0;
    for (int t = 0; t < 1024; ++t) {
      int32_t v = part[t];
      part[t] = run;
      run += v;
    }
    *total = run;
  }
  __syncthreads();
  int32_t run = part[threadIdx.x];
  for (int b = b0; b < b1; ++b) {
    int32_t v = counts[b];
    counts[b] = run;
    run += v;
  }
}

__global__ __launch_bounds__(kCompactBlock) void compact_scatter_kernel(const float* alpha, int64_t n,
                                                                        const int32_t* offsets,
                                                                        int32_t* idx_out) {
  __shared__ int32_t wc[kCompactBlock / 64];
  const int64_t i = (int64_t)blockIdx.x * kCompactBlock + threadIdx.x;
  const bool p = i < n && alpha[i] > 0.f;
  const uint64_t m = __ballot(p);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) wc[wave] = __popcll(m);
  __syncthreads();
  int32_t base = offsets[blockIdx.x];
  for (int w = 0; w < wave; ++w) base += wc[w];
  const int32_t rank = __popcll(m & ((1ull << lane) - 1ull));
  if (p) idx_out[base + rank] = (int32_t)i;
}

__global__ void gather_sv_kernel(const float* x, int64_t x_row0, const float* xsq, const float* alpha,
                                 const float* y, const int32_t* idx, int64_t nsv, int dp, float* sv,
                                 float* svsq, float* coef) {
  const int64_t r = blockIdx.x;
  if (r >= nsv) return;
  const int64_t g = idx[r];
  const float* src = x + (g - x_row0) * dp;
  for (int k = threadIdx.x; k < dp; k += blockDim.x) sv[r * dp + k] = src[k];
  if (threadIdx.x == 0) {
    svsq[r] = xsq[g];
    coef[r] = alpha[g] * y[g];
  }
}

}  // namespace dev

namespace launch {

int64_t compact_scratch_ints(int64_t n) { return (n + dev::kCompactBlock - 1) / dev::kCompactBlock + 1; }

void compact_positive(const float* alpha, int64_t n, int32_t* idx_out, int32_t* count_dev,
                      int32_t* scratch, hipStream_t s) {
  const int nb = (int)((n + dev::kCompactBlock - 1) / dev::kCompactBlock);
  dev::compact_count_kernel<<<dim3(nb), dev::kCompactBlock, 0, s>>>(alpha, n, scratch);
  post_launch("compact_count", s);
  dev::compact_scan_kernel<<<dim3(1), 1024, 0, s>>>(scratch, nb, count_dev);
  post_launch("compact_scan", s);
  dev::compact_scatter_kernel<<<dim3(nb), dev::kCompactBlock, 0, s>>>(alpha, n, scratch, idx_out);
  post_launch("compact_scatter", s);
}

void gather_sv(const float* x, int64_t x_row0, const float* xsq, const float* alpha,
               const float* y, const int32_t* idx, int64_t nsv, int dp, float* sv, float* svsq,
               float* coef, hipStream_t s) {
  if (nsv <= 0) return;
  dev::gather_sv_kernel<<<dim3((unsigned)nsv), 256, 0, s>>>(x, x_row0, xsq, alpha, y, idx, nsv, dp,
                                                           sv, svsq, coef);
  post_launch("gather_sv", s);
}

}  // namespace launch
}  // namespace dpsvm
