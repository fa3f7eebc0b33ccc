// Wave-64 / workgroup reduction helpers for CDNA4 (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dpsvm/common.hpp"

namespace dpsvm {
namespace dev {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl_xor(lo, m, 64);
  hi = __shfl_xor(hi, m, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = shfl_xor_u64(v, m);
    v = o < v ? o : v;
  }
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// |x_h - x_l|^2 over dp floats (multiple of 4, zero padded, 16-B aligned) by
// one wave.  Every kernel that derives eta uses this exact lane mapping and
// summation tree, so all iteration variants agree bit for bit.
__device__ __forceinline__ float wave_dist2(const float* xh, const float* xl, int dp, int lane) {
#pragma clang fp contract(off)
  float part = 0.f;
  for (int k = 4 * lane; k < dp; k += 256) {
    const f4 h = *(const f4*)(xh + k), l = *(const f4*)(xl + k);
    const f4 t = h - l;
    part += (t.x * t.x + t.y * t.y) + (t.z * t.z + t.w * t.w);
  }
  return wave_sum(part);
}

// Block-wide min of two u64 keys; result valid in every thread.
// `scratch` must hold 2*(blockDim/64) u64.
template <int THREADS>
__device__ __forceinline__ void block_min2_u64(uint64_t& a, uint64_t& b, uint64_t* scratch) {
  constexpr int W = THREADS / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a = wave_min_u64(a);
  b = wave_min_u64(b);
  if (lane == 0) {
    scratch[wave] = a;
    scratch[W + wave] = b;
  }
  __syncthreads();
  uint64_t ra = kKeyNone, rb = kKeyNone;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    ra = scratch[w] < ra ? scratch[w] : ra;
    rb = scratch[W + w] < rb ? scratch[W + w] : rb;
  }
  a = ra;
  b = rb;
  __syncthreads();
}

// Deterministic block sum (fixed tree: wave shuffles then waves in order).
template <int THREADS>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  constexpr int W = THREADS / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int w = 0; w < W; ++w) r += scratch[w];
  __syncthreads();
  return r;
}

__device__ __forceinline__ f4 mfma16(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// f_j + c_hi K_hi,j + c_lo K_lo,j (svmTrain.cu:133-135) with every rounding
// explicit: no FMA contraction, so the result does not depend on how the
// surrounding code is if-converted or scheduled.  All engines (chain, fused,
// fused cache, persistent) update f through this one function and therefore
// follow bit-identical SMO trajectories.  A zero coefficient (with a finite K,
// pass 0 for an absent row) contributes an exact zero: no branch on which
// rows are live.
__device__ __forceinline__ float f_apply(float fj, float c_hi, float k_hi, float c_lo, float k_lo) {
#pragma clang fp contract(off)
  const float delta = c_hi * k_hi + c_lo * k_lo;
  return fj + delta;
}

__device__ __forceinline__ float rbf_from_dot(float sq_a, float sq_b, float dot, float gamma) {
#pragma clang fp contract(off)  // same rounding in every row kernel (GEMM, rows, fused X pass)
  float d2 = sq_a + sq_b - 2.0f * dot;  // expansion as svmTrain.cu:128-130
  d2 = d2 > 0.f ? d2 : 0.f;             // clamp
  return expf(-gamma * d2);
}

}  // namespace dev
}  // namespace dpsvm
