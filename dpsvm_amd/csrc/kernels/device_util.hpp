// Wave-64 / workgroup reduction helpers for CDNA4 (gfx950).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dpsvm/common.hpp"

namespace dpsvm {
namespace dev {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

// ---- full-wave reductions on DPP (no LDS round trips) ----
// Within each 16-lane row: quad_perm xor 1, quad_perm xor 2, row_half_mirror
// (i <-> 7-i) and row_mirror (i <-> 15-i) leave every lane of the row holding
// the row's reduction (each step pairs lanes that already agree, so the
// operands are identical on both sides); the four rows are then combined from
// lanes 0/16/32/48 through v_readlane (uniform operands).  A ds_bpermute
// butterfly costs an LDS round trip per step; these steps are plain VALU ops.
// All 64 lanes must be active (every call site reduces full waves).
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;
constexpr int kDppMirror = 0x140;

template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}
template <int kCtrl>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xF, 0xF, false));
}
template <int kCtrl>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint64_t lo = dpp_u32<kCtrl>((uint32_t)v), hi = dpp_u32<kCtrl>((uint32_t)(v >> 32));
  return (hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return (hi << 32) | lo;
}
__device__ __forceinline__ float readlane_f32(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <int kCtrl>
__device__ __forceinline__ uint64_t min_step_u64(uint64_t v) {
  const uint64_t o = dpp_u64<kCtrl>(v);
  return o < v ? o : v;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  v = min_step_u64<kDppXor1>(v);
  v = min_step_u64<kDppXor2>(v);
  v = min_step_u64<kDppHalfMirror>(v);
  v = min_step_u64<kDppMirror>(v);
  uint64_t r = readlane_u64(v, 0);
#pragma unroll
  for (int row = 1; row < 4; ++row) {
    const uint64_t o = readlane_u64(v, 16 * row);
    r = o < r ? o : r;
  }
  return r;
}

// Deterministic wave sum: the same tree (and the same bits) in every lane.
__device__ __forceinline__ float wave_sum(float v) {
#pragma clang fp contract(off)
  v = v + dpp_f32<kDppXor1>(v);
  v = v + dpp_f32<kDppXor2>(v);
  v = v + dpp_f32<kDppHalfMirror>(v);
  v = v + dpp_f32<kDppMirror>(v);
  return (readlane_f32(v, 0) + readlane_f32(v, 16)) + (readlane_f32(v, 32) + readlane_f32(v, 48));
}

// |x_h - x_l|^2 over dp floats (multiple of 4, zero padded, 16-B aligned) by
// one wave.  Every kernel that derives eta uses this exact lane mapping and
// summation tree, so all iteration variants agree bit for bit.
__device__ __forceinline__ float dist2_term(f4 h, f4 l) {
#pragma clang fp contract(off)
  const f4 t = h - l;
  return (t.x * t.x + t.y * t.y) + (t.z * t.z + t.w * t.w);
}

__device__ __forceinline__ float wave_dist2(const float* xh, const float* xl, int dp, int lane) {
#pragma clang fp contract(off)
  float part = 0.f;
  if (dp <= 1024) {
    // d <= 1024 (every BASELINE config): all eight 16-B loads of the lane are
    // issued before the first use — one memory round trip instead of one per
    // 256-column step (the loop below waits for each step's loads).  Same
    // per-lane summation order as the loop, so both forms agree bit for bit.
    f4 h[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 4 * lane + 256 * i;
      const int kk = k < dp ? k : 0;  // in-bounds address for idle slots
      h[i] = *(const f4*)(xh + kk);
      l[i] = *(const f4*)(xl + kk);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float s = dist2_term(h[i], l[i]);
      part = 4 * lane + 256 * i < dp ? part + s : part;
    }
  } else {
    for (int k = 4 * lane; k < dp; k += 256) part += dist2_term(*(const f4*)(xh + k), *(const f4*)(xl + k));
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

// Residency census of a persistent grid (run once at setup with the engine's
// own kernel, grid and resources, before that engine is chosen).  Thread 0 of
// every workgroup counts itself in and waits until the whole grid has arrived.
// A grid that cannot be co-resident (a partitioned device, CUs held by another
// job, an oversized grid) times out instead of hanging: the first workgroup to
// give up raises the abort word, and workgroups that only get a CU after
// others left see it and leave at once without counting themselves.  All
// accesses are memory-side atomics (never a stale line of a per-XCD L2).
// words: [arrivals, abort], zeroed by the host; success = {gridDim.x, 0}.
__device__ inline void census_arrive(int32_t* words, int64_t ticks) {
  if (threadIdx.x != 0) return;
  auto rd = [&](int i) { return __hip_atomic_fetch_add(words + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  if (rd(1) != 0) return;
  __hip_atomic_fetch_add(words, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (rd(0) < (int)gridDim.x && rd(1) == 0) {
    if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > ticks) {
      __hip_atomic_fetch_add(words + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

}  // namespace dev
}  // namespace dpsvm
