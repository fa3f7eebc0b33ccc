// Workgroup helpers of the cache-mode iteration plans (fused and persistent
// cache engines): block-wide exclusive scan and the ballot radix select of the
// speculative rows.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dpsvm/device_state.hpp"

namespace dpsvm {
namespace dev {

// exclusive prefix sum of v over the workgroup (kFusedThreads); *total = sum
__device__ __forceinline__ int block_excl_scan(int v, int* total, int* wsum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kFusedThreads / 64; ++w) {
    before += w < wave ? wsum[w] : 0;
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return before + incl - v;
}

// lanes holding the t smallest of the wave's values among `valid` lanes
// (values unique): MSB-first radix select on ballots, uniform SALU control
__device__ __forceinline__ uint64_t wave_smallest(uint64_t v, int t, uint64_t valid) {
  uint64_t chosen = 0, active = valid;
  int need = t;
  for (int bit = 63; bit >= 0 && need > 0 && active; --bit) {
    const uint64_t zero = __ballot(((v >> bit) & 1ull) == 0ull) & active;
    const int nz = __popcll(zero);
    if (nz <= need) {
      chosen |= zero;
      need -= nz;
      active &= ~zero;
    } else {
      active = zero;
    }
  }
  return chosen;
}

}  // namespace dev
}  // namespace dpsvm
