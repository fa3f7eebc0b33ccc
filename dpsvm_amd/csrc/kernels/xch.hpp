// Peer exchange of per-workgroup selection keys (dense fused mode, world > 1):
// the in-kernel replacement of the per-iteration all-reduce.
//
// Each workgroup of launch t pushes its (up, low) keys to every rank as four
// 8-byte granules {tag, 32-bit half} with system-scope relaxed stores (one
// aligned store per granule: never torn; the data IS the flag, no fence).
// Launch t+1 on every rank polls its own receive buffer with system-scope
// loads until every granule of the parity carries the expected tag, then
// reduces exactly as from an all-reduced buffer — so every rank derives the
// same pair.  Tags are the iteration count + 1 (never 0; buffers are zeroed
// before each solve); keys tagged T live in parity T & 1, and a rank cannot lap a peer: its
// launch t+2 needs that peer's launch-t+1 keys, which the peer publishes only
// after it has read the parity t+2 overwrites.
// Reference: one 16-byte MPI Allgather per iteration (svmTrainMain.cpp:244).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"

namespace dpsvm {
namespace dev {

__device__ __forceinline__ uint64_t* xch_entry(uint64_t* base, int par, const SmoArgs& a, int rank, int b) {
  return base + (((int64_t)par * a.xworld + rank) * a.fused_G + b) * kXchGranules;
}

// global (address space 1) pointers: global_ instructions count only in
// vmcnt, so two poll rounds can be in flight (flat ops also count in lgkmcnt
// and make the compiler drain everything before each check)
typedef __attribute__((address_space(1))) uint64_t gu64;

// system scope across GPUs (xGMI peer memory), agent scope within one GPU
template <bool kSys>
__device__ __forceinline__ void xch_store(uint64_t* g, uint64_t v) {
  gu64* p = (gu64*)g;
  if constexpr (kSys) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kSys>
__device__ __forceinline__ uint64_t xch_load(const uint64_t* g) {
  gu64* p = (gu64*)g;
  if constexpr (kSys) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kSys>
__device__ __forceinline__ void xch_push_t(const SmoArgs& a, int par, int b, uint64_t kh, uint64_t kl, uint32_t tag,
                                           int lane) {
  if (lane < a.xworld) {
    uint64_t* g = xch_entry(a.xpeer[lane], par, a, a.xrank, b);
    const uint64_t t = (uint64_t)tag << 32;
    xch_store<kSys>(g + 0, t | (kh >> 32));
    xch_store<kSys>(g + 1, t | (kh & 0xffffffffull));
    xch_store<kSys>(g + 2, t | (kl >> 32));
    xch_store<kSys>(g + 3, t | (kl & 0xffffffffull));
  }
}

template <bool kSys>
__device__ __forceinline__ bool xch_pull_t(const SmoArgs& a, int par, uint32_t tag, uint64_t& kh, uint64_t& kl,
                                           int lane) {
  const int E = a.xworld * a.fused_G;
  const uint64_t* base = a.xpeer[a.xrank] + (int64_t)par * E * kXchGranules;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    uint64_t h = kKeyNone, l = kKeyNone;
    bool ok = true;
    for (int e = lane; e < E; e += 64) {
      const uint64_t* g = base + (int64_t)e * kXchGranules;
      const uint64_t g0 = xch_load<kSys>(g), g1 = xch_load<kSys>(g + 1), g2 = xch_load<kSys>(g + 2),
                     g3 = xch_load<kSys>(g + 3);
      ok &= (uint32_t)(g0 >> 32) == tag && (uint32_t)(g1 >> 32) == tag && (uint32_t)(g2 >> 32) == tag &&
            (uint32_t)(g3 >> 32) == tag;
      const uint64_t vh = (g0 << 32) | (g1 & 0xffffffffull), vl = (g2 << 32) | (g3 & 0xffffffffull);
      h = vh < h ? vh : h;
      l = vl < l ? vl : l;
    }
    if (__all(ok)) {
      kh = h;
      kl = l;
      return true;
    }
    if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// Workgroup-parallel poll for the persistent engine: thread `tid` of the
// workgroup watches entries tid, tid + 256, ... and keeps two load rounds in
// flight (the next round is issued before the previous one is checked), so
// an arrival is seen about half a round trip after it lands instead of up to
// a full one.  Returns this thread's minima (the caller reduces); false on
// give-up.
template <bool kSys>
__device__ __forceinline__ bool xch_poll_t(const SmoArgs& a, int par, uint32_t tag, uint64_t& kh, uint64_t& kl,
                                           int tid, int nthreads) {
  const int E = a.xworld * a.fused_G;
  const uint64_t* base = a.xpeer[a.xrank] + (int64_t)par * E * kXchGranules;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t h = kKeyNone, l = kKeyNone;
  for (int c = 0; c < E; c += nthreads) {
    const int e = c + tid;
    const bool mine = e < E;
    const uint64_t* g = base + (int64_t)(mine ? e : 0) * kXchGranules;
    auto ready = [&](uint64_t x0, uint64_t x1, uint64_t x2, uint64_t x3) {
      return !mine || ((uint32_t)(x0 >> 32) == tag && (uint32_t)(x1 >> 32) == tag && (uint32_t)(x2 >> 32) == tag &&
                       (uint32_t)(x3 >> 32) == tag);
    };
    uint64_t a0 = xch_load<kSys>(g), a1 = xch_load<kSys>(g + 1), a2 = xch_load<kSys>(g + 2),
             a3 = xch_load<kSys>(g + 3);
    uint64_t r0, r1, r2, r3;
    while (true) {
      const uint64_t b0 = xch_load<kSys>(g), b1 = xch_load<kSys>(g + 1), b2 = xch_load<kSys>(g + 2),
                     b3 = xch_load<kSys>(g + 3);
      if (__all(ready(a0, a1, a2, a3))) {
        r0 = a0; r1 = a1; r2 = a2; r3 = a3;
        break;
      }
      a0 = xch_load<kSys>(g);
      a1 = xch_load<kSys>(g + 1);
      a2 = xch_load<kSys>(g + 2);
      a3 = xch_load<kSys>(g + 3);
      if (__all(ready(b0, b1, b2, b3))) {
        r0 = b0; r1 = b1; r2 = b2; r3 = b3;
        break;
      }
      if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) return false;
    }
    if (mine) {
      const uint64_t vh = (r0 << 32) | (r1 & 0xffffffffull), vl = (r2 << 32) | (r3 & 0xffffffffull);
      h = vh < h ? vh : h;
      l = vl < l ? vl : l;
    }
  }
  kh = h;
  kl = l;
  return true;
}

__device__ __forceinline__ bool xch_poll(const SmoArgs& a, int par, uint32_t tag, uint64_t& kh, uint64_t& kl, int tid,
                                         int nthreads) {
  return a.xworld > 1 ? xch_poll_t<true>(a, par, tag, kh, kl, tid, nthreads)
                      : xch_poll_t<false>(a, par, tag, kh, kl, tid, nthreads);
}

// lane p < xworld pushes workgroup b's keys to rank p (parity par)
__device__ __forceinline__ void xch_push(const SmoArgs& a, int par, int b, uint64_t kh, uint64_t kl, uint32_t tag,
                                         int lane) {
  if (a.xworld > 1) xch_push_t<true>(a, par, b, kh, kl, tag, lane);
  else xch_push_t<false>(a, par, b, kh, kl, tag, lane);
}

// every lane of the calling wave: min keys over ITS entries (lane, lane + 64,
// ...) of all ranks' workgroups of parity par, polling until every granule
// carries `tag` (the caller reduces across the wave); false on give-up
__device__ __forceinline__ bool xch_pull(const SmoArgs& a, int par, uint32_t tag, uint64_t& kh, uint64_t& kl,
                                         int lane) {
  return a.xworld > 1 ? xch_pull_t<true>(a, par, tag, kh, kl, lane) : xch_pull_t<false>(a, par, tag, kh, kl, lane);
}

}  // namespace dev
}  // namespace dpsvm
