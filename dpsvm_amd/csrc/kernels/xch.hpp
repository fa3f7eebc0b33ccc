// Peer exchange of per-workgroup selection keys (dense engines, and the
// in-kernel replacement of the per-iteration all-reduce when world > 1).
//
// Each workgroup pushes its (up, low) keys — and the current alphas of the
// two rows behind them — to every rank as four 8-byte granules {16-bit tag,
// 48-bit payload} with relaxed atomic stores (one aligned store per granule:
// never torn; the data IS the flag, no fence): per side, the key's upper 48
// bits, then its lower 16 bits with the 32-bit alpha.  Consumers poll their
// own receive buffer until every granule of the parity carries the expected
// tag, then reduce exactly as from an all-reduced buffer — every rank derives
// the same pair, and the pair's alphas come from their owners' registers, so
// no consumer ever reads a cross-workgroup-written alpha through a possibly
// stale cache line (L2s are per XCD).  Iteration tags T = iteration + 1 are
// sent as (T mod 65535) + 1: never 0 (buffers are zeroed before each solve)
// and never equal for T and T - 2, the only older publication a slot can
// still hold; keys tagged T live in parity T & 1, and no workgroup can lap
// another: its publication T+2 needs every T+1 publication, each made after
// its author had read parity T.
// Scope: system across GPUs (xGMI peer memory), agent within one GPU.
// Reference: one 16-byte MPI Allgather per iteration (svmTrainMain.cpp:244).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"

namespace dpsvm {
namespace dev {

// global (address space 1) pointers: global_ instructions count only in
// vmcnt, so two poll rounds can be in flight (flat ops also count in lgkmcnt
// and make the compiler drain everything before each check)
typedef __attribute__((address_space(1))) uint64_t gu64;

// one workgroup's publication
struct XKeys {
  uint64_t kh, kl;  // up / low selection keys
  float ah, al;     // alphas of the rows behind kh / kl
};

__device__ __forceinline__ uint64_t* xch_entry(uint64_t* base, int par, const SmoArgs& a, int rank, int b) {
  return base + (((int64_t)par * a.xworld + rank) * a.fused_G + b) * a.xstride;
}

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

__device__ __forceinline__ uint32_t fbits(float v) { return __float_as_uint(v); }

// granule tag of iteration tag T (>= 1): 16 bits, never 0, T and T - 2 differ
__device__ __forceinline__ uint64_t xtag(uint32_t T) { return (uint64_t)(T % 65535u + 1u) << 48; }

// keep the smaller key (keys are unique; kKeyNone never wins) with its alpha
__device__ __forceinline__ void xk_min(XKeys& m, const XKeys& o) {
  if (o.kh < m.kh) {
    m.kh = o.kh;
    m.ah = o.ah;
  }
  if (o.kl < m.kl) {
    m.kl = o.kl;
    m.al = o.al;
  }
}

__device__ __forceinline__ XKeys xk_none() { return XKeys{kKeyNone, kKeyNone, 0.f, 0.f}; }

template <int kCtrl>
__device__ __forceinline__ void xk_min_step(XKeys& v) {
  xk_min(v, XKeys{dpp_u64<kCtrl>(v.kh), dpp_u64<kCtrl>(v.kl), dpp_f32<kCtrl>(v.ah), dpp_f32<kCtrl>(v.al)});
}

// full-wave minimum with payloads (DPP row steps + readlane across rows, see
// wave_min_u64); the result is uniform
__device__ __forceinline__ XKeys wave_min_xk(XKeys v) {
  xk_min_step<kDppXor1>(v);
  xk_min_step<kDppXor2>(v);
  xk_min_step<kDppHalfMirror>(v);
  xk_min_step<kDppMirror>(v);
  XKeys r{readlane_u64(v.kh, 0), readlane_u64(v.kl, 0), readlane_f32(v.ah, 0), readlane_f32(v.al, 0)};
#pragma unroll
  for (int row = 1; row < 4; ++row)
    xk_min(r, XKeys{readlane_u64(v.kh, 16 * row), readlane_u64(v.kl, 16 * row), readlane_f32(v.ah, 16 * row),
                    readlane_f32(v.al, 16 * row)});
  return r;
}

// lane p < xworld pushes to rank p; peer = that rank's receive buffer
// (loaded once per launch: a pointer load here would make the compiler wait
// for every earlier store of the wave first)
template <bool kSys>
__device__ __forceinline__ void xch_push_t(const SmoArgs& a, uint64_t* peer, int par, int b, const XKeys& k,
                                           uint32_t tag, int lane) {
  if (lane < a.xworld) {
    uint64_t* g = xch_entry(peer, par, a, a.xrank, b);
    const uint64_t t = xtag(tag);
    xch_store<kSys>(g + 0, t | (k.kh >> 16));
    xch_store<kSys>(g + 1, t | ((k.kh & 0xffffull) << 32) | fbits(k.ah));
    xch_store<kSys>(g + 2, t | (k.kl >> 16));
    xch_store<kSys>(g + 3, t | ((k.kl & 0xffffull) << 32) | fbits(k.al));
  }
}

// lane p < xworld pushes workgroup b's publication to rank p (parity par)
__device__ __forceinline__ void xch_push(const SmoArgs& a, uint64_t* peer, int par, int b, const XKeys& k,
                                         uint32_t tag, int lane) {
  if (a.xworld > 1) xch_push_t<true>(a, peer, par, b, k, tag, lane);
  else xch_push_t<false>(a, peer, par, b, k, tag, lane);
}

__device__ __forceinline__ uint64_t* xch_peer(const SmoArgs& a, int lane) {
  return lane < a.xworld ? a.xpeer[lane] : nullptr;
}

__device__ __forceinline__ bool xg_ready(const uint64_t (&x)[kXchGranules], uint64_t t) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < kXchGranules; ++i) ok &= (x[i] >> 48) == (t >> 48);
  return ok;
}

__device__ __forceinline__ XKeys xg_decode(const uint64_t (&x)[kXchGranules]) {
  constexpr uint64_t m48 = (1ull << 48) - 1;
  XKeys k;
  k.kh = ((x[0] & m48) << 16) | ((x[1] >> 32) & 0xffffull);
  k.ah = __uint_as_float((uint32_t)x[1]);
  k.kl = ((x[2] & m48) << 16) | ((x[3] >> 32) & 0xffffull);
  k.al = __uint_as_float((uint32_t)x[3]);
  return k;
}

// Poll: thread `tid` of `nthreads` watches entries tid, tid + nthreads, ...
// One round = one load of each watched granule; kPipe keeps two rounds in
// flight (the next one issued before the previous is checked: arrivals seen
// half a round trip earlier, at twice the polling traffic — every round of
// every workgroup reads all E entries past the L2).  Returns this thread's
// minimum (the caller reduces); false on give-up.
template <bool kSys, bool kPipe>
__device__ __forceinline__ bool xch_poll_t(const SmoArgs& a, const uint64_t* mine_buf, int par, uint32_t tag,
                                           XKeys& out, int tid, int nthreads) {
  const int E = a.xworld * a.fused_G;
  const uint64_t* base = mine_buf + (int64_t)par * E * a.xstride;
  const uint64_t xt = xtag(tag);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  XKeys m = xk_none();
  for (int c = 0; c < E; c += nthreads) {
    const int e = c + tid;
    const bool mine = e < E;
    const uint64_t* g = base + (int64_t)(mine ? e : 0) * a.xstride;
    uint64_t ra[kXchGranules], rb[kXchGranules];
#pragma unroll
    for (int i = 0; i < kXchGranules; ++i) ra[i] = xch_load<kSys>(g + i);
    bool got_a = false;
    if constexpr (kPipe) {
      while (true) {
#pragma unroll
        for (int i = 0; i < kXchGranules; ++i) rb[i] = xch_load<kSys>(g + i);
        if (__all(!mine || xg_ready(ra, xt))) {
          got_a = true;
          break;
        }
#pragma unroll
        for (int i = 0; i < kXchGranules; ++i) ra[i] = xch_load<kSys>(g + i);
        if (__all(!mine || xg_ready(rb, xt))) break;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) return false;
      }
    } else {
      got_a = true;
      while (!__all(!mine || xg_ready(ra, xt))) {
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) return false;
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int i = 0; i < kXchGranules; ++i) ra[i] = xch_load<kSys>(g + i);
      }
    }
    if (mine) xk_min(m, got_a ? xg_decode(ra) : xg_decode(rb));
  }
  out = m;
  return true;
}

// One wave watches ALL entries (lane l: entries l + 64 i, up to kB per lane
// per batch, every load of a batch in flight together), sleeping between
// rounds: the fewest poll requests on the hot buffer lines (every workgroup
// polls the same few KB, so polling traffic itself delays the publications).
// kB = ceil(E / 64) up to 4, so no load is issued for an absent entry.
template <bool kSys, int kB>
__device__ __forceinline__ bool xch_poll_wave_t(const SmoArgs& a, const uint64_t* mine_buf, int par, uint32_t tag,
                                                XKeys& out, int lane) {
  const int E = a.xworld * a.fused_G;
  const uint64_t* base = mine_buf + (int64_t)par * E * a.xstride;
  const uint64_t xt = xtag(tag);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  XKeys m = xk_none();
  for (int c = 0; c < E; c += 64 * kB) {
    uint64_t r[kB][kXchGranules];
    bool mine[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) mine[j] = c + lane + 64 * j < E;
    while (true) {
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        const uint64_t* g = base + (int64_t)(mine[j] ? c + lane + 64 * j : 0) * a.xstride;
#pragma unroll
        for (int i = 0; i < kXchGranules; ++i) r[j][i] = xch_load<kSys>(g + i);
      }
      bool ok = true;
#pragma unroll
      for (int j = 0; j < kB; ++j) ok &= !mine[j] || xg_ready(r[j], xt);
      if (__all(ok)) break;
      if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) return false;
      for (int z = 0; z < a.xpoll_sleep; ++z) __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < kB; ++j)
      if (mine[j]) xk_min(m, xg_decode(r[j]));
  }
  out = m;
  return true;
}

// mine_buf: this rank's receive buffer (a.xpeer[a.xrank], loaded once)
template <bool kPipe = false>
__device__ __forceinline__ bool xch_poll(const SmoArgs& a, const uint64_t* mine_buf, int par, uint32_t tag,
                                         XKeys& out, int tid, int nthreads) {
  return a.xworld > 1 ? xch_poll_t<true, kPipe>(a, mine_buf, par, tag, out, tid, nthreads)
                      : xch_poll_t<false, kPipe>(a, mine_buf, par, tag, out, tid, nthreads);
}

}  // namespace dev
}  // namespace dpsvm
