// Working-set engine (smo_ws): device helpers shared by its translation units
// ws_select.hip (f update + candidates), ws_merge.hip (merge, sub-Gram gather,
// multi-block union) and ws_solve.hip (the LDS sub-problem).  One round (Gram
// resident, one block) = three launches:
//
//   ws_gather  (q_max workgroups of 256 threads)
//       every workgroup merges the candidate lists redundantly (identical
//       inputs, identical arithmetic: no grid synchronisation needed): the
//       global stop test — the reference's !(b_lo > b_hi + 2 eps)
//       (svmTrainMain.cpp:310) on the exact f — then per side a 16-bit key
//       prefix threshold from two radix-histogram passes (no sort), and the
//       new working set: the most violating rows alternately from I_up /
//       I_low (the global extremes first), duplicates removed through LDS
//       hash tables, then the newest rows of the previous set.  Workgroup a then
//       gathers row a of the q x q sub-Gram from the resident Gram (q random
//       columns of one row: one load per thread — the whole grid does the
//       scattered reads a single CU could not issue fast enough);
//   ws_solve   (ONE workgroup; the sub-problem runs on wave 0 alone)
//       sub-Gram -> LDS, then the reference's pair rule (selection
//       svmTrainMain.cpp:255-277, update :282-299 through the same
//       pair_update as every engine) on the q rows: per step two DPP wave
//       minima (row_bcast reductions), ballots for the lowest position, seven
//       LDS reads and a register update of f / alpha — no barrier, no global
//       memory, ~150 instructions of one wave;
//   ws_select  (grid over the local rows, 256-thread workgroups)
//       f_j += sum_k coef_k K(idx_k, j) for the round's alpha changes (a
//       stream over the changed Gram rows), I_up / I_low classification and
//       each workgroup's kWsCand smallest keys per side.
//
// The reference spends one MPI Allgather and >= 7 host round trips per pair
// (svmTrainMain.cpp:235-310); the persistent SMO engine one grid-wide key
// exchange (~4.3 us).  Here a pair step costs ~0.3 us of one wave and the
// grid-wide work happens once per round of ~50 pair steps.
#pragma once

#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "xch.hpp"

namespace dpsvm {
namespace dev {

constexpr int kWsGatherThreads = 256;
constexpr int kWsMaxCand = kWsMaxGroups * kWsCand1;  // per side, one-block merge
constexpr int kWsHash = 1024;                        // LDS hash slots per side (load factor <= 0.19)

// Phase stamps (DPSVM_STAMPS), ring slot = round: ws_gather workgroup 0
// [1] entry [2] merged [8] exit; ws_solve [0] entry [3] sub-Gram loaded
// [4] solved [5] pair steps; ws_select workgroup 0 [6] entry [7] exit.
#define WS_STAMP(k)                                                                            \
  do {                                                                                         \
    if (a.stamps) a.stamps[(size_t)(c->outer % kStampRing) * 2 * kStampSlots + (k)] =          \
        __builtin_amdgcn_s_memrealtime();                                                      \
  } while (0)

__device__ __forceinline__ float f_add1(float fj, float c, float k) {
#pragma clang fp contract(off)
  return fj + c * k;
}

// full-wave minima of two floats: v_min_f32 with DPP operands (in-row
// butterflies, then row_bcast15 / row_bcast31 fold the rows into lane 63,
// GFX9 DPP), the two chains interleaved so each fills the other's DPP read-
// after-write wait states; one readlane each.  (The intrinsic path emits a
// separate dpp move plus an IEEE canonicalize per step: 2.5x the issue slots.)
__device__ __forceinline__ void wave_min2_f32(float& a, float& b) {
  asm volatile(
      "s_nop 1\n"
      "v_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_min_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "s_nop 0\n"
      "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_min_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "s_nop 0\n"
      "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_min_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "s_nop 0\n"
      "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n"
      "v_min_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf\n"
      "s_nop 0\n"
      "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
      "v_min_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
      "s_nop 0\n"
      "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
      "v_min_f32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
      "s_nop 1\n"
      : "+v"(a), "+v"(b));
  a = readlane_f32(a, 63);
  b = readlane_f32(b, 63);
}

// exclusive prefix of small counts (0..15) over a 256-thread block in thread
// order, via bit-plane ballots; *total = block sum.  wsum: 4 ints.
__device__ __forceinline__ int block_scan_small256(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  int pre = 0, wtot = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const uint64_t m = __ballot((v >> b) & 1);
    pre += __popcll(m & below) << b;
    wtot += __popcll(m) << b;
  }
  if (lane == 0) wsum[wave] = wtot;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWsGatherThreads / 64; ++w) {
    off += w < wave ? wsum[w] : 0;
    tot += wsum[w];
  }
  *total = tot;
  __syncthreads();
  return off + pre;
}

// first bin b of a 256-bin histogram (one wave: 4 bins per lane) whose
// inclusive prefix reaches `target`; *below = count in bins < b.  -1 when the
// histogram holds fewer than target.  Uniform result.
__device__ __forceinline__ int wave_find_bin(const int* hist, int target, int* below) {
  const int lane = threadIdx.x & 63;
  const int h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
  const int s4 = h0 + h1 + h2 + h3;
  int incl = s4;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o);
    incl += lane >= o ? t : 0;
  }
  const uint64_t hit = __ballot(incl >= target);
  if (!hit) {
    *below = __shfl(incl, 63);
    return -1;
  }
  const int L = (int)__builtin_ctzll(hit);
  int acc = __shfl(incl - s4, L);
  const int g0 = __shfl(h0, L), g1 = __shfl(h1, L), g2 = __shfl(h2, L);
  int bin = 4 * L;
  if (acc + g0 < target) {
    acc += g0;
    ++bin;
    if (acc + g1 < target) {
      acc += g1;
      ++bin;
      if (acc + g2 < target) {
        acc += g2;
        ++bin;
      }
    }
  }
  *below = acc;
  return bin;
}

// exclusive prefix over a 256-thread block (thread order) of four packed
// 12-bit fields (each per-thread value <= 7): bit-plane ballots of the three
// low bits of every field; *total = block sums.  wsum: 4 u64.
__device__ __forceinline__ uint64_t block_scan_fields(uint64_t v, uint64_t* wsum, uint64_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  uint64_t pre = 0, wtot = 0;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int bit = 12 * f + b;
      const uint64_t mk = __ballot((v >> bit) & 1);
      pre += (uint64_t)__popcll(mk & below) << bit;
      wtot += (uint64_t)__popcll(mk) << bit;
    }
  }
  if (lane == 0) wsum[wave] = wtot;
  __syncthreads();
  uint64_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWsGatherThreads / 64; ++w) {
    off += w < wave ? wsum[w] : 0;
    tot += wsum[w];
  }
  *total = tot;
  __syncthreads();
  return off + pre;
}

__device__ __forceinline__ uint32_t ws_hash(int32_t idx) { return ((uint32_t)idx * 2654435761u) >> 22; }

__device__ __forceinline__ void ws_hash_insert(int32_t* keys, int32_t* vals, int32_t idx, int32_t v) {
  uint32_t h = ws_hash(idx);
  while (true) {
    const int32_t old = atomicCAS(keys + h, -1, idx);
    if (old == -1) {
      vals[h] = v;
      return;
    }
    h = (h + 1) & (kWsHash - 1);
  }
}

__device__ __forceinline__ int32_t ws_hash_find(const int32_t* keys, const int32_t* vals, int32_t idx) {
  uint32_t h = ws_hash(idx);
  for (int probe = 0; probe < kWsHash; ++probe) {
    const int32_t k = keys[h];
    if (k == idx) return vals[h];
    if (k == -1) return -1;
    h = (h + 1) & (kWsHash - 1);
  }
  return -1;
}

__device__ __forceinline__ void ws_status(SmoStatus* s, const WsCtrl* c) {
  if (!s) return;
  s->iter = c->iter;
  s->done = c->done;
  s->b_hi = c->b_hi;
  s->b_lo = c->b_lo;
  s->outer = c->outer;
  s->rows_computed = c->rows_computed;  // cache mode: kernel rows computed, member rows found cached
  s->misses = c->rows_computed;
  s->hits = c->row_hits;
  s->ws_p1_round = c->p1_round;
  s->ws_p = c->p_act;
  s->ws_damped = c->n_damped;
  __atomic_store_n(&s->seq, (int32_t)c->outer, __ATOMIC_RELEASE);
}

// ---------------------------------------------------------------------------
// Peer exchange of the rounds (world > 1 with a.xpeer: replaces the candidate
// all-gather and the sub-Gram sum all-reduce, so a round has no collective
// launch and no host step).  Round R = c->outer uses parity R & 1 and granule
// tag xtag(R + 1) (xch.hpp: 16-bit tag << 48 | 48-bit payload, one aligned
// 8-byte system-scope store — never torn, the data is the flag).  Producers:
// each ws_select workgroup stores its 2 x kWsCand1 keys (two granules each: bits
// 63..16, 15..0) into slot rank * G + b of EVERY rank's buffer; gather workgroup
// a stores the sub-Gram entries (a, b) of the columns b its rank owns, and the
// row's f when it owns row a, into row a of every rank's buffer.  Consumers
// poll their own buffer: every merge workgroup the G_all candidate slots,
// gather workgroup a its row a.  Every entry has exactly one producer, so the
// assembled values are the owners' bits (== the sum all-reduce's x + 0 + ...).
// A parity-(R & 1) slot is rewritten (round R + 2) only after every rank
// finished round R + 1's merge, which on each rank follows its round-R reads in
// stream order: no slot is lapped.  Buffers are zeroed before each solve (a tag
// is never 0).  A poll gives up after a.xtimeout_ticks: the run then ends with
// kCommFail on this rank, and its peers time out the same way.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t ws_xcand(const WsArgs& a, int par, int slot) {
  return ((int64_t)par * a.G_all + slot) * a.xcw;
}

__device__ __forceinline__ int64_t ws_xrow(const WsArgs& a, int par, int row) {
  return a.xsub + ((int64_t)par * a.xsub_rows + row) * (a.q_max + 1);
}

// multi-block rounds: the line-search partial slots of every rank, world x
// p1G groups x ks slices; slot k = (rank p1G + group) ks + slice
__device__ __forceinline__ int64_t ws_nparts(const WsArgs& a) {
  return (int64_t)a.world * a.p1G * max(1, a.ks);
}
__device__ __forceinline__ int64_t ws_xpart(const WsArgs& a, int par, int64_t k) {
  return a.xpart + ((int64_t)par * ws_nparts(a) + k) * 4;
}

__device__ __forceinline__ bool ws_tag_ok(uint64_t g, uint64_t t) { return (g >> 48) == (t >> 48); }

// a 64-bit payload as two granules (bits 63..16, bits 15..0) and back
__device__ __forceinline__ void ws_put64(uint64_t* dst, uint64_t t, uint64_t v) {
  xch_store<true>(dst, t | (v >> 16));
  xch_store<true>(dst + 1, t | (v & 0xffffull));
}
__device__ __forceinline__ uint64_t ws_get64(uint64_t g0, uint64_t g1) {
  return ((g0 & ((1ull << 48) - 1)) << 16) | (g1 & 0xffffull);
}

// poll n consecutive granules of this rank's buffer until all carry tag t;
// false after a.xtimeout_ticks (the caller fails the round)
template <int N>
__device__ __forceinline__ bool ws_poll(const WsArgs& a, const uint64_t* g, uint64_t t, uint64_t (&out)[N]) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = xch_load<true>(g + i);
    bool all = true;
#pragma unroll
    for (int i = 0; i < N; ++i) all &= ws_tag_ok(out[i], t);
    if (all) return true;
    if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// a <- the kWsCand1 smallest of the two ascending lists a, b (unique keys):
// min(a[i], b[3 - i]) is a bitonic sequence of the 4 smallest, two
// compare-exchange stages sort it
__device__ __forceinline__ void ws_cx(uint64_t& x, uint64_t& y) {
  const uint64_t lo = x < y ? x : y, hi = x < y ? y : x;
  x = lo;
  y = hi;
}

__device__ __forceinline__ void ws_top4_merge(uint64_t (&a)[kWsCand1], const uint64_t (&b)[kWsCand1]) {
  static_assert(kWsCand1 == 4, "4-entry bitonic merge");
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = a[i] < b[3 - i] ? a[i] : b[3 - i];
  ws_cx(a[0], a[2]);
  ws_cx(a[1], a[3]);
  ws_cx(a[0], a[1]);
  ws_cx(a[2], a[3]);
}

// a poll gave up: the run stops here (any workgroup may call it; same values)
__device__ __forceinline__ void ws_comm_fail(const WsArgs& a, WsCtrl* c) {
  if (threadIdx.x == 0) {
    c->done = kCommFail;
    c->n_apply = 0;  // nothing of this round is applied
    ws_status(a.status, c);
  }
}

// the same from any single thread (no threadIdx condition)
__device__ __forceinline__ void ws_comm_fail_thread(const WsArgs& a, WsCtrl* c) {
  c->done = kCommFail;
  c->n_apply = 0;
  ws_status(a.status, c);
}

// fixed-order wave sum (xor butterfly: every lane ends with the same bits)
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// multi-block rounds: the line search along the combined step d of the round's
// P sub-problems.  W(alpha + t d) = W + t g'd - t^2 d'Qd / 2 peaks at
// t* = g'd / d'Qd, and W(alpha + d) - W(alpha) = d'Qd (t* - 1/2).  The step
// taken is
//   t = 1       P = 1 (one block: its own sub-problem step, exactly the
//               one-block engine's round), or t* >= kWsTFull — the full step
//               keeps >= 99% of the optimal gain, and keeps every alpha the
//               blocks put on a bound exactly there (a factor a hair below 1
//               would leave alpha_new - (1 - t) d_alpha a hair inside the box:
//               a row every later round selects for a zero-length step — the
//               diagnosed cause of the ~3.5-pair-step rounds of round 2);
//   t = t*      kWsTFull > t* (strongly coupled blocks: damped, ascent);
//   t = 0       g'd <= 0: no ascent along d (float cancellation, or an
//               independent-clip round whose steps do not follow W) — the round
//               is discarded and the next one runs with fewer blocks.
// Every wave reduces the workgroup partials in the same order: identical t
// everywhere (and on every rank).
constexpr float kWsTFull = 0.9f;

__device__ __forceinline__ float ws_line_search(const WsArgs& a, int P) {
  if (P <= 1) return 1.f;
  const int lane = threadIdx.x & 63;
  double q = 0.0, g = 0.0;
  for (int k = lane; k < ws_nparts(a); k += 64) {  // every rank's partials (all-gathered / collected)
    q += a.part[2 * k];
    g += a.part[2 * k + 1];
  }
  q = wave_sum_f64(q);
  g = wave_sum_f64(g);
  if (!(g > 0.0)) return 0.f;
  if (!(q > g)) return 1.f;
  const float t = (float)(g / q);
  return t >= kWsTFull ? 1.f : t;
}

}  // namespace dev
}  // namespace dpsvm
