// Working-set engine (Gram resident).  One round = three launches:
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
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "xch.hpp"
#include "../runtime/hip_check.hpp"

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
  return ((int64_t)par * a.G_all + slot) * (4 * kWsCand1);
}

__device__ __forceinline__ int64_t ws_xrow(const WsArgs& a, int par, int row) {
  return a.xsub + ((int64_t)par * a.q_max + row) * (a.q_max + 1);
}

__device__ __forceinline__ bool ws_tag_ok(uint64_t g, uint64_t t) { return (g >> 48) == (t >> 48); }

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
  for (int k = lane; k < a.G_all * max(1, a.ks); k += 64) {  // every rank's partials (all-gathered)
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

// ---------------------------------------------------------------------------
// ws_select: f update of the last round + per-workgroup candidates
// ---------------------------------------------------------------------------
// Threads of a workgroup: 256 rows (x RPT) times PARTS partitions of the
// changed-row list.  Each partition sums its contiguous slice of the list in
// list order; the slices combine in partition order — the rounding depends on
// the list only (never on the grid or the rank count), and every thread has at
// most ~48 Gram loads of one batch in flight instead of a chain of batches.
template <int RPT>
constexpr int ws_parts() {
  // register budget: <= 4 waves per SIMD at RPT <= 4, 2 up to 16, 1 at 32 (2M rows on one GPU)
  return RPT <= 4 ? 4 : RPT <= 16 ? 2 : 1;
}

// MODE 0: one pass (f += the round's change, then candidates).  Multi-block
// rounds split it: MODE 1 computes the change d_f into a.dfs and per-workgroup
// partial sums of the line search (d'Qd = sum_j c_j d_f_j and g'd = -sum_j c_j
// f_j over the changed rows j, c_j = d_alpha_j y_j), MODE 2 takes
// t = min(1, g'd / d'Qd) from the partials (fixed order: every workgroup the
// same t), applies f += t d_f and alpha = alpha_new - (1 - t) d_alpha, then
// selects the candidates.  Pass 2 walks no list: one partition, 256 threads.
template <int RPT, int MODE>
constexpr int ws_sel_parts() {
  return MODE == 2 ? 1 : ws_parts<RPT>();
}

template <int RPT, int MODE>
__global__ __launch_bounds__((kWsSelThreads * ws_sel_parts<RPT, MODE>())) void ws_select_kernel(WsArgs a) {
  constexpr int PARTS = ws_sel_parts<RPT, MODE>();
  constexpr int CH = RPT >= 32 ? 1 : RPT >= 8 ? 4 : 48 / RPT;  // Gram loads in flight per thread (vmcnt <= 63)
  constexpr int LMAX = MODE == 1 ? kWsMaxAll : MODE == 0 ? kWsMax : 1;
  __shared__ int32_t s_idx[LMAX];  // lines of the changed rows
  __shared__ float s_coef[LMAX];
  __shared__ double s_red[2][kWsSelThreads * PARTS / 64];
  __shared__ float s_part[PARTS > 1 ? PARTS - 1 : 1][PARTS > 1 ? kWsSelThreads * RPT : 1];
  __shared__ uint64_t s_wc[kWsSelThreads / 64][2][kWsCand];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x & (kWsSelThreads - 1), part = threadIdx.x / kWsSelThreads;
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(MODE == 1 ? 22 : 6);  // pass 1: own slots (22, 23)
  const int na = c->n_apply;
  const int done = c->done;
  if (na == 0 && (done != kRunning || MODE == 1)) return;
  if constexpr (MODE == 0) {
    for (int k = threadIdx.x; k < na; k += kWsSelThreads * PARTS) {
      s_idx[k] = c->apply_line[k];
      s_coef[k] = c->apply_coef[k];
    }
  }
  // a workgroup owns a.rpt x 256 rows (ws_geometry); RPT (>= a.rpt) only sizes the registers.
  // MODE 1 runs KS = a.ks workgroups per row group, each over its KS-th of the
  // changed-row list (pass 1 fills the device when G is small: 30 groups per rank at
  // 8 ranks on the headline); pass 2 sums the KS partial changes in slice order.
  const int KS = MODE == 1 ? max(1, a.ks) : 1;
  const int grp = MODE == 1 ? (int)(blockIdx.x % a.G) : (int)blockIdx.x, ksi = MODE == 1 ? (int)(blockIdx.x / a.G) : 0;
  if constexpr (MODE == 1) {
    // the blocks' apply segments, concatenated in block order; this workgroup
    // loads only its slice [e_lo, e_hi) of the list (at their list positions)
    const int per_wg = PARTS * ((na + PARTS * KS - 1) / (PARTS * KS));
    const int e_lo = min(na, ksi * per_wg), e_hi = min(na, e_lo + per_wg);
    int at = 0;
    for (int p = 0; p < a.blocks && at < e_hi; ++p) {
      const int nb = c->nab[p];
      const int k0 = max(0, e_lo - at), k1 = min(nb, e_hi - at);
      for (int k = k0 + threadIdx.x; k < k1; k += kWsSelThreads * PARTS) {
        s_idx[at + k] = c->apply_line[p * a.q_max + k];
        s_coef[at + k] = c->apply_coef[p * a.q_max + k];
      }
      at += nb;
    }
  }
  __syncthreads();
  const int64_t base = (int64_t)grp * a.rpt * kWsSelThreads + tid;
  float f[RPT];
  bool has[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int64_t j = base + (int64_t)r * kWsSelThreads;
    has[r] = r < a.rpt && j < a.nl;
    f[r] = has[r] && part == 0 ? a.f[j] : 0.f;
  }
  if (na > 0) {
    float acc[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) acc[r] = 0.f;
    if constexpr (MODE != 2) {
    const int per = (na + PARTS * KS - 1) / (PARTS * KS);
    const int k_lo = min(na, (ksi * PARTS + part) * per), k_hi = min(na, k_lo + per);
    for (int k0 = k_lo; k0 < k_hi; k0 += CH) {
      float kv[CH][RPT];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int kk = min(k0 + u, k_hi - 1);
        const float* row = a.gram + (int64_t)s_idx[kk] * a.ldg;
#pragma unroll
        for (int r = 0; r < RPT; ++r) kv[u][r] = has[r] ? row[base + r * kWsSelThreads] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        if (k0 + u < k_hi) {
          const float cc = s_coef[k0 + u];
#pragma unroll
          for (int r = 0; r < RPT; ++r) acc[r] = f_add1(acc[r], cc, kv[u][r]);
        }
      }
    }
    if (PARTS > 1) {
      if (part > 0) {
#pragma unroll
        for (int r = 0; r < RPT; ++r) s_part[part - 1][r * kWsSelThreads + tid] = acc[r];
      }
      __syncthreads();
#pragma unroll
      for (int p = 1; p < PARTS; ++p) {
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
#pragma clang fp contract(off)
          acc[r] = acc[r] + s_part[p - 1][r * kWsSelThreads + tid];
        }
      }
    }
    }  // MODE != 2
    if constexpr (MODE == 1) {
      double sq = 0.0, sg = 0.0;
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        if (has[r] && part == 0) {
          const int64_t j = base + r * kWsSelThreads;
          a.dfs[(int64_t)ksi * a.nl + j] = acc[r];
          const float dj = a.dalpha[a.off + j];
          if (dj != 0.f) {
            const double cj = (double)dj * (double)a.y[a.off + j];
            sq += cj * (double)acc[r];  // d'Qd is linear in the KS partial changes
            if (ksi == 0) sg -= cj * (double)f[r];
          }
        }
      }
      // fixed-order block sums (butterfly per wave, waves in order)
      sq = wave_sum_f64(sq);
      sg = wave_sum_f64(sg);
      const int w = threadIdx.x >> 6;
      if ((threadIdx.x & 63) == 0) {
        s_red[0][w] = sq;
        s_red[1][w] = sg;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        double tq = 0.0, tg = 0.0;
        for (int k = 0; k < kWsSelThreads * PARTS / 64; ++k) {
          tq += s_red[0][k];
          tg += s_red[1][k];
        }
        const int64_t slot = ((int64_t)a.rank * a.G + grp) * KS + ksi;
        a.part[2 * slot] = tq;
        a.part[2 * slot + 1] = tg;
        if (blockIdx.x == 0) WS_STAMP(23);
      }
      return;
    }
    if constexpr (MODE == 2) {
      const int pr = c->p_round;  // written by this round's merge (p_act may change below)
      const float t = ws_line_search(a, pr);
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->t_last = t;
        if (t < 1.f) {
          // strongly coupled blocks: fewer from the next round on (the solve's
          // commit may have set p_act = 1 already: an independent-clip event)
          c->n_damped = c->n_damped + 1;
          const int np = t < a.t_halve ? max(1, pr / 2) : pr;
          if (np < c->p_act) c->p_act = np;
          if (c->p_act == 1 && c->p1_round == 0) c->p1_round = c->outer;
          ws_status(a.status, c);  // p1_round visible with the round that set it (gpu_engines.hip)
        }
      }
      if (a.world > 1 && blockIdx.x == 0) {
        // alpha is global on every rank: the changed rows this rank does not own
        // (its threads below fix the owned ones before classifying them)
        for (int p = 0; p < a.blocks; ++p) {
          const int nb = c->nab[p];
          for (int k = threadIdx.x; k < nb; k += kWsSelThreads * PARTS) {
            const int64_t gi = c->apply_idx[p * a.q_max + k];
            if (gi >= a.off && gi < a.off + a.nl) continue;
            if (t < 1.f) a.alpha[gi] = clip01(a.alpha[gi] - (1.f - t) * a.dalpha[gi], 0.f, a.C);
            a.dalpha[gi] = 0.f;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        if (has[r] && part == 0) {
          const int64_t j = base + r * kWsSelThreads;
          float d = a.dfs[j];
          for (int k = 1; k < a.ks; ++k) {
#pragma clang fp contract(off)
            d = d + a.dfs[(int64_t)k * a.nl + j];
          }
          acc[r] = t == 1.f ? d : t * d;
          const float dj = a.dalpha[a.off + j];
          if (dj != 0.f) {
            if (t < 1.f) a.alpha[a.off + j] = clip01(a.alpha[a.off + j] - (1.f - t) * dj, 0.f, a.C);
            a.dalpha[a.off + j] = 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
#pragma clang fp contract(off)
      f[r] = f[r] + acc[r];
    }
    bool bad = false;
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      if (has[r] && part == 0) a.f[base + r * kWsSelThreads] = f[r];
      bad |= has[r] && part == 0 && !isfinite(f[r]);
    }
    if (bad) atomicOr(&c->nonfinite, 1);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(10);
  if (done != kRunning) return;  // uniform

  // partition 0 (waves 0..3) classifies and extracts; the other waves idle to
  // the one barrier below (no wave leaves before it)
  uint64_t ku[RPT], kl[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    ku[r] = kl[r] = kKeyNone;
    if (has[r] && part == 0) {
      const int64_t gj = a.off + base + r * kWsSelThreads;
      const float av = a.alpha[gj], yv = a.y[gj];
      if (in_up(av, yv, a.C)) ku[r] = make_key(f[r], (uint32_t)gj);
      if (in_low(av, yv, a.C)) kl[r] = make_key(-f[r], (uint32_t)gj);
    }
  }
  // each wave's kWsCand smallest keys per side (DPP minima, no barrier), then
  // wave 0 merges the four lists; the owner of a winner drops it (keys are
  // unique: the global index is in the low bits)
  const int lane = tid & 63, wave = tid >> 6;
  // multi-block merges read kWsCand keys per list (MODE 2: every multi-block
  // round, the seed included), the one-block merge kWsCand1 (MODE 0)
  constexpr int nc = MODE == 0 ? kWsCand1 : kWsCand;
  for (int round = 0; round < nc && part == 0; ++round) {
    uint64_t mu = kKeyNone, ml = kKeyNone;
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      mu = ku[r] < mu ? ku[r] : mu;
      ml = kl[r] < ml ? kl[r] : ml;
    }
    mu = wave_min_u64(mu);
    ml = wave_min_u64(ml);
    if (lane == 0) {
      s_wc[wave][0][round] = mu;
      s_wc[wave][1][round] = ml;
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      if (ku[r] == mu) ku[r] = kKeyNone;
      if (kl[r] == ml) kl[r] = kKeyNone;
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    constexpr int W = kWsSelThreads / 64;
    const bool have = lane < W * kWsCand && (nc == kWsCand || lane % kWsCand < nc);  // the waves' nc entries
    uint64_t eu = have ? s_wc[lane / kWsCand][0][lane % kWsCand] : kKeyNone;
    uint64_t el = have ? s_wc[lane / kWsCand][1][lane % kWsCand] : kKeyNone;
    uint64_t* out = a.cand_out + (size_t)blockIdx.x * 2 * kWsCand;
    uint64_t pu[kWsCand1], pl[kWsCand1];  // uniform: every lane holds the first kWsCand1
    for (int round = 0; round < nc; ++round) {
      const uint64_t mu = wave_min_u64(eu), ml = wave_min_u64(el);
      if (lane == 0) {
        out[round] = mu;
        out[kWsCand + round] = ml;
      }
      if (round < kWsCand1) {
        pu[round] = mu;
        pl[round] = ml;
      }
      if (eu == mu) eu = kKeyNone;
      if (el == ml) el = kKeyNone;
    }
    if (a.xpeer != nullptr && lane < a.world) {  // lane p publishes to rank p
      uint64_t* dst = a.xpeer[lane] + ws_xcand(a, (int)(c->outer & 1), a.xrank * a.G + blockIdx.x);
      const uint64_t t = xtag((uint32_t)c->outer + 1u);
#pragma unroll
      for (int r = 0; r < kWsCand1; ++r) {
        xch_store<true>(dst + 2 * r, t | (pu[r] >> 16));
        xch_store<true>(dst + 2 * r + 1, t | (pu[r] & 0xffffull));
        xch_store<true>(dst + 2 * kWsCand1 + 2 * r, t | (pl[r] >> 16));
        xch_store<true>(dst + 2 * kWsCand1 + 2 * r + 1, t | (pl[r] & 0xffffull));
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(7);
}

// ---------------------------------------------------------------------------
// the merge: stop test and the new working set (one 256-thread workgroup;
// identical result in every workgroup that runs it).  Returns false when the
// run stopped (done is then set by workgroup 0).  s_idx[0..*q) = the set,
// newest first; *b_hi / *b_lo = the global selection.
// ---------------------------------------------------------------------------
__device__ bool ws_merge(const WsArgs& a, WsCtrl* c, int32_t* s_idx, int* q_out, float* bh_out, float* bl_out) {
  __shared__ int s_hist[2][256];
  __shared__ int s_sel[2][2];
  __shared__ int s_thr[2];
  __shared__ uint64_t s_wsum64[4];
  __shared__ uint64_t s_sv[2][kWsMaxCand];
  __shared__ int32_t s_hash[4][kWsHash];  // up keys, up ranks, low keys, low ranks
  __shared__ int32_t s_keep[2 * kWsMax];  // per interleaved position: final slot or -1
  __shared__ uint64_t s_scr[8];
  __shared__ int s_wsum[4];
  const int tid = threadIdx.x;
  const bool lead = blockIdx.x == 0 && tid == 0;
  if (c->done != kRunning) {
    // a round ended the run (max_iter / no pair): its changes were applied by
    // the ws_select that followed it; nothing may be applied twice
    if (lead) c->n_apply = 0;
    return false;
  }
  const int G = a.G_all;
  const int64_t r_now = c->outer;
  const int par = (int)(r_now & 1);
  const int q_prev = c->q[par ^ 1];
  const int want = q_prev == 0 ? a.q_max : min(a.n_new, a.q_max);
  // the previous set's row (read at the end) in the same load batch as the
  // candidate lists: one global round trip fewer on the merge's serial path
  const int32_t pidx_pre = tid < q_prev ? c->idx[par ^ 1][tid] : -1;

  // ---- every candidate list in registers: thread t holds lists t, t + 256,
  // ... (up to kWsListsPerThread, merged to one sorted top-kWsCand list per side:
  // the same as one selection workgroup over their rows) ----
  uint64_t lu[kWsCand1], ll[kWsCand1];
#pragma unroll
  for (int r = 0; r < kWsCand1; ++r) lu[r] = ll[r] = kKeyNone;
  bool ok = true;
  const uint64_t xt = xtag((uint32_t)r_now + 1u);
  for (int j = 0; j < kWsListsPerThread; ++j) {
    const int slot = tid + j * kWsGatherThreads;
    if (slot >= G) break;
    uint64_t cu[kWsCand1], cl[kWsCand1];
    if (a.xpeer == nullptr) {
#pragma unroll
      for (int r = 0; r < kWsCand1; ++r) {
        cu[r] = a.cand[(size_t)slot * 2 * kWsCand + r];
        cl[r] = a.cand[(size_t)slot * 2 * kWsCand + kWsCand + r];
      }
    } else {
      // peer exchange: poll slot `slot` of this rank's buffer
      const uint64_t* e = a.xpeer[a.xrank] + ws_xcand(a, par, slot);
      uint64_t g[4 * kWsCand1];
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (true) {
#pragma unroll
        for (int i = 0; i < 4 * kWsCand1; ++i) g[i] = xch_load<true>(e + i);
        bool all = true;
#pragma unroll
        for (int i = 0; i < 4 * kWsCand1; ++i) all &= ws_tag_ok(g[i], xt);
        if (all) break;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      constexpr uint64_t m48 = (1ull << 48) - 1;
#pragma unroll
      for (int r = 0; r < kWsCand1; ++r) {
        cu[r] = ((g[2 * r] & m48) << 16) | (g[2 * r + 1] & 0xffffull);
        cl[r] = ((g[2 * kWsCand1 + 2 * r] & m48) << 16) | (g[2 * kWsCand1 + 2 * r + 1] & 0xffffull);
      }
    }
    if (j == 0) {
#pragma unroll
      for (int r = 0; r < kWsCand1; ++r) {
        lu[r] = cu[r];
        ll[r] = cl[r];
      }
    } else {
      ws_top4_merge(lu, cu);
      ws_top4_merge(ll, cl);
    }
  }
  if (a.xpeer != nullptr && !__syncthreads_and(ok)) {
    ws_comm_fail(a, c);
    return false;
  }
  // ---- global minima (stop test) ----
  uint64_t gu = lu[0], gl = ll[0];
  block_min2_u64<kWsGatherThreads>(gu, gl, s_scr);
  const float b_hi = key_value(gu), b_lo = -key_value(gl);
  if (lead) WS_STAMP(11);
  const int64_t it0 = c->iter;
  int stop = kRunning;
  if (c->nonfinite) stop = kNonFinite;
  else if (gu == kKeyNone || gl == kKeyNone) stop = kNoPair;
  else if (!isfinite(b_hi) || !isfinite(b_lo)) stop = kNonFinite;
  else if (!(b_lo > b_hi + 2.0f * a.eps)) stop = kConverged;
  else if (it0 >= a.max_iter) stop = kMaxIter;
  if (stop != kRunning) {
    if (lead) {
      c->done = stop;
      c->n_apply = 0;  // applied by the last ws_select already
      c->b_hi = b_hi;
      c->b_lo = b_lo;
      ws_status(a.status, c);
    }
    return false;
  }

  // ---- per side, a 16-bit key prefix T: the rows whose prefix is <= T hold
  // >= m depth-d list entries, hence >= m (d + 1) >= ceil(want / 2)
  // candidates.  Two 8-bit radix passes over the depth-d entries (LDS
  // histograms): no sort.  The new rows are then taken by class — the global
  // extreme first, prefix < T, prefix == T — each class in list (row) order,
  // so a cut only ever drops rows of the boundary class. ----
  const int half = (want + 1) / 2;
  const int Gl = min(G, kWsGatherThreads);  // lists held (one merged list per thread)
  const int d = min(kWsCand1 - 1, (half + Gl - 1) / Gl - 1);
  const int m = (half + d) / (d + 1);
  uint64_t hd[2] = {lu[0], ll[0]};
#pragma unroll
  for (int r = 1; r < kWsCand1; ++r) {
    hd[0] = r == d ? lu[r] : hd[0];
    hd[1] = r == d ? ll[r] : hd[1];
  }
  for (int t = tid; t < 4 * kWsHash; t += kWsGatherThreads) (&s_hash[0][0])[t] = -1;
  s_hist[0][tid] = 0;
  s_hist[1][tid] = 0;
  __syncthreads();
#pragma unroll
  for (int sd = 0; sd < 2; ++sd)
    if (hd[sd] != kKeyNone) atomicAdd(&s_hist[sd][(int)(hd[sd] >> 56)], 1);
  __syncthreads();
  if (tid < 128) {  // wave 0: up side, wave 1: low side
    const int sd = tid >> 6;
    int below = 0;
    const int b1 = wave_find_bin(s_hist[sd], m, &below);
    if ((tid & 63) == 0) {
      s_sel[sd][0] = b1;
      s_sel[sd][1] = below;
    }
  }
  __syncthreads();
  s_hist[0][tid] = 0;
  s_hist[1][tid] = 0;
  __syncthreads();
#pragma unroll
  for (int sd = 0; sd < 2; ++sd)
    if (hd[sd] != kKeyNone && s_sel[sd][0] >= 0 && (int)(hd[sd] >> 56) == s_sel[sd][0])
      atomicAdd(&s_hist[sd][(int)(hd[sd] >> 48) & 255], 1);
  __syncthreads();
  if (tid < 128) {
    const int sd = tid >> 6;
    int below = 0;
    const int b1 = s_sel[sd][0];
    const int b2 = b1 >= 0 ? wave_find_bin(s_hist[sd], m - s_sel[sd][1], &below) : -1;
    if ((tid & 63) == 0) s_thr[sd] = b1 >= 0 && b2 >= 0 ? (b1 << 8) | b2 : 0xFFFF;  // too few: every row
  }
  __syncthreads();
  if (lead) WS_STAMP(12);
  const uint32_t T[2] = {(uint32_t)s_thr[0], (uint32_t)s_thr[1]};
  const uint64_t gmin[2] = {gu, gl};
  // class counts per thread (the global extreme is placed first, separately)
  uint64_t packed = 0;  // 12-bit fields: [up A, up B, low A, low B]
#pragma unroll
  for (int sd = 0; sd < 2; ++sd) {
#pragma unroll
    for (int r = 0; r < kWsCand1; ++r) {
      const uint64_t k = sd ? ll[r] : lu[r];
      if (k == kKeyNone || k == gmin[sd]) continue;
      const uint32_t pre = (uint32_t)(k >> 48);
      if (pre < T[sd]) packed += 1ull << (24 * sd);
      else if (pre == T[sd]) packed += 1ull << (24 * sd + 12);
    }
  }
  uint64_t ptot = 0;
  const uint64_t pofs = block_scan_fields(packed, s_wsum64, &ptot);
  int S[2];
#pragma unroll
  for (int sd = 0; sd < 2; ++sd) {
    const int totA = (int)((ptot >> (24 * sd)) & 4095), totB = (int)((ptot >> (24 * sd + 12)) & 4095);
    int oA = 1 + (int)((pofs >> (24 * sd)) & 4095), oB = 1 + totA + (int)((pofs >> (24 * sd + 12)) & 4095);
    S[sd] = 1 + totA + totB;
#pragma unroll
    for (int r = 0; r < kWsCand1; ++r) {
      const uint64_t k = sd ? ll[r] : lu[r];
      if (k == kKeyNone) continue;
      if (k == gmin[sd]) {
        s_sv[sd][0] = k;
        continue;
      }
      const uint32_t pre = (uint32_t)(k >> 48);
      if (pre < T[sd]) s_sv[sd][oA++] = k;
      else if (pre == T[sd]) s_sv[sd][oB++] = k;
    }
  }
  __syncthreads();

  if (lead) WS_STAMP(13);
  // ---- the new working set ----
  int32_t* hk_u = s_hash[0];
  int32_t* hv_u = s_hash[1];
  int32_t* hk_l = s_hash[2];
  int32_t* hv_l = s_hash[3];
  if (tid < want) {
    if (tid < S[0]) ws_hash_insert(hk_u, hv_u, (int32_t)key_index(s_sv[0][tid]), tid);
    if (tid < S[1]) ws_hash_insert(hk_l, hv_l, (int32_t)key_index(s_sv[1][tid]), tid);
  }
  __syncthreads();
  // interleaved positions 2r (up rank r), 2r + 1 (low rank r); a row's first
  // position wins; thread t owns positions 2t and 2t + 1
  bool kp[2] = {false, false};
  int32_t ki[2] = {-1, -1};
  if (tid < want) {
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      const uint64_t kk = tid < S[sd] ? s_sv[sd][tid] : kKeyNone;
      if (kk != kKeyNone) {
        ki[sd] = (int32_t)key_index(kk);
        if (sd == 0) {
          const int rl = ws_hash_find(hk_l, hv_l, ki[sd]);
          kp[sd] = !(rl >= 0 && rl < tid);
        } else {
          const int ru = ws_hash_find(hk_u, hv_u, ki[sd]);
          kp[sd] = !(ru >= 0 && ru <= tid);
        }
      }
    }
  }
  int kept = 0;
  const int slot0 = block_scan_small256((int)kp[0] + (int)kp[1], s_wsum, &kept);
  const int n_chosen = min(kept, want);
  if (tid < want) {
    const int s0 = slot0, s1 = slot0 + (int)kp[0];
    const bool c0 = kp[0] && s0 < want, c1 = kp[1] && s1 < want;
    s_keep[2 * tid] = c0 ? s0 : -1;
    s_keep[2 * tid + 1] = c1 ? s1 : -1;
    if (c0) s_idx[s0] = ki[0];
    if (c1) s_idx[s1] = ki[1];
  }
  __syncthreads();
  if (lead) WS_STAMP(14);
  // the previous set (newest first): rows not chosen again, up to q_max
  bool pk = false;
  int32_t pidx = -1;
  if (tid < q_prev) {
    pidx = pidx_pre;
    const int ru = ws_hash_find(hk_u, hv_u, pidx);
    const int rl = ws_hash_find(hk_l, hv_l, pidx);
    pk = !((ru >= 0 && s_keep[2 * ru] >= 0) || (rl >= 0 && s_keep[2 * rl + 1] >= 0));
  }
  int ptotal = 0;
  const int pslot = block_scan_small256((int)pk, s_wsum, &ptotal);
  if (pk && n_chosen + pslot < a.q_max) s_idx[n_chosen + pslot] = pidx;
  const int q = min(a.q_max, n_chosen + ptotal);
  __syncthreads();
  *q_out = q;
  *bh_out = b_hi;
  *bl_out = b_lo;
  return true;
}

// Row ra of the q_max-stride sub-Gram from line `line` (K(idx_ra, off + j) at
// line[j]), plus the row's f / alpha / y.  A rank fills only the columns (and
// the f) of rows it owns and zeros the rest, so at world > 1 one sum all-reduce
// assembles the exact matrix (each entry has exactly one owner).  Rows ra >= q
// are zeroed.
__device__ __forceinline__ void ws_gather_row(const WsArgs& a, WsCtrl* c, const int32_t* s_idx, int q, int ra,
                                              const float* line) {
  const int tid = threadIdx.x;
  float* dst = a.subg + (size_t)ra * a.q_max;
  if (ra >= q) {
    for (int b = tid; b < a.q_max; b += kWsGatherThreads) dst[b] = 0.f;
    if (tid == 0) a.aux[ra] = 0.f;
    return;
  }
  const int64_t lo = a.off, hi = a.off + a.nl;
  if (a.xpeer != nullptr) {
    // peer exchange: push the owned entries of row ra (+ its f) to every rank,
    // then poll this rank's copy of the row (q_max <= 192 < 256: one column per
    // thread, the last thread takes f)
    const int64_t R = c->outer;
    const uint64_t t = xtag((uint32_t)R + 1u);
    const int64_t row = ws_xrow(a, (int)(R & 1), ra);
    constexpr int kF = kWsGatherThreads - 1;
    const int64_t gi = s_idx[ra];
    if (tid < q) {
      const int64_t gj = s_idx[tid];
      if (gj >= lo && gj < hi) {
        const uint64_t v = t | __float_as_uint(line[gj - lo]);
        for (int p = 0; p < a.world; ++p) xch_store<true>(a.xpeer[p] + row + tid, v);
      }
    } else if (tid == kF && gi >= lo && gi < hi) {
      const uint64_t v = t | __float_as_uint(a.f[gi - lo]);
      for (int p = 0; p < a.world; ++p) xch_store<true>(a.xpeer[p] + row + a.q_max, v);
    }
    bool ok = true;
    const int col = tid < q ? tid : tid == kF ? a.q_max : -1;
    if (col >= 0) {
      const uint64_t* g = a.xpeer[a.xrank] + row + col;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t v = xch_load<true>(g);
      while (!ws_tag_ok(v, t)) {
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = xch_load<true>(g);
      }
      const float fv = __uint_as_float((uint32_t)v);
      if (tid == kF) a.aux[ra] = fv;
      else dst[tid] = fv;
    } else if (tid < a.q_max) {
      dst[tid] = 0.f;
    }
    if (tid == 0) {
      a.aux[a.aux_stride + ra] = a.alpha[gi];
      a.aux[2 * a.aux_stride + ra] = a.y[gi];
    }
    if (!__syncthreads_and(ok)) ws_comm_fail(a, c);
    return;
  }
  for (int b = tid; b < a.q_max; b += kWsGatherThreads) {
    const int64_t gj = b < q ? (int64_t)s_idx[b] : -1;
    dst[b] = gj >= lo && gj < hi ? line[gj - lo] : 0.f;
  }
  if (tid == 0) {
    const int64_t gi = s_idx[ra];
    a.aux[ra] = gi >= lo && gi < hi ? a.f[gi - lo] : 0.f;
    a.aux[a.aux_stride + ra] = a.alpha[gi];
    a.aux[2 * a.aux_stride + ra] = a.y[gi];
  }
}

// ---------------------------------------------------------------------------
// ws_gather (dense mode): the merge in every workgroup + one sub-Gram row per
// workgroup (row a: q random columns of Gram row idx_a — one load per thread;
// the whole grid issues the scattered reads a single CU could not)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kWsGatherThreads) void ws_gather_kernel(WsArgs a) {
  __shared__ int32_t s_idx[kWsMax];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  const bool lead = blockIdx.x == 0 && tid == 0;
  if (lead) WS_STAMP(1);
  const int par = (int)(c->outer & 1);
  int q = 0;
  float b_hi = 0.f, b_lo = 0.f;
  if (!ws_merge(a, c, s_idx, &q, &b_hi, &b_lo)) return;
  if (lead) WS_STAMP(2);
  if (blockIdx.x == 0) {
    for (int t = tid; t < q; t += kWsGatherThreads) {
      c->idx[par][t] = s_idx[t];
      c->line[par][t] = s_idx[t];  // the resident Gram: line i is row i
    }
    if (tid == 0) {
      c->q[par] = q;
      c->b_hi = b_hi;
      c->b_lo = b_lo;
    }
  }
  ws_gather_row(a, c, s_idx, q, blockIdx.x, blockIdx.x < q ? a.gram + (int64_t)s_idx[blockIdx.x] * a.ldg : nullptr);
  if (lead) WS_STAMP(8);
}

// ---------------------------------------------------------------------------
// cache mode, round part 1 — ws_merge (ONE workgroup): the merge, then lines
// for the members: a member's row is cached (slot_of) or takes a victim line.
// Victims come from a window of up to 512 lines after the CLOCK hand, skipping
// lines that hold a member (pinned while the round uses them); all misses are
// assigned at once (one prefix scan), their rows computed next by one GEMM.
// ---------------------------------------------------------------------------
constexpr int kWsWindow = 512;

__global__ __launch_bounds__(kWsGatherThreads) void ws_merge_kernel(WsArgs a) {
  __shared__ int32_t s_idx[kWsMax];
  __shared__ int32_t s_line[kWsMax];
  __shared__ int32_t s_pin[kWsWindow];
  __shared__ int32_t s_victim[kWsMax];
  __shared__ int s_wsum[4];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  if (tid == 0) WS_STAMP(1);
  const int par = (int)(c->outer & 1);
  int q = 0;
  float b_hi = 0.f, b_lo = 0.f;
  if (!ws_merge(a, c, s_idx, &q, &b_hi, &b_lo)) return;
  if (tid == 0) WS_STAMP(2);
  const int L = a.L, hand = c->hand;
  const int W = min(L, kWsWindow);
  for (int w = tid; w < kWsWindow; w += kWsGatherThreads) s_pin[w] = 0;
  __syncthreads();
  int32_t my_line = -1, my_row = -1;
  if (tid < q) {
    my_row = s_idx[tid];
    my_line = a.slot_of[my_row];
    if (my_line >= 0) {
      const int o = (my_line - hand + L) % L;
      if (o < W) s_pin[o] = 1;
    }
  }
  __syncthreads();
  int n_miss = 0;
  const bool miss = tid < q && my_line < 0;
  const int mrank = block_scan_small256((int)miss, s_wsum, &n_miss);
  // free window slots 2t, 2t + 1 in window order
  const bool f0 = 2 * tid < W && !s_pin[2 * tid], f1 = 2 * tid + 1 < W && !s_pin[2 * tid + 1];
  int n_free = 0;
  const int frank = block_scan_small256((int)f0 + (int)f1, s_wsum, &n_free);
  int last_used = -1;
  if (f0 && frank < n_miss) {
    s_victim[frank] = (hand + 2 * tid) % L;
    last_used = 2 * tid;
  }
  if (f1 && frank + (int)f0 < n_miss) {
    s_victim[frank + (int)f0] = (hand + 2 * tid + 1) % L;
    last_used = 2 * tid + 1;
  }
  __syncthreads();
  if (miss) {  // n_free >= W - q >= n_miss whenever L >= q + 256 (setup guarantees L >= 2 q_max + 512)
    const int32_t ln = s_victim[mrank];
    const int32_t old = a.key_of[ln];
    if (old >= 0) a.slot_of[old] = -1;  // evicted (never a member: members' lines are pinned)
    a.key_of[ln] = my_row;
    a.slot_of[my_row] = ln;
    my_line = ln;
    c->miss_row[mrank] = my_row;
    c->miss_line[mrank] = ln;
  }
  if (tid < q) {
    c->idx[par][tid] = my_row;
    c->line[par][tid] = my_line;
  }
  if (n_miss > 0 && last_used >= 0 && (frank + (int)f0 + (int)f1 >= n_miss) && (frank < n_miss))
    c->hand = (hand + last_used + 1) % L;  // the thread holding the last victim
  if (tid == 0) {
    c->q[par] = q;
    c->b_hi = b_hi;
    c->b_lo = b_lo;
    c->n_miss = n_miss;
    c->rows_computed += n_miss;
    c->row_hits += q - n_miss;
  }
}

// cache mode, round part 3 — ws_gather_lines (q_max workgroups): row a of the
// sub-Gram from member a's line, its alpha / y / f
__global__ __launch_bounds__(kWsGatherThreads) void ws_gather_lines_kernel(WsArgs a) {
  __shared__ int32_t s_idx[kWsMax];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  if (c->done != kRunning) return;
  const int par = (int)(c->outer & 1);
  const int q = c->q[par];
  const int ra = blockIdx.x;
  if (ra >= q) {
    ws_gather_row(a, c, s_idx, q, ra, nullptr);
    return;
  }
  for (int t = tid; t < q; t += kWsGatherThreads) s_idx[t] = c->idx[par][t];
  __syncthreads();
  ws_gather_row(a, c, s_idx, q, ra, a.gram + (int64_t)c->line[par][ra] * a.ldg);
  if (tid == 0 && ra == 0) WS_STAMP(8);
}

// ---------------------------------------------------------------------------
// multi-block rounds (a.blocks = P > 1; ws-dense at world 1).  The grid-wide
// work of a round (merge, f update, candidates) is shared by P sub-problems
// solved at once on P workgroups (the one-wave solve leaves the other CUs
// idle): ws_merge_multi picks up to P q_max rows, ws_gather_multi their P
// diagonal q x q blocks, ws_solve<kMulti> one block per workgroup, and the
// two-pass ws_select applies the combined step with the exact line search.
// ---------------------------------------------------------------------------
// exclusive prefix of counts 0 .. 2^BITS - 1 over kWsMergeThreads threads in
// thread order (bit-plane ballots)
template <int BITS = 2>
__device__ __forceinline__ int block_scan_merge(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  int pre = 0, wtot = 0;
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const uint64_t m = __ballot((v >> b) & 1);
    pre += __popcll(m & below) << b;
    wtot += __popcll(m) << b;
  }
  if (lane == 0) wsum[wave] = wtot;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWsMergeThreads / 64; ++w) {
    off += w < wave ? wsum[w] : 0;
    tot += wsum[w];
  }
  *total = tot;
  __syncthreads();
  return off + pre;
}

// ONE workgroup: every candidate key of both sides sorted (bitonic, 2048 per
// side, two per thread), the stop test, then the union: up rank r / low rank r
// interleaved (most violating first, a row's first position wins), then the
// newest rows of the previous union.  Union position i goes to block
// ((i / 2) mod P): each block gets up / low pairs, block 0 the global extremes
// (so a round always holds the maximal violating pair and makes progress).
constexpr int kMH = 4096;  // merge hash slots per side (load <= 0.38)
constexpr int kWsWindowMulti = 8192;  // cache mode: CLOCK victim window of the multi-block merge
__device__ __forceinline__ uint32_t mh_hash(int32_t idx) { return ((uint32_t)idx * 2654435761u) >> 20; }
__device__ __forceinline__ void mh_insert(int32_t* keys, int32_t* vals, int32_t idx, int32_t v) {
  uint32_t h = mh_hash(idx);
  while (true) {
    const int32_t old = atomicCAS(keys + h, -1, idx);
    if (old == -1) {
      vals[h] = v;
      return;
    }
    h = (h + 1) & (kMH - 1);
  }
}
__device__ __forceinline__ int32_t mh_find(const int32_t* keys, const int32_t* vals, int32_t idx) {
  uint32_t h = mh_hash(idx);
  for (int probe = 0; probe < kMH; ++probe) {
    const int32_t k = keys[h];
    if (k == idx) return vals[h];
    if (k == -1) return -1;
    h = (h + 1) & (kMH - 1);
  }
  return -1;
}

// ws_rank: the multi-block merge's sort, spread over a grid of 2 sides x
// kRankChunks workgroups instead of one workgroup's bitonic network (29 of the
// merge's 41 us at 3,072-row unions, profiles/r3_ws_stamps_32x96.json).  A
// key's position in its side's ascending order is the number of keys below it:
// real keys are unique (the global row index is in the low bits), so these
// counts are a permutation of [0, n_real); the absent keys (kKeyNone) fill the
// tail.  Each workgroup holds its side's NK keys in LDS and ranks KPW of them,
// SUB = 16 threads per key each counting over every SUB-th key pair (the SUB
// lanes of one key read 16 consecutive 16-B pairs: no bank conflict, broadcast
// over keys).
constexpr int kRankThreads = 512;
constexpr int kRankChunks = 64;
__global__ __launch_bounds__(kRankThreads) void ws_rank_kernel(WsArgs a) {
  constexpr int NK = kWsMaxGroups * kWsCand;
  constexpr int KPW = NK / kRankChunks, SUB = kRankThreads / KPW, PAIRS = NK / (2 * SUB);
  static_assert(NK % kRankChunks == 0 && kRankThreads % KPW == 0 && SUB == 16 && NK % (2 * SUB) == 0, "rank geometry");
  __shared__ uint64_t s_k[NK];
  __shared__ int s_real[kRankThreads / 64];
  const WsCtrl* c = a.ctrl;
  if (c->done != kRunning) return;
  const int side = blockIdx.x / kRankChunks, chunk = blockIdx.x % kRankChunks, tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) WS_STAMP(21);
  const int G = a.G_all;
  int real = 0;
  for (int e = tid; e < NK; e += kRankThreads) {
    const int l = e / kWsCand, r = e % kWsCand;
    const uint64_t k = l < G ? a.cand[(size_t)l * 2 * kWsCand + side * kWsCand + r] : kKeyNone;
    s_k[e] = k;
    real += k != kKeyNone ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) real += __shfl_xor(real, o);
  if ((tid & 63) == 0) s_real[tid >> 6] = real;
  __syncthreads();
  int n_real = 0;
#pragma unroll
  for (int w = 0; w < kRankThreads / 64; ++w) n_real += s_real[w];
  const int e = chunk * KPW + tid / SUB, sub = tid % SUB;
  const uint64_t k = s_k[e];
  int cnt = 0;
#pragma unroll 8
  for (int i = 0; i < PAIRS; ++i) {
    const int e2 = 2 * (sub + SUB * i);
    cnt += (s_k[e2] < k ? 1 : 0) + (s_k[e2 + 1] < k ? 1 : 0);
  }
#pragma unroll
  for (int o = 1; o < SUB; o <<= 1) cnt += __shfl_xor(cnt, o);
  uint64_t* out = a.sorted + (size_t)side * NK;
  if (sub == 0 && k != kKeyNone) out[cnt] = k;
  if (tid < KPW && chunk * KPW + tid >= n_real) out[chunk * KPW + tid] = kKeyNone;
}

__global__ __launch_bounds__(kWsMergeThreads) void ws_merge_multi_kernel(WsArgs a) {
  constexpr int T = kWsMergeThreads;
  constexpr int NK = kWsMaxGroups * kWsCand;  // keys per side
  constexpr int U = kWsMaxAll / T;            // previous-union rows per thread
  static_assert(NK == 2 * T, "two keys per thread and side: elements tid and tid + T");
  static_assert(kWsMaxAll % T == 0 && U <= 3, "previous union: <= 3 rows per thread (scan counts <= 3)");
  static_assert(kMH >= kWsMaxAll && kWsWindowMulti == 8 * T, "cache-mode aliases of the hash tables / sort keys");
  __shared__ uint64_t s_k[2][NK];
  __shared__ int32_t s_hash[4][kMH];
  __shared__ int32_t s_keep[kWsMaxAll + 2];
  __shared__ int32_t s_idx[kWsMaxAll];
  __shared__ int s_wsum[T / 64];
  __shared__ int s_qb[kWsMaxBlocks];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  const bool lead = tid == 0;
  if (c->done != kRunning) {
    if (lead) c->n_apply = 0;  // applied by the last ws_select already
    return;
  }
  if (lead) WS_STAMP(1);
  const int G = a.G_all;
  const int par = (int)(c->outer & 1);
  const int P = max(1, min(c->p_act, a.blocks)), Qmax = P * a.q_max;
  const int q_prev = c->uq[par ^ 1];
  const int want = q_prev == 0 ? Qmax : min(P * a.n_new, Qmax);
  // the previous union, newest first: thread t holds rows U t .. U t + U - 1
  int32_t pidx[U];
#pragma unroll
  for (int h = 0; h < U; ++h) pidx[h] = U * tid + h < q_prev ? c->uidx[par ^ 1][U * tid + h] : -1;
  // keys e = tid and e = tid + T of each side, in ascending order (ws_rank)
  uint64_t v[2][2];  // [side][element]
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    v[0][x] = a.sorted[tid + x * T];
    v[1][x] = a.sorted[NK + tid + x * T];
  }
  if (tid < kWsMaxBlocks) s_qb[tid] = 0;
  for (int t = tid; t < 4 * kMH; t += T) (&s_hash[0][0])[t] = -1;
  if (lead) WS_STAMP(20);
#pragma unroll
  for (int sd = 0; sd < 2; ++sd) {
    s_k[sd][tid] = v[sd][0];
    s_k[sd][tid + T] = v[sd][1];
  }
  __syncthreads();
  if (lead) WS_STAMP(11);
  const uint64_t gu = s_k[0][0], gl = s_k[1][0];
  const float b_hi = key_value(gu), b_lo = -key_value(gl);
  const int64_t it0 = c->iter;
  int stop = kRunning;
  if (c->nonfinite) stop = kNonFinite;
  else if (gu == kKeyNone || gl == kKeyNone) stop = kNoPair;
  else if (!isfinite(b_hi) || !isfinite(b_lo)) stop = kNonFinite;
  else if (!(b_lo > b_hi + 2.0f * a.eps)) stop = kConverged;
  else if (it0 >= a.max_iter) stop = kMaxIter;
  if (stop != kRunning) {
    if (lead) {
      c->done = stop;
      c->n_apply = 0;
      c->b_hi = b_hi;
      c->b_lo = b_lo;
      ws_status(a.status, c);
    }
    return;
  }
  int32_t* hk_u = s_hash[0];
  int32_t* hv_u = s_hash[1];
  int32_t* hk_l = s_hash[2];
  int32_t* hv_l = s_hash[3];
  const int half = (want + 1) / 2;  // <= kWsMaxAll / 2 = T + T / 2 ranks per side
  uint64_t ku[2], kl[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int e = tid + x * T;
    ku[x] = e < half ? v[0][x] : kKeyNone;
    kl[x] = e < half ? v[1][x] : kKeyNone;
    if (ku[x] != kKeyNone) mh_insert(hk_u, hv_u, (int32_t)key_index(ku[x]), e);
    if (kl[x] != kKeyNone) mh_insert(hk_l, hv_l, (int32_t)key_index(kl[x]), e);
  }
  __syncthreads();
  if (lead) WS_STAMP(12);
  // rank e keeps its up row unless the low side has it at a smaller rank, its
  // low row unless the up side has it at a rank <= e (the up copy comes first)
  bool kpu[2] = {false, false}, kpl[2] = {false, false};
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int e = tid + x * T;
    if (ku[x] != kKeyNone) {
      const int rl = mh_find(hk_l, hv_l, (int32_t)key_index(ku[x]));
      kpu[x] = !(rl >= 0 && rl < e);
    }
    if (kl[x] != kKeyNone) {
      const int ru = mh_find(hk_u, hv_u, (int32_t)key_index(kl[x]));
      kpl[x] = !(ru >= 0 && ru <= e);
    }
  }
  // union order: ranks 0 .. T - 1 (element 0 of threads in order), then ranks
  // T .. (element 1): two scans
  int tot0 = 0, tot1 = 0;
  const int slot0 = block_scan_merge((int)kpu[0] + (int)kpl[0], s_wsum, &tot0);
  const int slot1 = tot0 + block_scan_merge((int)kpu[1] + (int)kpl[1], s_wsum, &tot1);
  const int kept = tot0 + tot1;
  const int n_chosen = min(kept, want);
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int e = tid + x * T;
    if (e < half) {
      const int su = x == 0 ? slot0 : slot1, sl = su + (int)kpu[x];
      const bool cu = kpu[x] && su < want, cl = kpl[x] && sl < want;
      s_keep[2 * e] = cu ? su : -1;
      s_keep[2 * e + 1] = cl ? sl : -1;
      if (cu) s_idx[su] = (int32_t)key_index(ku[x]);
      if (cl) s_idx[sl] = (int32_t)key_index(kl[x]);
    }
  }
  __syncthreads();
  if (lead) WS_STAMP(13);
  // previous-union rows not chosen again keep their order after the new rows
  // (uniform skip when the new rows already fill the union)
  bool pk[U];
  int npk = 0;
#pragma unroll
  for (int h = 0; h < U; ++h) {
    pk[h] = false;
    if (n_chosen < Qmax && pidx[h] >= 0) {
      const int ru = mh_find(hk_u, hv_u, pidx[h]), rl = mh_find(hk_l, hv_l, pidx[h]);
      pk[h] = !((ru >= 0 && s_keep[2 * ru] >= 0) || (rl >= 0 && s_keep[2 * rl + 1] >= 0));
    }
    npk += (int)pk[h];
  }
  int ptotal = 0;
  if (n_chosen < Qmax) {  // uniform
    int at = n_chosen + block_scan_merge(npk, s_wsum, &ptotal);
#pragma unroll
    for (int h = 0; h < U; ++h) {
      if (pk[h]) {
        if (at < Qmax) s_idx[at] = pidx[h];
        ++at;
      }
    }
  }
  const int Q = min(Qmax, n_chosen + ptotal);
  __syncthreads();
  if (lead) WS_STAMP(14);
  if (a.cache) {
    // ---- kernel-row cache: a line for every union row.  A member's row is
    // cached (slot_of) or takes a victim from the window of kWsWindowMulti
    // lines after the CLOCK hand, skipping lines that hold a member (pinned
    // while the round uses them); all misses at once (prefix scans), their
    // rows computed next by one row GEMM.  Setup guarantees
    // L >= 2 Qmax + kWsWindowMulti, so the window holds >= n_miss free lines. ----
    int32_t* s_pin = (int32_t*)&s_k[0][0];  // the sort keys are dead: 8192 words
    int32_t* s_victim = s_hash[0];         // the hash tables too: kMH words each
    int32_t* s_line = s_hash[1];
    const int L = a.L, hand = c->hand;
    const int W = min(L, kWsWindowMulti);
    for (int w = tid; w < kWsWindowMulti; w += T) s_pin[w] = 0;
    __syncthreads();
    int32_t ln[U];
#pragma unroll
    for (int h = 0; h < U; ++h) {
      ln[h] = -1;
      const int u = tid + h * T;
      if (u < Q) {
        ln[h] = a.slot_of[s_idx[u]];
        if (ln[h] >= 0) {
          const int o = (ln[h] - hand + L) % L;
          if (o < W) s_pin[o] = 1;
        }
      }
    }
    __syncthreads();
    // misses in union order: element h of every thread is union row tid + h T,
    // so one scan per h
    int mrank[U], n_miss = 0;
#pragma unroll
    for (int h = 0; h < U; ++h) {
      const bool mh = tid + h * T < Q && ln[h] < 0;
      int tot = 0;
      mrank[h] = n_miss + block_scan_merge<1>((int)mh, s_wsum, &tot);
      n_miss += tot;
    }
    // free window slots SPT t .. SPT t + SPT - 1 in window order
    constexpr int SPT = kWsWindowMulti / T;
    bool fr[SPT];
    int nf = 0;
#pragma unroll
    for (int k = 0; k < SPT; ++k) {
      fr[k] = SPT * tid + k < W && !s_pin[SPT * tid + k];
      nf += (int)fr[k];
    }
    int n_free = 0;
    const int frank = block_scan_merge<4>(nf, s_wsum, &n_free);
    int at = frank, last_used = -1;
#pragma unroll
    for (int k = 0; k < SPT; ++k) {
      if (fr[k]) {
        if (at < n_miss) {
          s_victim[at] = (hand + SPT * tid + k) % L;
          last_used = SPT * tid + k;
        }
        ++at;
      }
    }
    __syncthreads();
    if (last_used >= 0 && frank < n_miss && at >= n_miss) c->hand = (hand + last_used + 1) % L;  // the last victim
#pragma unroll
    for (int h = 0; h < U; ++h) {
      const int u = tid + h * T;
      if (u < Q && ln[h] < 0) {
        const int r = mrank[h];
        const int32_t row = s_idx[u];
        const int32_t vl = s_victim[r];
        const int32_t old = a.key_of[vl];
        if (old >= 0) a.slot_of[old] = -1;  // evicted (never a member: members' lines are pinned)
        a.key_of[vl] = row;
        a.slot_of[row] = vl;
        c->miss_row[r] = row;
        c->miss_line[r] = vl;
        ln[h] = vl;
      }
      if (u < Q) s_line[u] = ln[h];
    }
    if (lead) {
      c->n_miss = n_miss;
      c->rows_computed += n_miss;
      c->row_hits += Q - n_miss;
    }
    __syncthreads();
  }
  for (int u = tid; u < Q; u += T) {
    const int32_t row = s_idx[u];
    c->uidx[par][u] = row;
    const int pi = u >> 1, b = pi % P, la = 2 * (pi / P) + (u & 1);
    c->idx[par][b * a.q_max + la] = row;
    c->line[par][b * a.q_max + la] = a.cache ? s_hash[1][u] : row;  // cache: s_line; dense: line i is row i
    atomicMax(&s_qb[b], la + 1);
  }
  __syncthreads();
  if (tid < a.blocks) c->qb[par][tid] = s_qb[tid];  // inactive blocks: 0 rows
  if (lead) {
    c->uq[par] = Q;
    c->q[par] = Q;
    c->p_round = P;
    c->b_hi = b_hi;
    c->b_lo = b_lo;
    WS_STAMP(2);
  }
}


// P x q_max workgroups: workgroup p q_max + a gathers row a of block p's
// sub-Gram (block p's columns) and the row's f / alpha / y
__global__ __launch_bounds__(kWsGatherThreads) void ws_gather_multi_kernel(WsArgs a) {
  __shared__ int32_t s_idx[kWsMax];
  WsCtrl* c = a.ctrl;
  if (c->done != kRunning) return;
  const int tid = threadIdx.x;
  const int par = (int)(c->outer & 1);
  const int p = (int)blockIdx.x / a.q_max, ra = (int)blockIdx.x % a.q_max;
  const int q = c->qb[par][p];
  WsArgs b = a;
  b.subg = a.subg + (size_t)p * a.q_max * a.q_max;
  b.aux = a.aux + (size_t)p * kWsMax;  // f / alpha / y of block p at stride aux_stride
  if (ra >= q) {
    ws_gather_row(b, c, s_idx, q, ra, nullptr);
    return;
  }
  for (int t = tid; t < q; t += kWsGatherThreads) s_idx[t] = c->idx[par][p * a.q_max + t];
  __syncthreads();
  // the row's line (dense: the resident Gram's row itself)
  const int64_t line = a.cache ? (int64_t)c->line[par][p * a.q_max + ra] : (int64_t)s_idx[ra];
  ws_gather_row(b, c, s_idx, q, ra, a.gram + line * a.ldg);
  if (tid == 0 && blockIdx.x == 0) WS_STAMP(8);
}

// ---------------------------------------------------------------------------
// ws_solve: the sub-problem on wave 0
// ---------------------------------------------------------------------------
// Row `pos` (uniform) took alpha `an` and now has gradient fp (both uniform,
// computed from values every lane holds): its I_up / I_low test
// (svmTrain.cu:56-91) as mask logic on uniform operands, then the owner lane's
// slot registers take the new fu / fl by selects.  No branch (every branch of a
// one-wave loop is a fetch bubble) and no per-lane recomputation.
// per lane: the lanes set in the (uniform) mask m take b, the others keep a
__device__ __forceinline__ float sel_lanes(float a, float b, uint64_t m) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}

template <int NS>
__device__ __forceinline__ void ws_place(int pos, float an, float yv, float fp, int lane, float C, float (&fu)[NS],
                                         float (&fl)[NS]) {
  const float INF = __builtin_inff();
  // the operands are uniform: each test as a wave mask (all ones or zero; wave
  // 0 runs with a full exec mask) keeps the set logic on the scalar unit
  // instead of 0/1 VGPRs (~20 VALU per placement)
  // with alpha in [0, C] (clipped), in_up(a, y) == (y > 0 ? a < C : a > 0) and
  // in_low(a, y) == (y > 0 ? a > 0 : a < C) (common.hpp): three compares
  const uint64_t lt = __ballot(an < C), gt = __ballot(an > 0.f), py = __ballot(yv > 0.f);
  const float nu = (((py & lt) | (~py & gt)) != 0) ? fp : INF;
  const float nl = (((py & gt) | (~py & lt)) != 0) ? -fp : INF;
  // the owner lane of slot pos >> 6 as a scalar lane mask per slot, applied by
  // v_cndmask straight from the SGPR pair (no per-lane compare)
  const uint64_t bit = 1ull << (pos & 63);
  const int s = pos >> 6;
  (void)lane;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const uint64_t w = s == k ? bit : 0ull;
    fu[k] = sel_lanes(fu[k], nu, w);
    fl[k] = sel_lanes(fl[k], nl, w);
  }
}

// The reference's pair update (svmTrainMain.cpp:282-295; pair_update in
// common.hpp, same clipping modes) on uniform operands, with the quotient
// y_lo (b_hi - b_lo) / eta from a refined hardware reciprocal: the sub-problem
// step needs no bit parity with the pair-at-a-time engines (f is updated from
// the alphas actually taken, so it stays consistent), and the IEEE division
// sequence is the longest dependent chain of a step.
template <bool kBox>
__device__ __forceinline__ PairUpdate ws_pair_step(float a_hi, float a_lo, float y_hi, float y_lo, float bh, float bl,
                                                   float khl, float C, float tau, bool same, bool* clipped) {
#pragma clang fp contract(off)
  float eta = (1.0f + 1.0f) - 2.0f * khl;
  eta = eta >= tau ? eta : tau;
  float r = __builtin_amdgcn_rcpf(eta);
  r = r + r * __builtin_fmaf(-eta, r, 1.0f);  // one Newton step: ~0.5 ulp
  const float s = y_lo * y_hi;
  float a_lo_new = a_lo + (y_lo * (bh - bl)) * r;
  float a_hi_new;
  if (kBox && !same) {
    float L, H, hL, hH;
    if (y_hi != y_lo) {
      const float dl = a_lo - a_hi;
      L = dl > 0.f ? dl : 0.f;
      hL = dl > 0.f ? 0.f : -1.f;
      H = C + dl < C ? C + dl : C;
      hH = C + dl < C ? C : -1.f;
    } else {
      const float sm = a_lo + a_hi;
      L = sm - C > 0.f ? sm - C : 0.f;
      hL = sm - C > 0.f ? C : -1.f;
      H = sm < C ? sm : C;
      hH = sm < C ? 0.f : -1.f;
    }
    const bool atL = a_lo_new <= L, atH = !atL && a_lo_new >= H;
    a_lo_new = atL ? L : (atH ? H : a_lo_new);
    const float snap = atL ? hL : (atH ? hH : -1.f);
    a_hi_new = snap >= 0.f ? snap : a_hi + (s * (a_lo - a_lo_new));
    a_hi_new = clip01(a_hi_new, 0.0f, C);
  } else {
    a_hi_new = a_hi + (s * (a_lo - a_lo_new));
    const float lo_raw = a_lo_new, hi_raw = a_hi_new;
    a_lo_new = clip01(a_lo_new, 0.0f, C);
    a_hi_new = clip01(a_hi_new, 0.0f, C);
    *clipped = (lo_raw != a_lo_new) | (hi_raw != a_hi_new);  // sum(alpha y) no longer kept
  }
  PairUpdate u;
  u.a_hi_new = a_hi_new;
  u.a_lo_new = a_lo_new;
  u.c_hi = (a_hi_new - a_hi) * y_hi;
  u.c_lo = (a_lo_new - a_lo) * y_lo;
  return u;
}

// lowest working-set position whose value equals the (uniform) minimum v
// (-1: none, i.e. NaN); scalar selects, no branch
// s_ff1 of an SGPR-pair mask: the lowest set bit, 0xFFFFFFFF when none (the
// builtins add a zero test and a select per mask)
__device__ __forceinline__ uint32_t sff1_u64(uint64_t m) {
  uint32_t r;
  asm volatile("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m));
  return r;
}

__device__ __forceinline__ int ws_argpos(const float (&x)[3], float v) {
  const uint64_t m0 = __ballot(x[0] == v), m1 = __ballot(x[1] == v), m2 = __ballot(x[2] == v);
  // slot s's first lane | 64 s (none stays all ones), the lowest valid one wins
  // as an unsigned minimum: 3 compares, 3 s_ff1, 2 s_or, 2 s_min
  const uint32_t r0 = sff1_u64(m0), r1 = sff1_u64(m1) | 64u, r2 = sff1_u64(m2) | 128u;
  uint32_t r;
  asm volatile("s_min_u32 %0, %1, %2\n\ts_min_u32 %0, %0, %3" : "=&s"(r) : "s"(r0), "s"(r1), "s"(r2));
  return (int)r;
}

__device__ __forceinline__ int ws_argpos(const float (&x)[2], float v) {
  const uint64_t m0 = __ballot(x[0] == v), m1 = __ballot(x[1] == v);
  const uint32_t r0 = sff1_u64(m0), r1 = sff1_u64(m1) | 64u;
  uint32_t r;
  asm volatile("s_min_u32 %0, %1, %2" : "=s"(r) : "s"(r0), "s"(r1));
  return (int)r;
}

// kFull: q_max == kWsMax, the three 64-row slots fill a sub-Gram row (stride
// 192): row reads need no clamp (columns q..191 hold zeros) and take immediate
// LDS offsets
// kW2: second-order choice of the low row (Fan, Chen & Lin's WSS2, the rule
// LIBSVM uses): hi = argmin f over I_up as in the reference, then lo = the
// I_low row with f_lo > b_hi that maximises (f_lo - b_hi)^2 / eta(hi, lo) —
// the pair whose step gains the most dual objective — instead of argmax f.
// The stop test stays the reference's first-order one (b_lo = max f over I_low).
// NS: 64-row slots per lane (3 for q_max <= 192, 2 for q_max <= 128 — the
// multi-block rounds' 96-row blocks: a third less work per pair step)
template <bool kBox, bool kFull, bool kMulti, bool kW2, int NS = 3>
__global__ __launch_bounds__(kWsSolveThreads) void ws_solve_kernel(WsArgs a) {
  static_assert(NS == 3 || (NS == 2 && !kFull), "slots");
  extern __shared__ __attribute__((aligned(16))) float K[];  // q rows of the sub-Gram, stride q_max
  __shared__ float s_a[kWsMax + 128], s_y[kWsMax], s_f[kWsMax];  // s_a: + 2 x 64 scratch words
  __shared__ int32_t s_idx[kWsMax], s_line[kWsMax];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) WS_STAMP(0);
  if (c->done != kRunning) return;
  const int par = (int)(c->outer & 1);
  // multi-block rounds: workgroup p solves block p (rows idx[par][p q_max ..])
  const int blk = kMulti ? (int)blockIdx.x : 0;
  const int q = kMulti ? c->qb[par][blk] : c->q[par];
  const float b_hi = c->b_hi, b_lo = c->b_lo;
  const int64_t it0 = c->iter;
  const int ldk = a.q_max;  // LDS keeps the q_max stride: the load is one contiguous copy
  const int ib = blk * a.q_max;
  const float* subg = a.subg + (size_t)blk * ldk * ldk;
  const float* aux = a.aux + (size_t)blk * kWsMax;
  {
    // q rows of the q_max-stride sub-Gram into LDS (147 KiB at q = 192): 16-B
    // loads, four in flight per thread before their stores
    const int n = q * ldk;
    if ((ldk & 3) == 0) {
      const f4* src = (const f4*)subg;
      f4* dst = (f4*)K;
      const int n4 = n >> 2;
      for (int e = tid; e < n4; e += 4 * kWsSolveThreads) {
        f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = e + u * kWsSolveThreads;
          v[u] = src[k < n4 ? k : 0];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (e + u * kWsSolveThreads < n4) dst[e + u * kWsSolveThreads] = v[u];
      }
    } else {
      for (int e = tid; e < n; e += kWsSolveThreads) K[e] = subg[e];
    }
    if (tid < q) {
      s_f[tid] = aux[tid];
      s_a[tid] = aux[a.aux_stride + tid];
      s_y[tid] = aux[2 * a.aux_stride + tid];
      s_idx[tid] = c->idx[par][ib + tid];
      s_line[tid] = c->line[par][ib + tid];
    }
  }
  __syncthreads();
  if (tid == 0) WS_STAMP(3);
  if (wave != 0) return;

  const float INF = __builtin_inff();
  const float C = a.C;
  const float eps_in = fmaxf(a.eps_floor, a.rel_local * 0.5f * (b_lo - b_hi));
  float fu[NS], fl[NS], yr[NS], a0[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int p = lane + 64 * s;
    const bool v = p < q;
    const float fv = v ? s_f[p] : 0.f;
    a0[s] = v ? s_a[p] : 0.f;
    yr[s] = v ? s_y[p] : 1.f;
    fu[s] = v && in_up(a0[s], yr[s], C) ? fv : INF;
    fl[s] = v && in_low(a0[s], yr[s], C) ? -fv : INF;
  }
  int64_t room = a.max_iter - it0;
  if (kMulti) {  // the active blocks share max_iter
    const int pa = c->p_round;
    room = blk < pa ? room / pa + (blk < room % pa ? 1 : 0) : 0;
  }
  // uniform: in an SGPR, so the loop test is one scalar compare
  const int cap = __builtin_amdgcn_readfirstlane((int)(room < (int64_t)a.inner_max ? room : (int64_t)a.inner_max));
  int inner = 0;
  bool bad = false, clipped_any = false;
  while (inner < cap) {
    float mu = fminf(fu[0], fu[1]), ml = fminf(fl[0], fl[1]);
    if constexpr (NS == 3) {
      mu = fminf(mu, fu[2]);
      ml = fminf(ml, fl[2]);
    }
    wave_min2_f32(mu, ml);
    const float bh = mu;
    float bl = -ml;  // first order: b_lo = max f over I_low (also the stop test's)
    const int ph = ws_argpos(fu, mu);
    int pl = -1;
    float kh[NS], kl[NS];
    if constexpr (!kW2) pl = ws_argpos(fl, ml);
    // one exit test: an empty side, the sub-problem's stop test, or NaN
    const bool open = (mu < INF) & (ml < INF) & (bl > bh + 2.0f * eps_in);
    if constexpr (kW2) {
      if (open && ph >= 0) {
        // hi's sub-Gram row first, then the gain of every violating I_low row
        // as a minimum of -gain (INF: not a candidate)
#pragma unroll
        for (int s = 0; s < NS; ++s) kh[s] = K[ph * ldk + (kFull ? lane + 64 * s : min(lane + 64 * s, q - 1))];
        float g[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const float dv = -fl[s] - bh;
          float eta = (1.0f + 1.0f) - 2.0f * kh[s];
          eta = eta >= a.tau ? eta : a.tau;
          g[s] = ((fl[s] < INF) & (dv > 0.f)) ? -(dv * dv) * __builtin_amdgcn_rcpf(eta) : INF;
        }
        float gm = fminf(g[0], g[1]);
        if constexpr (NS == 3) gm = fminf(gm, g[2]);
        float gm2 = gm;
        wave_min2_f32(gm, gm2);
        pl = gm < INF ? ws_argpos(g, gm) : -1;
        if (pl >= 0) {
          const int sl = pl >> 6;
          bl = -readlane_f32(sl == 0 ? fl[0] : (NS == 2 || sl == 1) ? fl[1] : fl[NS - 1], pl & 63);  // f of the chosen lo
        }
      }
    }
    if (!open || (ph | pl) < 0) {
      bad = open;  // a violating pair exists but no position matches it: NaN
      break;
    }
    // every remaining LDS read of the step in one batch: the pair's alphas /
    // labels, the 2 x 2 block K(hi|lo, hi|lo) and the sub-Gram rows
    const float a_hi = s_a[ph], y_hi = s_y[ph], a_lo = s_a[pl], y_lo = s_y[pl];
    const float khl = K[ph * ldk + pl], klh = K[pl * ldk + ph], khh = K[ph * ldk + ph], kll = K[pl * ldk + pl];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int p = kFull ? lane + 64 * s : min(lane + 64 * s, q - 1);
      if constexpr (!kW2) kh[s] = K[ph * ldk + p];
      kl[s] = K[pl * ldk + p];
    }
    bool clipped = false;
    const PairUpdate up = ws_pair_step<kBox>(a_hi, a_lo, y_hi, y_lo, bh, bl, khl, C, a.tau, ph == pl, &clipped);
    if (kMulti && !kBox) clipped_any |= clipped;
    float f_lo_new, f_hi_new;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float dl;
      {
#pragma clang fp contract(off)
        dl = up.c_hi * kh[s] + up.c_lo * kl[s];  // f_apply's delta (device_util.hpp)
        fu[s] = fu[s] + dl;
        fl[s] = fl[s] - dl;  // -(f + delta): exact negation of the same rounding
      }
    }
    {
      // the pair's own new gradients, uniformly: the owners computed exactly
      // these sums (row ph: kh = K(hi,hi), kl = K(lo,hi); row pl: K(hi,lo), K(lo,lo))
#pragma clang fp contract(off)
      f_lo_new = bl + (up.c_hi * khl + up.c_lo * kll);
      f_hi_new = bh + (up.c_hi * khh + up.c_lo * klh);
    }
    ws_place(pl, up.a_lo_new, y_lo, f_lo_new, lane, C, fu, fl);
    ws_place(ph, up.a_hi_new, y_hi, f_hi_new, lane, C, fu, fl);  // hi written last (svmTrainMain.cpp:298-299)
    // lane 0 writes the pair's alphas, the other lanes a private scratch word
    // each (no exec-mask branch in the loop, no bank conflict)
    s_a[lane == 0 ? pl : kWsMax + lane] = up.a_lo_new;
    s_a[lane == 0 ? ph : kWsMax + 64 + lane] = up.a_hi_new;
    ++inner;
  }
  // ---- commit: alphas, the changed rows for the f update, control, status ----
  int n_apply = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int p = lane + 64 * s;
    const float an = p < q ? s_a[p] : 0.f;
    const bool nz = p < q && an != a0[s];
    const uint64_t mk = __ballot(nz);
    const int at = n_apply + __popcll(mk & ((1ull << lane) - 1ull));
    if (nz) {
      const int32_t gi = s_idx[p];
      a.alpha[gi] = an;
      float dc;
      {
#pragma clang fp contract(off)
        dc = (an - a0[s]) * yr[s];
      }
      c->apply_idx[ib + at] = gi;
      c->apply_line[ib + at] = s_line[p];
      c->apply_coef[ib + at] = dc;
      if (kMulti) a.dalpha[gi] = an - a0[s];
    }
    n_apply += __popcll(mk);
  }
  if (lane == 0 && !kMulti) {
    WS_STAMP(4);
    if (a.stamps) a.stamps[(size_t)(c->outer % kStampRing) * 2 * kStampSlots + 5] = (uint64_t)inner;
    c->n_apply = n_apply;
    c->iter = it0 + inner;
    c->outer = c->outer + 1;
    c->done = bad ? kNonFinite : inner == 0 ? kNoPair : (it0 + inner >= a.max_iter ? kMaxIter : kRunning);
    ws_status(a.status, c);
  }
  if (lane == 0 && kMulti) {
    // publish this block's counts; the last block to finish commits the round
    // (threadfence + counter: no workgroup waits for another)
    c->nab[blk] = n_apply;
    c->inb[blk] = inner;
    c->badb[blk] = bad ? 1 : 0;
    c->clipb[blk] = clipped_any ? 1 : 0;
    __threadfence();
    const int prev = atomicAdd(&c->solve_cnt, 1);
    if (prev == a.blocks - 1) {
      __threadfence();
      int tot_a = 0, tot_i = 0, any_bad = 0, any_clip = 0;
      for (int p = 0; p < a.blocks; ++p) {
        tot_a += __hip_atomic_load(&c->nab[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tot_i += __hip_atomic_load(&c->inb[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        any_bad |= __hip_atomic_load(&c->badb[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        any_clip |= __hip_atomic_load(&c->clipb[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      c->solve_cnt = 0;
      // the reference's independent clipping does not keep sum(alpha y) = 0: once
      // a clip broke it, the blocks' combined steps drift it further (measured:
      // adult-shape P = 8 never converges) — one block per round from here on
      WS_STAMP(4);
      if (a.stamps) a.stamps[(size_t)(c->outer % kStampRing) * 2 * kStampSlots + 5] = (uint64_t)tot_i;
      c->n_apply = tot_a;
      c->iter = it0 + tot_i;
      c->outer = c->outer + 1;
      if (any_clip && a.clip_fallback && c->p_act > 1) {
        c->p_act = 1;
        if (c->p1_round == 0) c->p1_round = c->outer;
      }
      c->done = any_bad ? kNonFinite : tot_i == 0 ? kNoPair : (it0 + tot_i >= a.max_iter ? kMaxIter : kRunning);
      ws_status(a.status, c);
    }
  }
}

// The adaptive block count reached 1: the host switches to the one-block round
// kernels at a block boundary (gpu_engines.hip).  Their merge retains the
// previous set from idx[par ^ 1][0 .. q[par ^ 1]) in newest-first order, which
// the multi-block merge kept as the union (uidx, uq): copy it over (at most
// q_max rows, the newest).  One workgroup, stream-ordered between two rounds.
__global__ __launch_bounds__(256) void ws_to_single_kernel(WsArgs a) {
  WsCtrl* c = a.ctrl;
  const int pp = (int)((c->outer + 1) & 1);  // the last round's parity (outer - 1) & 1
  const int q = min(c->uq[pp], a.q_max);
  for (int i = threadIdx.x; i < q; i += blockDim.x) c->idx[pp][i] = c->uidx[pp][i];
  if (threadIdx.x == 0) c->q[pp] = q;
}

// Partitioned X, cache mode: the X rows of this round's cache misses, packed
// for the row GEMM.  Block i < q_max: row i of the pack = X row miss_row[i]
// when this rank owns it, else zeros — the sum all-reduce over ranks then
// leaves every rank holding the exact rows (x + 0 + ... = x); rows past n_miss
// are zeroed too (never read by the GEMM, kept finite).  xsq is global on
// every rank: the packed norms are local.
__global__ __launch_bounds__(256) void ws_pack_rows_kernel(const float* __restrict__ x, int64_t off, int64_t nl,
                                                           int dp, const float* __restrict__ xsq,
                                                           const WsCtrl* __restrict__ c, float* __restrict__ out,
                                                           float* __restrict__ out_sq) {
  const int i = blockIdx.x;
  const int m = c->n_miss;
  const int64_t row = i < m ? (int64_t)c->miss_row[i] : -1;
  const bool own = row >= off && row < off + nl;
  f4* dst = (f4*)(out + (size_t)i * dp);
  const f4* src = (const f4*)(x + (size_t)(own ? row - off : 0) * dp);
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  for (int k = threadIdx.x; k < dp / 4; k += blockDim.x) dst[k] = own ? src[k] : z;
  if (threadIdx.x == 0) out_sq[i] = row >= 0 ? xsq[row] : 0.f;
}

}  // namespace dev

namespace launch {

int ws_pass1_splits(int G) {
  // about one pass-1 workgroup per CU of the 256-CU device: the selection
  // geometry gives a rank of P only G = ceil(60000 / P / 256) groups on the
  // headline (30 at P = 8), and pass 1 is then bound by the few CUs issuing
  // loads — 3,072 changed rows x 7,500 columns: 114 us with 30 workgroups, 38 us
  // with 240; with 60,000 columns 235 workgroups beat 470 / 705 (158 vs 167 /
  // 189 us; profiles/r3_pass1_probe.txt).  Every rank uses the same G, so the
  // same slice count and the same summation order.
  return std::max(1, std::min(kWsMaxPass1Splits, 256 / std::max(1, G)));
}

void ws_geometry(int64_t nl_max, int world, int32_t* G, int32_t* rpt) {
  // every rank the same geometry (sized for the largest shard); the merge reads
  // world * G <= 1024 candidate lists (kWsListsPerThread per merge thread), so
  // up to 8 ranks keep 128-256 selection workgroups each
  const int64_t gmax = std::max<int64_t>(
      1, std::min<int64_t>(kWsMaxGroups, (int64_t)kWsListsPerThread * 256 / std::max(1, world)));
  const int64_t g = std::max<int64_t>(1, std::min<int64_t>(gmax, (nl_max + kWsSelThreads - 1) / kWsSelThreads));
  const int64_t r = (nl_max + g * kWsSelThreads - 1) / (g * kWsSelThreads);
  *G = (int32_t)g;
  *rpt = (int32_t)std::max<int64_t>(1, r);
}

bool ws_supported(int64_t nl_max, int world, int q_max) {
  int32_t G = 0, rpt = 0;
  ws_geometry(nl_max, world, &G, &rpt);
  return q_max >= 2 && q_max <= kWsMax && rpt <= kWsMaxRPT && nl_max < (int64_t)1 << 31 && world <= kWsMaxGroups;
}

template <int MODE>
static void ws_select_mode(const WsArgs& a, hipStream_t s) {
  const dim3 grid(a.G * (MODE == 1 ? std::max(1, a.ks) : 1));
  auto threads = [](int rpt) { return dim3(MODE == 2 ? kWsSelThreads : kWsSelThreads * (rpt <= 4 ? 4 : rpt <= 16 ? 2 : 1)); };
  if (a.rpt <= 1) dev::ws_select_kernel<1, MODE><<<grid, threads(1), 0, s>>>(a);
  else if (a.rpt <= 2) dev::ws_select_kernel<2, MODE><<<grid, threads(2), 0, s>>>(a);
  else if (a.rpt <= 4) dev::ws_select_kernel<4, MODE><<<grid, threads(4), 0, s>>>(a);
  else if (a.rpt <= 8) dev::ws_select_kernel<8, MODE><<<grid, threads(8), 0, s>>>(a);
  else if (a.rpt <= 16) dev::ws_select_kernel<16, MODE><<<grid, threads(16), 0, s>>>(a);
  else dev::ws_select_kernel<32, MODE><<<grid, threads(32), 0, s>>>(a);
  post_launch("ws_select", s);
}

void ws_select(const WsArgs& a, hipStream_t s) {
  if (a.blocks > 1) {
    ws_select_mode<1>(a, s);  // d_f + line-search partials
    ws_select_mode<2>(a, s);  // f += t d_f, candidates
  } else {
    ws_select_mode<0>(a, s);
  }
}

void ws_select_pass(const WsArgs& a, int pass, hipStream_t s) {
  if (pass == 1) ws_select_mode<1>(a, s);
  else ws_select_mode<2>(a, s);
}

void ws_merge_multi(const WsArgs& a, hipStream_t s) {
  DPSVM_CHECK(a.blocks > 1 && a.blocks <= kWsMaxBlocks && a.blocks * a.q_max <= kWsMaxAll && !a.xpeer && a.G_all <= kWsMaxGroups && a.q_max % 2 == 0 &&
                  (!a.cache || ws_cache_multi_supported(a.L, a.blocks, a.q_max)),
              "ws_merge_multi: multi-block rounds need the collectives, <= 256 candidate lists, an even q_max and "
              "(cache mode) L >= 2 P q_max + 4096 lines");
  DPSVM_CHECK(a.sorted != nullptr, "ws_merge_multi: no sort buffer");
  dev::ws_rank_kernel<<<2 * dev::kRankChunks, dev::kRankThreads, 0, s>>>(a);
  post_launch("ws_rank", s);
  dev::ws_merge_multi_kernel<<<1, kWsMergeThreads, 0, s>>>(a);
  post_launch("ws_merge_multi", s);
}

void ws_gather(const WsArgs& a, hipStream_t s) {
  if (a.blocks > 1) {
    dev::ws_gather_multi_kernel<<<dim3(a.blocks * a.q_max), dev::kWsGatherThreads, 0, s>>>(a);
    post_launch("ws_gather_multi", s);
  } else if (a.cache) {
    dev::ws_gather_lines_kernel<<<dim3(a.q_max), dev::kWsGatherThreads, 0, s>>>(a);
    post_launch("ws_gather_lines", s);
  } else {
    dev::ws_gather_kernel<<<dim3(a.q_max), dev::kWsGatherThreads, 0, s>>>(a);
    post_launch("ws_gather", s);
  }
}

void ws_merge(const WsArgs& a, hipStream_t s) {
  dev::ws_merge_kernel<<<1, dev::kWsGatherThreads, 0, s>>>(a);
  post_launch("ws_merge", s);
}

void ws_to_single(const WsArgs& a, hipStream_t s) {
  dev::ws_to_single_kernel<<<1, 256, 0, s>>>(a);
  post_launch("ws_to_single", s);
}

void ws_pack_rows(const float* x, int64_t off, int64_t nl, int dp, const float* xsq, const WsCtrl* ctrl, int q_max,
                  float* out, float* out_sq, hipStream_t s) {
  DPSVM_CHECK(dp % 16 == 0, "ws_pack_rows: dp must be a multiple of 16");
  dev::ws_pack_rows_kernel<<<dim3(q_max), 256, 0, s>>>(x, off, nl, dp, xsq, ctrl, out, out_sq);
  post_launch("ws_pack_rows", s);
}

bool ws_cache_supported(int64_t L, int q_max) { return L >= 2 * (int64_t)q_max + dev::kWsWindow; }

bool ws_cache_multi_supported(int64_t L, int blocks, int q_max) {
  return L >= 2 * (int64_t)blocks * q_max + dev::kWsWindowMulti;
}

void ws_solve(const WsArgs& a, hipStream_t s) {
  const size_t lds = (size_t)a.q_max * a.q_max * sizeof(float);
  const bool box = a.clip == (int)ClipMode::Box, full = a.q_max == kWsMax, multi = a.blocks > 1, w2 = a.wss == 2;
  using Fn = void (*)(WsArgs);
#define WS_SOLVE_FNS(W2)                                                                                         \
  dev::ws_solve_kernel<false, false, false, W2>, dev::ws_solve_kernel<false, true, false, W2>,                  \
      dev::ws_solve_kernel<true, false, false, W2>, dev::ws_solve_kernel<true, true, false, W2>,                \
      dev::ws_solve_kernel<false, false, true, W2>, dev::ws_solve_kernel<false, true, true, W2>,                \
      dev::ws_solve_kernel<true, false, true, W2>, dev::ws_solve_kernel<true, true, true, W2>
  static const Fn fns[16] = {WS_SOLVE_FNS(false), WS_SOLVE_FNS(true)};
#undef WS_SOLVE_FNS
  // two slots per lane when q_max <= 128 (never kFull)
#define WS_SOLVE_FNS2(W2)                                                                                        \
  dev::ws_solve_kernel<false, false, false, W2, 2>, dev::ws_solve_kernel<true, false, false, W2, 2>,            \
      dev::ws_solve_kernel<false, false, true, W2, 2>, dev::ws_solve_kernel<true, false, true, W2, 2>
  static const Fn fns2[8] = {WS_SOLVE_FNS2(false), WS_SOLVE_FNS2(true)};
#undef WS_SOLVE_FNS2
  const int v = (w2 ? 8 : 0) + (multi ? 4 : 0) + (box ? 2 : 0) + (full ? 1 : 0);
  const bool two = a.q_max <= 128;
  const Fn fn = two ? fns2[(w2 ? 4 : 0) + (multi ? 2 : 0) + (box ? 1 : 0)] : fns[v];
  // dynamic LDS above 64 KiB needs the attribute (160 KiB on gfx950)
  static size_t attr[16] = {64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024,
                            64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024};
  static size_t attr2[8] = {64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024, 64 * 1024};
  size_t& at = two ? attr2[(w2 ? 4 : 0) + (multi ? 2 : 0) + (box ? 1 : 0)] : attr[v];
  if (lds > at) {
    HIP_CHECK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    at = lds;
  }
  fn<<<multi ? a.blocks : 1, kWsSolveThreads, lds, s>>>(a);
  post_launch("ws_solve", s);
}

}  // namespace launch
}  // namespace dpsvm
