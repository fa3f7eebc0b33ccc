// Working-set engine, merge and gather: the stop test and the next working
// set from every workgroup's candidate lists (one-block: ws_gather / ws_merge;
// multi-block: ws_rank + ws_merge_multi, the union of P blocks), the cache
// mode's line assignment, and the sub-Gram rows of the set (ws_gather*).
// Round structure and shared helpers: ws_common.hpp.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "ws_common.hpp"
#include "ws_merge.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// Row ra of the q_max-stride sub-Gram from line `line` (K(idx_ra, off + j) at
// line[j]), plus the row's f / alpha / y.  A rank fills only the columns (and
// the f) of rows it owns and zeros the rest, so at world > 1 one sum all-reduce
// assembles the exact matrix (each entry has exactly one owner).  Rows ra >= q
// are zeroed.
// Peer exchange: xr is the row's slot in the receive buffers (block p's row
// ra of a multi-block round: p q_max + ra).
__device__ __forceinline__ void ws_gather_row(const WsArgs& a, WsCtrl* c, const int32_t* s_idx, int q, int ra,
                                              const float* line, int xr) {
  const int tid = threadIdx.x;
  float* dst = a.subg + (size_t)ra * a.q_max;
  if (ra >= q) {
    for (int b = tid; b < a.q_max; b += kWsGatherThreads) dst[b] = 0.f;
    if (tid == 0) a.aux[ra] = 0.f;
    return;
  }
  const int64_t lo = a.off, hi = a.off + a.nl;
  if (a.xpeer != nullptr) {
    // peer exchange: push the owned entries of row ra (+ its f) into row ra of
    // every rank's receive buffer and return — ws_solve polls the rows (push
    // only: no gather workgroup waits for a peer, so ranks sharing a device
    // never park q_max spinning workgroups on it).  alpha / y are global: local aux.
    const int64_t R = c->outer;
    const uint64_t t = xtag((uint32_t)R + 1u);
    const int64_t row = ws_xrow(a, (int)(R & 1), xr);
    const int64_t gi = s_idx[ra];
    for (int col = tid; col <= q; col += kWsGatherThreads) {
      uint64_t v;
      int at;
      if (col < q) {
        const int64_t gj = s_idx[col];
        if (gj < lo || gj >= hi) continue;
        v = t | __float_as_uint(line[gj - lo]);
        at = col;
      } else {  // the row's f, last column
        if (gi < lo || gi >= hi) continue;
        v = t | __float_as_uint(a.f[gi - lo]);
        at = a.q_max;
      }
      for (int p = 0; p < a.world; ++p) xch_store<true>(a.xpeer[p] + row + at, v);
    }
    if (tid == 0) {
      a.aux[a.aux_stride + ra] = a.alpha[gi];
      a.aux[2 * a.aux_stride + ra] = a.y[gi];
    }
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
  __shared__ WsMergeLds L;
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  const bool lead = blockIdx.x == 0 && tid == 0;
  if (lead) WS_STAMP(1);
  const int par = (int)(c->outer & 1);
  int q = 0;
  float b_hi = 0.f, b_lo = 0.f;
  if (!ws_merge(a, c, s_idx, &q, &b_hi, &b_lo, L)) return;
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
  ws_gather_row(a, c, s_idx, q, blockIdx.x, blockIdx.x < q ? a.gram + (int64_t)s_idx[blockIdx.x] * a.ldg : nullptr,
                blockIdx.x);
  if (lead) WS_STAMP(8);
}

// ---------------------------------------------------------------------------
// cache mode, round part 1 — ws_merge (ONE workgroup): the merge, then lines
// for the members: a member's row is cached (slot_of) or takes a victim line.
// Victims come from a window of up to 512 lines after the CLOCK hand, skipping
// lines that hold a member (pinned while the round uses them); all misses are
// assigned at once (one prefix scan), their rows computed next by one GEMM.
// ---------------------------------------------------------------------------
constexpr int kWsWindow = kWsCacheWindow;

__global__ __launch_bounds__(kWsGatherThreads) void ws_merge_kernel(WsArgs a) {
  __shared__ int32_t s_idx[kWsMax];
  __shared__ int32_t s_line[kWsMax];
  __shared__ int32_t s_pin[kWsWindow];
  __shared__ int32_t s_victim[kWsMax];
  __shared__ int s_wsum[4];
  __shared__ WsMergeLds ml;
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  if (tid == 0) WS_STAMP(1);
  const int par = (int)(c->outer & 1);
  int q = 0;
  float b_hi = 0.f, b_lo = 0.f;
  if (!ws_merge(a, c, s_idx, &q, &b_hi, &b_lo, ml)) return;
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
    ws_gather_row(a, c, s_idx, q, ra, nullptr, ra);
    return;
  }
  for (int t = tid; t < q; t += kWsGatherThreads) s_idx[t] = c->idx[par][t];
  __syncthreads();
  ws_gather_row(a, c, s_idx, q, ra, a.gram + (int64_t)c->line[par][ra] * a.ldg, ra);
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

// X exclusive scans of per-thread counts (each < 4) behind ONE barrier: the
// union's slots in scan order — slot[x] = the totals of scans 0 .. x - 1 plus
// this thread's prefix in scan x; scans x >= nact (uniform) are skipped.
// Returns the grand total.  msum: [X][kWsMergeThreads / 64], used once.
template <int X>
__device__ __forceinline__ int multi_scan_merge(const int (&v)[X], int (&slot)[X], int* msum, int nact) {
  constexpr int NW = kWsMergeThreads / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  int pre[X];
#pragma unroll
  for (int x = 0; x < X; ++x) {
    pre[x] = 0;
    if (x < nact) {
      int wt = 0;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const uint64_t m = __ballot((v[x] >> b) & 1);
        pre[x] += __popcll(m & below) << b;
        wt += __popcll(m) << b;
      }
      if (lane == 0) msum[x * NW + wave] = wt;
    }
  }
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int x = 0; x < X; ++x) {
    slot[x] = base;
    if (x < nact) {
      int off = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const int t = msum[x * NW + w];
        off += w < wave ? t : 0;
        tot += t;
      }
      slot[x] = base + off + pre[x];
      base += tot;
    }
  }
  return base;
}

// ONE workgroup: every candidate key of both sides sorted (bitonic, 2048 per
// side, two per thread), the stop test, then the union: up rank r / low rank r
// interleaved (most violating first, a row's first position wins), then the
// newest rows of the previous union.  Union position i goes to block
// ((i / 2) mod P): each block gets up / low pairs, block 0 the global extremes
// (so a round always holds the maximal violating pair and makes progress).
constexpr int kMH = 8192;  // merge hash slots per side (load <= 0.19 at 3,072-row unions, <= 0.38 at 6,144)
constexpr int kWsWindowMulti = 8192;  // cache mode: CLOCK victim window of the multi-block merge
static_assert(kMH == 8192, "11-bit bucket hash");
// keys: row indices (-1 empty) in buckets of four slots read as one 16-B LDS
// word (a bucket fills left to right: no holes, so a free last slot ends a
// search); values: 16-bit ranks (< kWsMaxGroups * kWsCand).  At the 6,144-row
// union's 0.38 load a search is one bucket read; linear probing of single
// slots took a dependent LDS trip per probe.
constexpr int kMHB = kMH / 4;  // buckets per side
typedef int mh_i4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t mh_bucket(int32_t idx) { return ((uint32_t)idx * 2654435761u) >> 21; }
__device__ __forceinline__ void mh_insert(int32_t* keys, uint16_t* vals, int32_t idx, int32_t v) {
  uint32_t b = mh_bucket(idx);
  while (true) {
    const mh_i4 kb = *(const mh_i4*)(keys + 4 * b);
    const int s = kb.x == -1 ? 0 : kb.y == -1 ? 1 : kb.z == -1 ? 2 : kb.w == -1 ? 3 : 4;
    if (s == 4) {
      b = (b + 1) & (kMHB - 1);
      continue;
    }
    if (atomicCAS(keys + 4 * b + s, -1, idx) == -1) {
      vals[4 * b + s] = (uint16_t)v;
      return;
    }
    // another row took that slot first: read the bucket again
  }
}
// N inserts of one thread with every first bucket read, then every claim, in
// flight together (one LDS round trip each instead of two per key in
// sequence); a claim another row won first, or a full first bucket (rare at
// the 0.38 load), takes the one-at-a-time path.  idx < 0: nothing to insert
template <int N>
__device__ __forceinline__ void mh_insert_n(int32_t* keys, uint16_t* vals, const int32_t (&idx)[N],
                                            const int32_t (&v)[N]) {
  uint32_t b[N];
  mh_i4 kb[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    b[j] = mh_bucket(idx[j] < 0 ? 0 : idx[j]);
    if (idx[j] >= 0) kb[j] = *(const mh_i4*)(keys + 4 * b[j]);
  }
  int sl[N];
  bool won[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    sl[j] = kb[j].x == -1 ? 0 : kb[j].y == -1 ? 1 : kb[j].z == -1 ? 2 : kb[j].w == -1 ? 3 : 4;
    won[j] = false;
    if (idx[j] >= 0 && sl[j] < 4) won[j] = atomicCAS(keys + 4 * b[j] + sl[j], -1, idx[j]) == -1;
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (idx[j] < 0) continue;
    if (won[j]) vals[4 * b[j] + sl[j]] = (uint16_t)v[j];
    else mh_insert(keys, vals, idx[j], v[j]);
  }
}

__device__ __forceinline__ int32_t mh_find_from(const int32_t* keys, const uint16_t* vals, int32_t idx, uint32_t b) {
  for (int probe = 0; probe < kMHB; ++probe) {
    const mh_i4 kb = *(const mh_i4*)(keys + 4 * b);
    const int s = kb.x == idx ? 0 : kb.y == idx ? 1 : kb.z == idx ? 2 : kb.w == idx ? 3 : -1;
    if (s >= 0) return (int32_t)vals[4 * b + s];
    if (kb.w == -1) return -1;
    b = (b + 1) & (kMHB - 1);
  }
  return -1;
}
__device__ __forceinline__ int32_t mh_find(const int32_t* keys, const uint16_t* vals, int32_t idx) {
  return mh_find_from(keys, vals, idx, mh_bucket(idx));
}

// N lookups of one thread with every first bucket read in flight together; a
// key not in a full first bucket probes on one at a time.  idx < 0: -1
template <int N>
__device__ __forceinline__ void mh_find_n(const int32_t* keys, const uint16_t* vals, const int32_t (&idx)[N],
                                          int32_t (&out)[N]) {
  uint32_t b[N];
  mh_i4 kb[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    b[j] = mh_bucket(idx[j] < 0 ? 0 : idx[j]);
    if (idx[j] >= 0) kb[j] = *(const mh_i4*)(keys + 4 * b[j]);
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    out[j] = -1;
    if (idx[j] < 0) continue;
    const int32_t k = idx[j];
    const int s = kb[j].x == k ? 0 : kb[j].y == k ? 1 : kb[j].z == k ? 2 : kb[j].w == k ? 3 : -1;
    if (s >= 0) out[j] = (int32_t)vals[4 * b[j] + s];
    else if (kb[j].w != -1) out[j] = mh_find_from(keys, vals, k, (b[j] + 1) & (kMHB - 1));
  }
}

// Multi-block rounds over the peer exchange: every rank's candidate lists
// (pushed by pass 2 of the previous round into this rank's receive buffer) into
// a.cand, the layout the all-gather leaves, so ws_rank reads them as from the
// collective.  A few workgroups spin here instead of ws_rank's 128: ranks
// sharing a device (rehearsals) must leave wave slots for each other's producers.
constexpr int kXCollectThreads = 256;
__global__ __launch_bounds__(kXCollectThreads) void ws_xcollect_cand_kernel(WsArgs a) {
  WsCtrl* c = a.ctrl;
  if (c->done != kRunning) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(15);
  const int e = (int)(blockIdx.x * kXCollectThreads + threadIdx.x);  // (list, side, rank) key
  // keys per side the previous round's selection pushed: ws_ncand by pass 2 of a
  // multi-block round (and the seed), kWsCand1 by a one-block round — also in the
  // one-block rounds of a multi-block engine, whose slots stay kWsCand wide
  const int nk = a.blocks > 1 ? ws_ncand(a.ncand) : kWsCand1;
  bool ok = true;
  if (e < a.G_all * 2 * kWsCand) {
    const int l = e / (2 * kWsCand), side = (e / kWsCand) & 1, r = e % kWsCand;
    if (r < nk) {
      uint64_t g[2];
      ok = ws_poll<2>(a, a.xpeer[a.xrank] + ws_xcand(a, (int)(c->outer & 1), l) + side * (a.xcw / 2) + 2 * r,
                      xtag((uint32_t)c->outer + 1u), g);
      a.cand[e] = ok ? ws_get64(g[0], g[1]) : kKeyNone;
    } else {
      a.cand[e] = kKeyNone;  // not pushed (the one-block merge reads kWsCand1 keys a side)
    }
  }
  if (!ok) ws_comm_fail_thread(a, c);
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(16);
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
constexpr int kRankChunks = kWsMaxGroups * kWsCand / 32;  // 32 keys per workgroup, 16 threads per key
template <int T>
struct RankLds {
  uint64_t k[kWsMaxGroups * kWsCand];
  int real[T / 64];
};
// one rank workgroup's work (the caller checked c->done): T threads rank T /
// 16 keys of one side, 16 threads per key; 2 x NK x 16 / T workgroups
template <int T>
constexpr int rank_chunks() { return kWsMaxGroups * kWsCand * 16 / T; }
template <int T, bool kCoherent = false>
__device__ __forceinline__ void ws_rank_body(const WsArgs& a, RankLds<T>& L) {
  constexpr int NK = kWsMaxGroups * kWsCand, CH = rank_chunks<T>();
  constexpr int KPW = NK / CH, SUB = T / KPW, PAIRS = NK / (2 * SUB);
  static_assert(NK % CH == 0 && T % KPW == 0 && SUB == 16 && NK % (2 * SUB) == 0, "rank geometry");
  constexpr int kRankThreads = T;
  uint64_t* const s_k = L.k;
  int* const s_real = L.real;
  const WsCtrl* c = a.ctrl;
  const int side = blockIdx.x / CH, chunk = blockIdx.x % CH, tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) WS_STAMP(21);
  const int G = a.G_all;
  int real = 0;
  {
    // all NK / threads loads in flight before the LDS stores (a rolled loop
    // paid one L2 round trip per key: ~5 of the kernel's 8 us)
    constexpr int PER = NK / kRankThreads;
    static_assert(NK % kRankThreads == 0, "rank load geometry");
    uint64_t kk[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = tid + j * kRankThreads, l = e / kWsCand, r = e % kWsCand;
      kk[j] = l < G ? a.cand[(size_t)l * 2 * kWsCand + side * kWsCand + r] : kKeyNone;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      s_k[tid + j * kRankThreads] = kk[j];
      real += kk[j] != kKeyNone ? 1 : 0;
    }
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
  // coherent (the fused rank + merge): agent-scope (sc1) stores, read by
  // another workgroup of the same launch with sc1 loads — no L2 write-back
  auto put = [&](int i, uint64_t v) {
    if constexpr (kCoherent) __hip_atomic_store(out + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else out[i] = v;
  };
  if (sub == 0 && k != kKeyNone) put(cnt, k);
  if (tid < KPW && chunk * KPW + tid >= n_real) put(chunk * KPW + tid, kKeyNone);
}

__global__ __launch_bounds__(kRankThreads) void ws_rank_kernel(WsArgs a) {
  static_assert(rank_chunks<kRankThreads>() == kRankChunks, "rank grid");
  __shared__ RankLds<kRankThreads> L;
  if (a.ctrl->done != kRunning) return;
  ws_rank_body<kRankThreads>(a, L);
}

struct MergeLds {
  __attribute__((aligned(16))) int32_t hk[2][kMH];  // [side] hash keys (row indices), 4-slot buckets
  uint16_t hv[2][kMH];                               // [side] their ranks
  int32_t keep[kWsMaxAll + 2];
  int32_t idx[kWsMaxAll];
  int wsum[kWsMergeThreads / 64];
  int msum[(kWsMaxGroups * kWsCand / kWsMergeThreads) * (kWsMergeThreads / 64)];
};
// the merge on one workgroup (the caller checked c->done).  coherent: the
// ranked keys were written by other workgroups of the same launch (the fused
// rank + merge): read them with agent-scope loads, not through this XCD's L2
template <bool kCoherent>
__device__ __forceinline__ void ws_merge_multi_body(const WsArgs& a, MergeLds& L) {
  constexpr int T = kWsMergeThreads;
  constexpr int NK = kWsMaxGroups * kWsCand;  // keys per side
  constexpr int X = NK / T;                   // keys per thread and side: elements tid + x T
  constexpr int U = kWsMaxAll / T;            // previous-union rows per thread
  static_assert(NK % T == 0 && kWsMaxAll % T == 0 && U <= 7, "previous union: <= 7 rows per thread (3-bit scans)");
  static_assert(kMH == kWsWindowMulti && kWsWindowMulti == 8 * T && NK <= 65536,
                "cache mode: the CLOCK window's pins alias the low side's key table; 16-bit ranks");
  auto& s_hk = L.hk;
  auto& s_hv = L.hv;
  int32_t* const s_keep = L.keep;
  int32_t* const s_idx = L.idx;
  int* const s_wsum = L.wsum;
  int* const s_msum = L.msum;
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  const bool lead = tid == 0;
  if (lead) WS_STAMP(1);
  const int par = (int)(c->outer & 1);
  const int P = max(1, min(c->p_act, a.blocks)), Qmax = P * a.q_max;
  const int q_prev = c->uq[par ^ 1];
  const int want = q_prev == 0 ? Qmax : min(P * a.n_new, Qmax);
  // the previous union, newest first: thread t holds rows U t .. U t + U - 1
  int32_t pidx[U];
#pragma unroll
  for (int h = 0; h < U; ++h) pidx[h] = U * tid + h < q_prev ? c->uidx[par ^ 1][U * tid + h] : -1;
  // keys e = tid + x T of each side, in ascending order (ws_rank)
  uint64_t v[2][X];  // [side][element]
  auto ld_sorted = [&](int i) -> uint64_t {
    if constexpr (kCoherent) return __hip_atomic_load(a.sorted + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return a.sorted[i];
  };
#pragma unroll
  for (int x = 0; x < X; ++x) {
    v[0][x] = ld_sorted(tid + x * T);
    v[1][x] = ld_sorted(NK + tid + x * T);
  }
  const uint64_t gu = ld_sorted(0), gl = ld_sorted(NK);  // each side's smallest key
  for (int t = tid; t < 2 * kMH; t += T) (&s_hk[0][0])[t] = -1;
  if (lead) WS_STAMP(20);
  __syncthreads();
  if (lead) WS_STAMP(11);
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
  int32_t* hk_u = s_hk[0];
  uint16_t* hv_u = s_hv[0];
  int32_t* hk_l = s_hk[1];
  uint16_t* hv_l = s_hv[1];
  int32_t* const s_line = s_hk[0] + kMH / 2;  // cache mode, once the tables are dead: the union's lines
  const int half = (want + 1) / 2;  // <= kWsMaxAll / 2 ranks per side
  uint64_t ku[X], kl[X];
  int32_t iu[X], il[X], er[X];  // the keys' rows (-1: none), their ranks
#pragma unroll
  for (int x = 0; x < X; ++x) {
    const int e = tid + x * T;
    ku[x] = e < half ? v[0][x] : kKeyNone;
    kl[x] = e < half ? v[1][x] : kKeyNone;
    iu[x] = ku[x] != kKeyNone ? (int32_t)key_index(ku[x]) : -1;
    il[x] = kl[x] != kKeyNone ? (int32_t)key_index(kl[x]) : -1;
    er[x] = e;
  }
  mh_insert_n<X>(hk_u, hv_u, iu, er);
  mh_insert_n<X>(hk_l, hv_l, il, er);
  __syncthreads();
  if (lead) WS_STAMP(12);
  // rank e keeps its up row unless the low side has it at a smaller rank, its
  // low row unless the up side has it at a rank <= e (the up copy comes first)
  bool kpu[X], kpl[X];
  {
    int32_t rl[X], ru[X];
    mh_find_n<X>(hk_l, hv_l, iu, rl);
    mh_find_n<X>(hk_u, hv_u, il, ru);
#pragma unroll
    for (int x = 0; x < X; ++x) {
      const int e = tid + x * T;
      kpu[x] = iu[x] >= 0 && !(rl[x] >= 0 && rl[x] < e);
      kpl[x] = il[x] >= 0 && !(ru[x] >= 0 && ru[x] <= e);
    }
  }
  // union order: ranks 0 .. T - 1 (element 0 of threads in order), then ranks
  // T .. 2 T - 1 (element 1), ...: one scan per element row that holds ranks
  // below half, all behind one barrier
  int cnt[X], slot[X];
#pragma unroll
  for (int x = 0; x < X; ++x) cnt[x] = (int)kpu[x] + (int)kpl[x];
  const int kept = multi_scan_merge<X>(cnt, slot, s_msum, min(X, (half + T - 1) / T));
  const int n_chosen = min(kept, want);
#pragma unroll
  for (int x = 0; x < X; ++x) {
    const int e = tid + x * T;
    if (e < half) {
      const int su = slot[x], sl = su + (int)kpu[x];
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
  for (int h = 0; h < U; ++h) pk[h] = false;
  if (n_chosen < Qmax) {  // uniform
    int32_t ru[U], rl[U];
    mh_find_n<U>(hk_u, hv_u, pidx, ru);
    mh_find_n<U>(hk_l, hv_l, pidx, rl);
#pragma unroll
    for (int h = 0; h < U; ++h)
      pk[h] = pidx[h] >= 0 && !((ru[h] >= 0 && s_keep[2 * ru[h]] >= 0) || (rl[h] >= 0 && s_keep[2 * rl[h] + 1] >= 0));
  }
#pragma unroll
  for (int h = 0; h < U; ++h) npk += (int)pk[h];
  int ptotal = 0;
  if (n_chosen < Qmax) {  // uniform
    int at = n_chosen + block_scan_merge<3>(npk, s_wsum, &ptotal);
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
    // the hash tables are dead: the pins take the low side's key table (kMH
    // words), victims and lines halves of the up side's (launch: Qmax <= kMH / 2)
    int32_t* s_pin = s_hk[1];
    int32_t* s_victim = s_hk[0];
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
      mrank[h] = n_miss;
      if (h * T < Q) {  // uniform
        const bool mh = tid + h * T < Q && ln[h] < 0;
        int tot = 0;
        mrank[h] = n_miss + block_scan_merge<1>((int)mh, s_wsum, &tot);
        n_miss += tot;
      }
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
  // union position u -> block (u / 2) mod P, row 2 ((u / 2) / P) + (u & 1) of it
  // (shifts for the power-of-two block counts the engine uses; integer
  // division by a runtime P costs ~40 instructions)
  const bool pow2 = (P & (P - 1)) == 0;
  const int lg = pow2 ? __ffs(P) - 1 : 0;
  for (int u = tid; u < Q; u += T) {
    const int32_t row = s_idx[u];
    c->uidx[par][u] = row;
    const int pi = u >> 1;
    const int b = pow2 ? pi & (P - 1) : pi % P, la = 2 * (pow2 ? pi >> lg : pi / P) + (u & 1);
    c->idx[par][b * a.q_max + la] = row;
    c->line[par][b * a.q_max + la] = a.cache ? s_line[u] : row;  // dense: line i is row i
  }
  if (tid < a.blocks) {
    // rows per block from the layout: block b holds pairs b, b + P, ... of the
    // NP = ceil(Q / 2) pairs; the last pair is one row when Q is odd
    const int NP = (Q + 1) >> 1, b = tid;
    const int cnt = b < P && b < NP ? (NP - 1 - b) / P + 1 : 0;
    const int last = b + P * (cnt - 1);
    c->qb[par][b] = cnt == 0 ? 0 : 2 * (cnt - 1) + ((last == NP - 1 && (Q & 1)) ? 1 : 2);  // inactive blocks: 0 rows
  }
  if (lead) {
    c->uq[par] = Q;
    c->q[par] = Q;
    c->p_round = P;
    c->b_hi = b_hi;
    c->b_lo = b_lo;
    WS_STAMP(2);
  }
}

__global__ __launch_bounds__(kWsMergeThreads) void ws_merge_multi_kernel(WsArgs a) {
  __shared__ MergeLds L;
  if (a.ctrl->done != kRunning) {
    if (threadIdx.x == 0) a.ctrl->n_apply = 0;  // applied by the last ws_select already
    return;
  }
  ws_merge_multi_body<false>(a, L);
}

// rank + merge in one launch: the rank workgroups publish their keys with
// agent-scope (sc1) stores, every storing wave waits for them, then one lane a
// workgroup takes a ticket (agent-scope add); the workgroup whose add comes
// last runs the merge, reading the keys with sc1 loads — the hand-off form of
// MI355X_MICROARCH.md that needs no L2 write-back or invalidate (a
// __threadfence in each of the 128 workgroups cost ~30 us a round, measured)
// — one launch gap and its dispatch less per round.
// LDS: the merge's tables, the rank's key copy aliased onto them; the merge's
// workgroup shape (1,024 threads: 2 x 64 rank workgroups of 64 keys).
__global__ __launch_bounds__(kWsMergeThreads) void ws_rank_merge_kernel(WsArgs a) {
  __shared__ union {
    RankLds<kWsMergeThreads> r;
    MergeLds m;
  } L;
  __shared__ int s_last;
  WsCtrl* c = a.ctrl;
  if (c->done != kRunning) {
    if (blockIdx.x == 0 && threadIdx.x == 0) c->n_apply = 0;  // (the merge's early exit)
    return;
  }
  ws_rank_body<kWsMergeThreads, true>(a, L.r);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores done
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(&c->rank_cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                     (int)gridDim.x - 1 ? 1 : 0;
  __syncthreads();
  if (!s_last) return;  // uniform
  if (threadIdx.x == 0) c->rank_cnt = 0;  // the next round's tickets (a later launch)
  ws_merge_multi_body<true>(a, L.m);
}


// P x q_max workgroups: workgroup p q_max + a gathers row a of block p's
// sub-Gram (block p's columns) and the row's f / alpha / y
__global__ __launch_bounds__(kWsGatherThreads) void ws_gather_multi_kernel(WsArgs a) {
  __shared__ int32_t s_idx[kWsMax];
  WsCtrl* c = a.ctrl;
  if (c->done != kRunning) return;
  const int tid = threadIdx.x;
  if (tid == 0 && blockIdx.x == 0) WS_STAMP(9);  // after ws-cache's miss-row GEMM (stamps 2 -> 9)
  const int par = (int)(c->outer & 1);
  const int p = (int)blockIdx.x / a.q_max, ra = (int)blockIdx.x % a.q_max;
  const int q = c->qb[par][p];
  WsArgs b = a;
  b.subg = a.subg + (size_t)p * a.q_max * a.q_max;
  b.aux = a.aux + (size_t)p * kWsMax;  // f / alpha / y of block p at stride aux_stride
  if (a.xpeer != nullptr && ra >= q) return;  // peer exchange: ws_solve zero-fills rows past q
  if (ra >= q) {
    ws_gather_row(b, c, s_idx, q, ra, nullptr, p * a.q_max + ra);
    return;
  }
  for (int t = tid; t < q; t += kWsGatherThreads) s_idx[t] = c->idx[par][p * a.q_max + t];
  __syncthreads();
  // the row's line (dense: the resident Gram's row itself)
  const int64_t line = a.cache ? (int64_t)c->line[par][p * a.q_max + ra] : (int64_t)s_idx[ra];
  ws_gather_row(b, c, s_idx, q, ra, a.gram + line * a.ldg, p * a.q_max + ra);
  if (tid == 0 && blockIdx.x == 0) WS_STAMP(8);
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

void ws_xcollect_cand(const WsArgs& a, hipStream_t s) {
  const int keys = a.G_all * 2 * kWsCand;
  dev::ws_xcollect_cand_kernel<<<dim3((unsigned)((keys + dev::kXCollectThreads - 1) / dev::kXCollectThreads)),
                                 dev::kXCollectThreads, 0, s>>>(a);
  post_launch("ws_xcollect_cand", s);
}

void ws_merge_multi(const WsArgs& a, hipStream_t s) {
  DPSVM_CHECK(a.blocks > 1 && a.blocks <= kWsMaxBlocks && a.blocks * a.q_max <= kWsMaxAll && a.G_all <= kWsMaxGroups && a.q_max % 2 == 0 &&
                  (!a.cache || (ws_cache_multi_supported(a.L, a.blocks, a.q_max) && a.blocks * a.q_max <= dev::kMH / 2)),
              "ws_merge_multi: multi-block rounds need <= 256 candidate lists, an even q_max and "
              "(cache mode) <= 4096 union rows and L >= 2 P q_max + 4096 lines");
  DPSVM_CHECK(a.sorted != nullptr, "ws_merge_multi: no sort buffer");
  DPSVM_CHECK(!a.xpeer || a.xcw >= 4 * kWsCand, "ws_merge_multi: peer exchange slots too narrow");
  static const bool split = [] {  // A/B: DPSVM_WS_RANK_MERGE=split, the two launches of round 5
    const char* e = std::getenv("DPSVM_WS_RANK_MERGE");
    return e && std::string(e) == "split";
  }();
  if (split) {
    dev::ws_rank_kernel<<<2 * dev::kRankChunks, dev::kRankThreads, 0, s>>>(a);
    post_launch("ws_rank", s);
    dev::ws_merge_multi_kernel<<<1, kWsMergeThreads, 0, s>>>(a);
    post_launch("ws_merge_multi", s);
  } else {
    dev::ws_rank_merge_kernel<<<2 * dev::rank_chunks<kWsMergeThreads>(), kWsMergeThreads, 0, s>>>(a);
    post_launch("ws_rank_merge", s);
  }
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

bool ws_cache_supported(int64_t L, int q_max) { return L >= ws_cache_min_lines(q_max); }

bool ws_cache_multi_supported(int64_t L, int blocks, int q_max) {
  return L >= 2 * (int64_t)blocks * q_max + dev::kWsWindowMulti;
}

}  // namespace launch
}  // namespace dpsvm
