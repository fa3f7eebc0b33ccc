// Fused SMO iteration for the kernel-row-cache mode (replicated X): ONE launch
// per iteration, like the dense smo_fused, but the kernel rows come from a
// CLOCK-managed cache of lines that is filled inside the same launch.
//
// Kernel t (every workgroup, redundantly where noted):
//   1. pair from the previous launch's keys (every wave), eta + alpha update;
//   2. wave 0 decides the cache actions for this iteration from the cache
//      state at launch start corrected by the previous launch's pending-commit
//      record (slot lookups for the two rows, speculative rows from the
//      workgroup winners, a CLOCK victim scan, host-tier fetch/spill choices)
//      — identical in every workgroup, so no inter-workgroup communication;
//   3. every workgroup fills ITS OWN rows of the newly assigned lines: spill the
//      victims' old segments to the pinned host tier, fetch host-tier hits, and
//      the X pass for computed rows (fp32 MFMA 16x16x4, query vectors in LDS);
//      i.e. the reference's cublasSgemv per miss (svmTrain.cu:212-249) becomes a
//      slice of one distributed X pass inside the iteration kernel;
//   4. f update from the two lines, classification, keys for iteration t+1;
//   5. the last workgroup (fewest rows) commits the previous record (alphas +
//      cache metadata) and publishes this iteration's record.
// Readers never depend on an entry that the committer writes in the same
// launch: they apply the previous record as a correction instead.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "plan_util.hpp"
#include "xpass.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

typedef unsigned long long u64x2l __attribute__((ext_vector_type(2)));


// ---- state as of the previous launch = memory + pending record ----
// The record's per-line arrays are staged in LDS (broadcast reads) and every
// lookup is branch-free with the memory load issued first: lookups sit on the
// serial critical path of every iteration.  Keys and evicted rows of one
// record are disjoint, lines are distinct, so at most one entry matches.
struct alignas(16) RecLds {
  int key[kNQ], old[kNQ], line[kNQ], hline[kNQ], hold[kNQ];
};

typedef int i4 __attribute__((ext_vector_type(4)));

// Lookups read the staged arrays as unconditional 16-B vectors (loop-invariant,
// hoisted by the compiler) and mask entries >= n with selects: no branch ever
// waits on an LDS round trip inside the loop.
struct View {
  const SmoArgs& a;
  const RecLds& r;
  int n, hit0, hit1, hand0, span;
  // *_fix(x, v): v = the memory value for x, corrected by the pending record
  __device__ int slot_fix(int k, int v) const {
#pragma unroll
    for (int q4 = 0; q4 < kNQ; q4 += 4) {
      const i4 kk = *(const i4*)&r.key[q4], oo = *(const i4*)&r.old[q4], ll = *(const i4*)&r.line[q4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bool in = q4 + c < n;
        v = (in && kk[c] == k) ? ll[c] : v;
        v = (in && oo[c] == k) ? -1 : v;
      }
    }
    return v;
  }
  __device__ int key_fix(int l, int v) const {
#pragma unroll
    for (int q4 = 0; q4 < kNQ; q4 += 4) {
      const i4 kk = *(const i4*)&r.key[q4], ll = *(const i4*)&r.line[q4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v = (q4 + c < n && ll[c] == l) ? kk[c] : v;
    }
    return v;
  }
  __device__ int ref_fix(int l, int v) const {
    if (span > 0) {
      int off = l - hand0;
      if (off < 0) off += a.L;
      if (off < span) v = 0;  // scanned: second chance consumed
    }
    if (l == hit0 || l == hit1) v = 1;
#pragma unroll
    for (int q4 = 0; q4 < kNQ; q4 += 4) {
      const i4 ll = *(const i4*)&r.line[q4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v = (q4 + c < n && ll[c] == l) ? 1 : v;
    }
    return v;
  }
  __device__ int hslot_fix(int k, int v) const {
#pragma unroll
    for (int q4 = 0; q4 < kNQ; q4 += 4) {
      const i4 hl = *(const i4*)&r.hline[q4], oo = *(const i4*)&r.old[q4], ho = *(const i4*)&r.hold[q4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bool in = q4 + c < n && hl[c] >= 0;
        v = (in && oo[c] == k) ? hl[c] : v;
        v = (in && ho[c] == k) ? -1 : v;
      }
    }
    return v;
  }
  __device__ int hkey_fix(int h, int v) const {
#pragma unroll
    for (int q4 = 0; q4 < kNQ; q4 += 4) {
      const i4 hl = *(const i4*)&r.hline[q4], oo = *(const i4*)&r.old[q4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v = (q4 + c < n && hl[c] == h) ? oo[c] : v;
    }
    return v;
  }
  __device__ int hslot(int k) const { return a.H == 0 ? -1 : hslot_fix(k, a.hslot_of[k]); }
  __device__ int hkey(int h) const { return hkey_fix(h, a.hkey_of[h]); }
};

// decisions shared by all waves of a workgroup (LDS)
struct Plan {
  int n_new, n_compute, n_fetch, n_spill, n_miss, n_need;
  int line_hi, line_lo, hit_hi, hit_lo, need_hi, miss_hi;
  int hand0, span, hand, hhand;
  int line[kNQ], key[kNQ], old[kNQ], op[kNQ], hsrc[kNQ], hline[kNQ], hold[kNQ];
};

__device__ __forceinline__ void publish_status_lru(SmoStatus* st, const FusedCacheRec& o) {
  if (!st) return;
  st->iter = o.iter;
  st->done = o.done;
  st->b_hi = o.b_hi;
  st->b_lo = o.b_lo;
  st->hits = o.hits;
  st->misses = o.misses;
  st->rows_computed = o.rows_computed;
  st->x_passes = o.x_passes;
  st->spec_rows = o.spec_rows;
  st->host_hits = o.host_hits;
  st->spills = o.spills;
  __atomic_store_n(&st->seq, o.iter, __ATOMIC_RELEASE);
}

// Apply the previous record to memory (alphas + cache metadata) with threads
// ct = 0..nt-1 (nt >= 32) of one workgroup, in parallel and without a barrier:
// scanned window bits are written once with their final value (1 for new /
// hit lines).  Readers never need the result in this launch (View).
__device__ void commit_record(const SmoArgs& a, const FusedCacheRec& r, const RecLds& rl, int ct, int nt) {
  const int n = r.n_new, h0 = r.hit_line[0], h1 = r.hit_line[1];
  if (ct == 0 && r.i_hi >= 0) {
    a.alpha[r.i_lo] = r.a_lo;
    a.alpha[r.i_hi] = r.a_hi;
  }
  for (int i = ct; i < r.span; i += nt) {
    const int ll = r.hand0 + i;  // span <= min(1024, L)
    const int l = ll >= a.L ? ll - a.L : ll;
    bool keep = l == h0 || l == h1;
#pragma unroll
    for (int q4 = 0; q4 < kNQ; q4 += 4) {
      const i4 ll = *(const i4*)&rl.line[q4];
#pragma unroll
      for (int c = 0; c < 4; ++c) keep |= q4 + c < n && ll[c] == l;
    }
    a.ref[l] = keep ? 1 : 0;
  }
  auto outside = [&](int l) {  // set bits of lines the window loop does not touch
    int off = l - r.hand0;
    if (off < 0) off += a.L;
    return off >= r.span;
  };
  if (ct == 1 || ct == 2) {
    const int l = ct == 1 ? h0 : h1;
    if (l >= 0 && outside(l)) a.ref[l] = 1;
  }
  if (ct >= 16 && ct < 16 + n) {
    const int q = ct - 16;
    const int l = rl.line[q], k = rl.key[q], o = rl.old[q];
    if (o >= 0) a.slot_of[o] = -1;
    a.key_of[l] = k;
    a.slot_of[k] = l;
    if (outside(l)) a.ref[l] = 1;
    const int hl = rl.hline[q];
    if (hl >= 0) {
      const int ho = rl.hold[q];
      if (ho >= 0) a.hslot_of[ho] = -1;
      a.hkey_of[hl] = o;
      a.hslot_of[o] = hl;
    }
  }
}

__global__ __launch_bounds__(kFusedThreads) void smo_fused_lru_kernel(SmoArgs a,
                                                                      const uint64_t* __restrict__ p_in,
                                                                      uint64_t* __restrict__ p_out,
                                                                      const FusedCacheRec* __restrict__ r_in,
                                                                      FusedCacheRec* __restrict__ r_out) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];  // [kNQ][dp+4] query vectors
  __shared__ uint64_t kscr[8];
  __shared__ int kscan[kFusedThreads / 64];
  __shared__ Plan pl;
  __shared__ RecLds rl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool committer = blockIdx.x == a.fused_G - 1;  // fewest rows
  const int64_t row0 = (int64_t)blockIdx.x * a.fused_rows;
  const int64_t row_end = min((int64_t)a.nl, row0 + (int64_t)a.fused_rows);
  const int64_t j0 = row0 + tid;
  const FusedCacheRec& rin = *r_in;  // read through the scalar cache (never written this launch)
  if (tid < 5 * kNQ) {
    const int arr = tid / kNQ, q = tid - arr * kNQ;
    const int32_t* src = arr == 0 ? rin.key : arr == 1 ? rin.old : arr == 2 ? rin.line : arr == 3 ? rin.hline : rin.hold;
    int* dst = arr == 0 ? rl.key : arr == 1 ? rl.old : arr == 2 ? rl.line : arr == 3 ? rl.hline : rl.hold;
    dst[q] = src[q];
  }
  const View view{a, rl, rin.n_new, rin.hit_line[0], rin.hit_line[1], rin.hand0, rin.span};
  // diagnostics only (a.stamps == nullptr in normal runs): 0 entry, 1 alpha
  // update, 8 need rows, 9/10 speculation, 2 rows chosen, 3 victims, 4 plan
  // done, 5 lines filled, 6 commit, 7 end
  const bool stamping = a.stamps != nullptr && tid == 0 && (blockIdx.x == 0 || committer);
  const uint64_t ts_entry = stamping ? __builtin_amdgcn_s_memrealtime() : 0;
  const int it_st = rin.iter;
  // stamps collect in LDS and are flushed once at the end (a global store
  // mid-kernel would add its completion wait to the next vmcnt(0))
  __shared__ uint64_t st_lds[kStampSlots];
  auto stamp = [&](int slot) {
    if (stamping) {
      if (slot == 0)
        for (int i = 1; i < kStampSlots; ++i) st_lds[i] = 0;
      st_lds[slot] = slot == 0 ? ts_entry : __builtin_amdgcn_s_memrealtime();
      if (slot == 7) {
        uint64_t* dst = a.stamps + ((size_t)(it_st % kStampRing) * 2 + (blockIdx.x == 0 ? 0 : 1)) * kStampSlots;
        for (int i = 0; i < kStampSlots; ++i) dst[i] = st_lds[i];
      }
    }
  };

  // ---- 0. everything that does not depend on this iteration's pair, in flight
  //         together: the previous launch's keys (pair + speculation
  //         candidates), the CLOCK window's bits and owners, candidate slots ----
  const u64x2l* pk = (const u64x2l*)p_in;
  uint64_t cand[8];  // [2i] up side, [2i+1] low side of workgroup lane + 64 i (fused_G <= 256)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = lane + 64 * i;
    cand[2 * i] = kKeyNone;
    cand[2 * i + 1] = kKeyNone;
    if (b < a.fused_G) {
      const u64x2l v = pk[b];
      cand[2 * i] = v.x;
      cand[2 * i + 1] = v.y;
    }
  }
  const int W = min(1024, a.L), hand = rin.hand;
  int wp[4], wref[4], wkey[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pos = 4 * tid + j;
    const int pp = hand + pos;  // hand < L; only pos < W <= L is used
    wp[j] = pp >= a.L ? pp - a.L : pp;
    wref[j] = 1;
    wkey[j] = -1;
    if (pos < W) {
      wref[j] = a.ref[wp[j]];
      wkey[j] = a.key_of[wp[j]];
    }
  }
  int cidx[8], cmem[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    cidx[i] = cand[i] != kKeyNone ? (int)key_index(cand[i]) : 0;
    cmem[i] = wave == 0 ? a.slot_of[cidx[i]] : -1;
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the prefetches here (the scheduler sinks loads to their uses)
  uint64_t kh = kKeyNone, kl = kKeyNone;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    kh = cand[2 * i] < kh ? cand[2 * i] : kh;
    kl = cand[2 * i + 1] < kl ? cand[2 * i + 1] : kl;
  }
  __syncthreads();  // staged record visible
  if (rin.done != kRunning) {
    if (committer) {
      commit_record(a, rin, rl, tid, kFusedThreads);
      if (tid == 0) {
        FusedCacheRec o = rin;
        o.i_hi = o.i_lo = -1;
        o.n_new = 0;
        o.span = 0;
        o.hit_line[0] = o.hit_line[1] = -1;
        *r_out = o;
        publish_status_lru(a.status, o);
      }
    }
    return;
  }

  // ---- 1. pair (every wave), alpha update ----
  kh = wave_min_u64(kh);
  kl = wave_min_u64(kl);
  const bool nopair = kh == kKeyNone || kl == kKeyNone;
  const int i_hi = nopair ? 0 : (int)key_index(kh), i_lo = nopair ? 0 : (int)key_index(kl);
  const float b_hi = key_value(kh), b_lo = -key_value(kl);
  // the f update may need either row: their slots load with the sample rows
  const int s_hi = a.slot_of[i_hi], s_lo = a.slot_of[i_lo];
  __builtin_amdgcn_sched_barrier(0);
  int done = kRunning;
  float c_hi = 0.f, c_lo = 0.f, a_hi_new = 0.f, a_lo_new = 0.f;
  const int iter = rin.iter + 1;
  if (nopair) {
    done = kNoPair;
  } else {
    const float* xh = a.x + ((int64_t)i_hi - a.x_row0) * a.dp;
    const float* xl = a.x + ((int64_t)i_lo - a.x_row0) * a.dp;
    const float y_hi = a.y[i_hi], y_lo = a.y[i_lo];
    const float al_hi = a.alpha[i_hi], al_lo = a.alpha[i_lo];
    const float dist2 = wave_dist2(xh, xl, a.dp, lane);
    const float a_hi_old = i_hi == rin.i_hi ? rin.a_hi : (i_hi == rin.i_lo ? rin.a_lo : al_hi);
    const float a_lo_old = i_lo == rin.i_hi ? rin.a_hi : (i_lo == rin.i_lo ? rin.a_lo : al_lo);
    a_hi_new = a_hi_old;
    a_lo_new = a_lo_old;
    if (!isfinite(b_hi) || !isfinite(b_lo)) {
      done = kNonFinite;
    } else {
      const float k_hl = expf(-a.gamma * dist2);
      const PairUpdate u =
          pair_update(a_hi_old, a_lo_old, y_hi, y_lo, b_hi, b_lo, k_hl, a.C, a.tau, a.clip, i_hi == i_lo);
      a_hi_new = u.a_hi_new;
      a_lo_new = u.a_lo_new;
      c_hi = u.c_hi;
      c_lo = u.c_lo;
      if (!gap_open(b_hi, b_lo, a.eps)) done = kConverged;
      else if (iter >= a.max_iter) done = kMaxIter;
    }
  }
  stamp(0);
  stamp(1);

  // ---- 2. cache plan (identical in every workgroup) ----
  // 2a. rows the f update needs and their lines (uniform), then speculative
  //     rows (wave 0): the best uncached workgroup winners, t per side by a
  //     ballot radix select.  Meanwhile waves 1-3 of the committing workgroup
  //     apply the previous record.
  const int need_hi = c_hi != 0.f ? i_hi : -1;
  const int need_lo = (c_lo != 0.f && !(i_lo == i_hi && c_hi != 0.f)) ? i_lo : -1;
  const int hit_hi = need_hi >= 0 ? view.slot_fix(need_hi, s_hi) : -1;
  const int hit_lo = need_lo >= 0 ? view.slot_fix(need_lo, s_lo) : -1;
  const int miss_hi = need_hi >= 0 && hit_hi < 0, miss_lo = need_lo >= 0 && hit_lo < 0;
  const int n_miss = miss_hi + miss_lo;
  stamp(8);
  const int budget = n_miss > 0 ? min(min(a.spec, kNQ - n_miss), max(0, a.L / 2 - n_miss)) : 0;
  if (tid == 0) {
    pl.key[0] = miss_hi ? need_hi : need_lo;  // misses first (hi before lo)
    pl.key[1] = need_lo;
    pl.n_new = n_miss;
    pl.n_miss = n_miss;
    pl.n_need = (need_hi >= 0) + (need_lo >= 0);
    pl.hit_hi = hit_hi;
    pl.hit_lo = hit_lo;
    pl.need_hi = need_hi;
    pl.miss_hi = miss_hi;
    pl.span = 0;
  }
  if (committer && wave > 0) commit_record(a, rin, rl, tid - 64, kFusedThreads - 64);
  if (budget > 0 && wave == 0) {  // uniform
    uint64_t ch = kKeyNone, cl = kKeyNone;  // lane's best uncached candidate per side
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = cidx[i];
      const bool ok = cand[i] != kKeyNone && idx != i_hi && idx != i_lo && view.slot_fix(idx, cmem[i]) < 0;
      if (ok && (i & 1) == 0) ch = cand[i] < ch ? cand[i] : ch;
      if (ok && (i & 1) == 1) cl = cand[i] < cl ? cand[i] : cl;
    }
    stamp(9);
    const uint64_t valid_h = __ballot(ch != kKeyNone), valid_l = __ballot(cl != kKeyNone);
    const int vh = __popcll(valid_h), vl = __popcll(valid_l);
    int take_h = min(vh, (budget + 1) / 2);
    const int take_l = min(vl, budget - take_h);
    take_h = min(vh, budget - take_l);  // an exhausted low side leaves room
    const uint64_t sel_h = wave_smallest(ch, take_h, valid_h);
    uint64_t sel_l = wave_smallest(cl, take_l, valid_l);
    const int ih = (int)key_index(ch), il = (int)key_index(cl);
    // a free SV can win on both sides: keep one copy
    bool dup = false;
    for (uint64_t m = sel_h; m; m &= m - 1) {
      const int src = __ffsll((unsigned long long)m) - 1;
      dup |= __builtin_amdgcn_readlane(ih, src) == il;
    }
    sel_l &= ~__ballot(dup);
    stamp(10);
    const uint64_t below = (1ull << lane) - 1ull;
    if ((sel_h >> lane) & 1ull) pl.key[n_miss + __popcll(sel_h & below)] = ih;
    if ((sel_l >> lane) & 1ull) pl.key[n_miss + __popcll(sel_h) + __popcll(sel_l & below)] = il;
    if (lane == 0) pl.n_new = n_miss + __popcll(sel_h) + __popcll(sel_l);
  }
  __syncthreads();
  stamp(2);

  // 2b. all waves: CLOCK victim scan of the window (prefetched bits), 4
  //     consecutive positions per thread, one block-wide rank
  const int M = pl.n_new;  // uniform
  if (M > 0) {
    const int pin0 = pl.hit_hi, pin1 = pl.hit_lo;
    bool e[4], unp[4];
    int cnt = 0, cnt2 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unp[j] = 4 * tid + j < W && wp[j] != pin0 && wp[j] != pin1;
      e[j] = unp[j] && view.ref_fix(wp[j], wref[j]) == 0;
      cnt += e[j];
      cnt2 += unp[j] && !e[j];
    }
    int total = 0;
    int r = block_excl_scan(cnt, &total, kscan);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (e[j]) {
        if (r < M) {
          pl.line[r] = wp[j];
          pl.old[r] = view.key_fix(wp[j], wkey[j]);
        }
        if (r == M - 1) pl.span = 4 * tid + j + 1;  // second chances consumed up to here
        ++r;
      }
    }
    if (total < M) {  // uniform: the window was (nearly) all referenced
      int total2 = 0;
      int r2 = block_excl_scan(cnt2, &total2, kscan);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (unp[j] && !e[j]) {
          if (total + r2 < M) {
            pl.line[total + r2] = wp[j];
            pl.old[total + r2] = view.key_fix(wp[j], wkey[j]);
          }
          ++r2;
        }
      }
      if (tid == 0) pl.span = W;
    }
    __syncthreads();
  }

  stamp(3);
  // 2c. wave 0: host-tier fetch / spill (lane q <-> new line q), f-update lines
  if (wave == 0) {
    int my_key = -1, my_line = -1, my_old = -1, my_hsrc = -1;
    if (lane < M) {
      my_key = pl.key[lane];
      my_line = pl.line[lane];
      my_old = pl.old[lane];
      my_hsrc = view.hslot(my_key);
    }
    const bool want_spill = lane < M && a.H > 0 && my_old >= 0 && view.hslot(my_old) < 0;
    const uint64_t sm = __ballot(want_spill);
    const int srank = __popcll(sm & ((1ull << lane) - 1ull));
    int my_hline = -1, my_hold = -1;
    const int hl = a.H > 0 ? (int)(((int64_t)rin.hhand + srank) % a.H) : -1;
    bool clash = false;  // never overwrite a host line this iteration fetches from
    for (int q = 0; q < M; ++q) clash |= __shfl(my_hsrc, q, 64) == hl;  // all lanes active
    if (want_spill && !clash && srank < a.H) {  // distinct host lines even when H < kNQ
      my_hline = hl;
      my_hold = view.hkey(hl);
    }
    const int n_fetch = __popcll(__ballot(lane < M && my_hsrc >= 0));
    const int n_spill_used = __popcll(__ballot(my_hline >= 0));
    const int line0 = __shfl(my_line, 0, 64), line1 = __shfl(my_line, 1, 64);
    if (lane < M) {
      pl.op[lane] = my_hsrc >= 0 ? kOpFetch : kOpCompute;
      pl.hsrc[lane] = my_hsrc;
      pl.hline[lane] = my_hline;
      pl.hold[lane] = my_hold;
    }
    if (lane == 0) {
      pl.n_fetch = n_fetch;
      pl.n_compute = M - n_fetch;
      pl.n_spill = n_spill_used;
      pl.line_hi = need_hi >= 0 ? (hit_hi >= 0 ? hit_hi : line0) : -1;
      if (c_lo != 0.f) {
        if (i_lo == i_hi && c_hi != 0.f) pl.line_lo = pl.line_hi;
        else pl.line_lo = hit_lo >= 0 ? hit_lo : (miss_hi ? line1 : line0);
      } else {
        pl.line_lo = -1;
      }
      const int span = M > 0 ? pl.span : 0;
      pl.span = span;
      pl.hand0 = rin.hand;
      pl.hand = (int)(((int64_t)rin.hand + span) % a.L);
      pl.hhand = a.H > 0 ? (int)(((int64_t)rin.hhand + __popcll(sm)) % a.H) : 0;
    }
  }
  __syncthreads();
  stamp(4);
  const int n_new = pl.n_new;

  // ---- 3. fill this workgroup's rows of the new lines ----
  if (n_new > 0 && done != kNonFinite && done != kNoPair) {
    if (a.hlines) {
      if (pl.n_spill > 0) {
        for (int q = 0; q < n_new; ++q) {
          const int h = pl.hline[q];
          if (h < 0) continue;
          const float* src = a.lines + (int64_t)pl.line[q] * a.ldl;
          float* dst = a.hlines + (int64_t)h * a.ldl;
          for (int64_t j = row0 + tid; j < row_end; j += kFusedThreads) dst[j] = src[j];
        }
        __syncthreads();  // old contents out before new values land
      }
      for (int q = 0; q < n_new; ++q) {
        if (pl.op[q] != kOpFetch) continue;
        const float* src = a.hlines + (int64_t)pl.hsrc[q] * a.ldl;
        float* dst = a.lines + (int64_t)pl.line[q] * a.ldl;
        for (int64_t j = row0 + tid; j < row_end; j += kFusedThreads) dst[j] = src[j];
      }
    }
    if (pl.n_compute > 0) xpass_fill(a, row0, row_end, n_new, pl.key, pl.line, pl.op, wsm, false);
    __syncthreads();  // this workgroup's new line segments are visible to all its waves
  }

  stamp(5);
  // ---- 5. (last workgroup: fewest rows) publish this iteration's record ----
  if (committer) {
    const bool upd = done != kNonFinite && done != kNoPair;
    if (tid < kNQ) {
      const int q = tid;
      const bool v = upd && q < n_new;
      r_out->line[q] = v ? pl.line[q] : -1;
      r_out->key[q] = v ? pl.key[q] : -1;
      r_out->old[q] = v ? pl.old[q] : -1;
      r_out->hline[q] = v ? pl.hline[q] : -1;
      r_out->hold[q] = v ? pl.hold[q] : -1;
    }
    if (tid == 0) {
      FusedCacheRec o;  // scalar part (arrays written above)
      o.i_hi = upd ? i_hi : -1;
      o.i_lo = upd ? i_lo : -1;
      o.a_hi = a_hi_new;
      o.a_lo = a_lo_new;
      o.iter = upd ? iter : rin.iter;
      o.done = done;
      o.b_hi = nopair ? rin.b_hi : b_hi;
      o.b_lo = nopair ? rin.b_lo : b_lo;
      o.n_new = upd ? n_new : 0;
      o.hand0 = pl.hand0;
      o.span = upd ? pl.span : 0;
      o.hand = upd ? pl.hand : rin.hand;
      o.hit_line[0] = upd ? pl.hit_hi : -1;
      o.hit_line[1] = upd ? pl.hit_lo : -1;
      o.hhand = upd ? pl.hhand : rin.hhand;
      o.hits = rin.hits + (upd ? pl.n_need - pl.n_miss : 0);
      o.misses = rin.misses + (upd ? pl.n_miss : 0);
      o.rows_computed = rin.rows_computed + (upd ? pl.n_compute : 0);
      o.x_passes = rin.x_passes + ((upd && pl.n_compute > 0) ? 1 : 0);
      o.spec_rows = rin.spec_rows + (upd ? n_new - pl.n_miss : 0);
      o.host_hits = rin.host_hits + (upd ? pl.n_fetch : 0);
      o.spills = rin.spills + (upd ? pl.n_spill : 0);
      r_out->i_hi = o.i_hi; r_out->i_lo = o.i_lo; r_out->a_hi = o.a_hi; r_out->a_lo = o.a_lo;
      r_out->iter = o.iter; r_out->done = o.done; r_out->b_hi = o.b_hi; r_out->b_lo = o.b_lo;
      r_out->n_new = o.n_new; r_out->hand0 = o.hand0; r_out->span = o.span; r_out->hand = o.hand;
      r_out->hit_line[0] = o.hit_line[0]; r_out->hit_line[1] = o.hit_line[1]; r_out->hhand = o.hhand;
      r_out->hits = o.hits; r_out->misses = o.misses; r_out->rows_computed = o.rows_computed;
      r_out->x_passes = o.x_passes; r_out->spec_rows = o.spec_rows; r_out->host_hits = o.host_hits;
      r_out->spills = o.spills;
      if (done != kRunning || iter % kStatusEvery == 0) publish_status_lru(a.status, o);
    }
  }
  stamp(6);
  if (done == kNonFinite || done == kNoPair) return;

  // ---- 4. f update + classification of this workgroup's rows ----
  // All of a thread's rows in one chunk when they fit (<= 12): every load of the
  // chunk is issued unconditionally (idle slots and absent lines read a safe
  // in-bounds address) so the whole chunk is one round trip with no branches.
  const bool upd_f = c_hi != 0.f || c_lo != 0.f;
  const float* lh = pl.line_hi >= 0 ? a.lines + (int64_t)pl.line_hi * a.ldl : a.f;
  const float* ll = pl.line_lo >= 0 ? a.lines + (int64_t)pl.line_lo * a.ldl : a.f;
  const float chv = c_hi, clv = c_lo;
  const float* fa = a.f;
  const float* aa = a.alpha + a.off;
  const float* ya = a.y + a.off;
  uint64_t nh = kKeyNone, nlk = kKeyNone;
  auto rows_chunked = [&](auto chunk) {
    constexpr int CH = decltype(chunk)::value;
    for (int64_t jb = j0; jb < row_end; jb += (int64_t)CH * kFusedThreads) {
      float fv[CH], hv[CH], lv[CH], av[CH], yy[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int64_t j = jb + (int64_t)c * kFusedThreads;
        const int64_t jj = j < row_end ? j : j0;  // in-bounds address for idle slots
        fv[c] = fa[jj];
        hv[c] = lh[jj];
        lv[c] = ll[jj];
        av[c] = aa[jj];
        yy[c] = ya[jj];
      }
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int64_t j = jb + (int64_t)c * kFusedThreads;
        if (j >= row_end) break;  // slots are in increasing j
        const int64_t g = a.off + j;
        float fj = fv[c];
        if (upd_f) {
          // absent lines read f (finite) through the dummy pointer: zero it
          fj = f_apply(fj, chv, chv != 0.f ? hv[c] : 0.f, clv, clv != 0.f ? lv[c] : 0.f);
          a.f[j] = fj;
        }
        if (done == kRunning) {
          float al;
          if (g == i_hi) al = a_hi_new;
          else if (g == i_lo) al = a_lo_new;
          else if (g == rin.i_hi) al = rin.a_hi;
          else if (g == rin.i_lo) al = rin.a_lo;
          else al = av[c];
          if (in_up(al, yy[c], a.C)) { const uint64_t k = make_key(fj, (uint32_t)g); nh = k < nh ? k : nh; }
          if (in_low(al, yy[c], a.C)) { const uint64_t k = make_key(-fj, (uint32_t)g); nlk = k < nlk ? k : nlk; }
        }
      }
    }
  };
  const int64_t rpt = (row_end - row0 + kFusedThreads - 1) / kFusedThreads;  // uniform
  if (rpt <= 2) rows_chunked(std::integral_constant<int, 2>{});
  else if (rpt <= 4) rows_chunked(std::integral_constant<int, 4>{});
  else rows_chunked(std::integral_constant<int, 12>{});
  if (done != kRunning) return;  // uniform
  nh = wave_min_u64(nh);
  nlk = wave_min_u64(nlk);
  if (lane == 0) {
    kscr[wave] = nh;
    kscr[4 + wave] = nlk;
  }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      nh = kscr[w] < nh ? kscr[w] : nh;
      nlk = kscr[4 + w] < nlk ? kscr[4 + w] : nlk;
    }
    u64x2l v;
    v.x = nh;
    v.y = nlk;
    *(u64x2l*)(p_out + 2 * blockIdx.x) = v;
  }
  stamp(7);
}

}  // namespace dev

namespace launch {

size_t smo_fused_lru_lds_bytes(int dp, int fused_rows) { return dev::xpass_lds_floats(dp, fused_rows) * sizeof(float); }

bool smo_fused_lru_supported(int dp) { return dp >= 16 && dp % 16 == 0; }

void smo_fused_lru(const SmoArgs& a, const uint64_t* p_in, uint64_t* p_out, const FusedCacheRec* r_in,
                   FusedCacheRec* r_out, hipStream_t s) {
  const size_t lds = smo_fused_lru_lds_bytes(a.dp, a.fused_rows);
  static size_t attr_bytes = 64 * 1024;  // dynamic LDS above 64 KiB needs the attribute (160 KiB LDS on gfx950)
  if (lds > attr_bytes) {
    HIP_CHECK(hipFuncSetAttribute((const void*)dev::smo_fused_lru_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
    attr_bytes = lds;
  }
  dev::smo_fused_lru_kernel<<<dim3(a.fused_G), kFusedThreads, lds, s>>>(a, p_in, p_out,
                                                                                                  r_in, r_out);
  post_launch("smo_fused_lru", s);
}

}  // namespace launch
}  // namespace dpsvm
