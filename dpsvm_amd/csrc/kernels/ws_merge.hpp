// Working-set engine: the one-block merge (stop test and the next working set
// from every selection workgroup's candidate lists), used by the round
// kernels of ws_merge.hip and ws_recompute.hip.  Round structure and helpers:
// ws_common.hpp.
#pragma once

#include "ws_common.hpp"

namespace dpsvm {
namespace dev {

// ---------------------------------------------------------------------------
// the merge: stop test and the new working set (one 256-thread workgroup;
// identical result in every workgroup that runs it).  Returns false when the
// run stopped (done is then set by workgroup 0).  s_idx[0..*q) = the set,
// newest first; *b_hi / *b_lo = the global selection.
// ---------------------------------------------------------------------------
// its LDS (the caller's: a persistent round kernel overlays it with the sub-Gram)
struct WsMergeLds {
  int hist[2][256];
  int sel[2][2];
  int thr[2];
  int wsum[4];
  uint64_t wsum64[4];
  uint64_t scr[8];
  uint64_t sv[2][kWsMaxCand];
  int32_t hash[4][kWsHash];  // up keys, up ranks, low keys, low ranks
  int32_t keep[2 * kWsMax];  // per interleaved position: final slot or -1
};

__device__ inline bool ws_merge(const WsArgs& a, WsCtrl* c, int32_t* s_idx, int* q_out, float* bh_out, float* bl_out,
                                WsMergeLds& L) {
  auto& s_hist = L.hist;
  auto& s_sel = L.sel;
  auto& s_thr = L.thr;
  auto& s_wsum64 = L.wsum64;
  auto& s_sv = L.sv;
  auto& s_hash = L.hash;
  auto& s_keep = L.keep;
  auto& s_scr = L.scr;
  auto& s_wsum = L.wsum;
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
  for (int j = 0; j < kWsListsPerThread; ++j) {
    const int slot = tid + j * kWsGatherThreads;
    if (slot >= G) break;
    // every rank's lists: all-gathered, or (peer exchange) collected from this
    // rank's receive buffer by ws_xcollect_cand — the merge never spins
    uint64_t cu[kWsCand1], cl[kWsCand1];
#pragma unroll
    for (int r = 0; r < kWsCand1; ++r) {
      cu[r] = a.cand[(size_t)slot * 2 * kWsCand + r];
      cl[r] = a.cand[(size_t)slot * 2 * kWsCand + kWsCand + r];
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

}  // namespace dev
}  // namespace dpsvm
