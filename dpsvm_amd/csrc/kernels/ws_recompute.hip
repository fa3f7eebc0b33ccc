// Working-set engine without a kernel-row cache (ws-cache engine, recompute
// mode): when the Gram does not fit and the rows are short (d <= 64 padded,
// covtype's 54 features), a kernel row costs one pass over X's split operands
// (256 B a row) plus a few MFMAs — less than writing it into a cache line and
// reading it back.  So a round computes only what it uses:
//
//   ws_subgram_split   the merge (redundantly in every workgroup, as ws_gather)
//                      and one 64 x 64 tile of the q x q sub-Gram K(set, set)
//                      per workgroup, straight from the members' split X rows;
//   ws_solve           unchanged (sub-Gram + aux from global memory);
//   ws_fupdate_split   the selection pass: f_j += sum_k c_k K(k, j) over the
//                      round's changed rows k for every column j (the changed
//                      rows' split X rows staged in LDS, the columns' rows
//                      streamed, K by the split MFMA and the Gram kernels'
//                      epilogue, the weighted sum over rows in a fixed order, f
//                      updated in place — no K row is ever stored), then each
//                      selection group's candidate lists (ws_select's lists:
//                      the same columns per group).
//
// The cache path of the same round (ws_merge line assignment, the miss-row GEMM
// writing ~44 rows x 581k columns, the f update re-reading ~58 cached rows)
// moves ~250 MB per covtype round; this one streams X once (~150 MB).  The K
// values are the split GEMMs' bits (same MFMA order, the same epilogue:
// rbf_split_value); the f update sums them per column over the rows instead of
// per row over the list, so the trajectory matches the cache path to rounding,
// not bit for bit.
// Reference: svmTrain.cu:98-137 (the f update), svmTrain.cu:212-249 (kernel rows).
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "split_util.hpp"
#include "ws_common.hpp"
#include "ws_merge.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// ---------------------------------------------------------------------------
// merge + one 64 x 64 tile of the sub-Gram (4 waves of 32 x 32)
// ---------------------------------------------------------------------------
template <int NKB>
__global__ __launch_bounds__(kWsGatherThreads) void ws_subgram_split_kernel(WsArgs a, const u4* __restrict__ xs,
                                                                            const int32_t* __restrict__ xsh,
                                                                            const float* __restrict__ xsq,
                                                                            float gamma) {
  __shared__ int32_t s_idx[kWsMax];
  __shared__ WsMergeLds L;
  __shared__ float s_sq[2][64];
  __shared__ int32_t s_sh[2][64];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5;
  const bool lead = blockIdx.x == 0 && tid == 0;
  if (lead) WS_STAMP(1);
  int q = 0;
  float b_hi = 0.f, b_lo = 0.f;
  if (!ws_merge(a, c, s_idx, &q, &b_hi, &b_lo, L)) return;
  if (lead) WS_STAMP(2);
  const int par = (int)(c->outer & 1);
  const int tn = (a.q_max + 63) / 64;
  const int tx = (int)blockIdx.x / tn, ty = (int)blockIdx.x % tn;
  if (blockIdx.x == 0) {
    for (int t = tid; t < q; t += kWsGatherThreads) {
      c->idx[par][t] = s_idx[t];
      c->line[par][t] = s_idx[t];  // no cache line: the row itself
    }
    if (tid == 0) {
      c->q[par] = q;
      c->b_hi = b_hi;
      c->b_lo = b_lo;
    }
  }
  if (tx * 64 >= q) return;  // uniform: no barrier after this
  if (tid < 128) {           // |x|^2 and shifts of the tile's rows (0..63) and columns (64..127)
    const int s = tid >> 6, k = (s ? ty : tx) * 64 + (tid & 63);
    const int64_t g = s_idx[min(k, q - 1)];
    s_sq[s][tid & 63] = xsq[g];
    s_sh[s][tid & 63] = xsh[g];
  }
  if (ty == 0 && tid < 64 && tx * 64 + tid < q) {  // aux: f / alpha / y of the tile's rows (one rank)
    const int ra = tx * 64 + tid;
    const int64_t gi = s_idx[ra];
    a.aux[ra] = a.f[gi];
    a.aux[a.aux_stride + ra] = a.alpha[gi];
    a.aux[2 * a.aux_stride + ra] = a.y[gi];
  }
  __syncthreads();
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;  // the wave's 32 x 32 block in the tile
  const int r_lane = tx * 64 + wr + (lane & 31), c_lane = ty * 64 + wc + (lane & 31);
  const u4* ar = xs + (int64_t)s_idx[min(r_lane, q - 1)] * (NKB * 8);
  const u4* br = xs + (int64_t)s_idx[min(c_lane, q - 1)] * (NKB * 8);
  f16v H, P, Q;
#pragma unroll
  for (int r = 0; r < 16; ++r) H[r] = P[r] = Q[r] = 0.f;
  // the split GEMMs' MFMA order: k blocks in order, two k16 steps each, H / P / Q
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = kb * 8 + 2 * ks + hl, cl = kb * 8 + 4 + 2 * ks + hl;
      const h8 ah = __builtin_bit_cast(h8, ar[ch]), al = __builtin_bit_cast(h8, ar[cl]);
      const h8 bh = __builtin_bit_cast(h8, br[ch]), bl = __builtin_bit_cast(h8, br[cl]);
      H = mfma32_f16(ah, bh, H);
      P = mfma32_f16(ah, bl, P);
      Q = mfma32_f16(al, bh, Q);
    }
  }
  const int cl_t = wc + (lane & 31);  // the lane's column inside the tile
  const float bsq = s_sq[1][cl_t];
  const int bsh = s_sh[1][cl_t];
  const int col = ty * 64 + cl_t;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int lr_t = wr + (r & 3) + 8 * (r >> 2) + 4 * hl;  // the value's row inside the tile
    const int row = tx * 64 + lr_t;
    const float dot = ldexpf(H[r] + (P[r] + Q[r]), -(s_sh[0][lr_t] + bsh));
    const float v = rbf_split_value(s_sq[0][lr_t], bsq, dot, gamma);
    if (row < q && col < a.q_max) a.subg[(int64_t)row * a.q_max + col] = col < q ? v : 0.f;
  }
  if (lead) WS_STAMP(8);
}

// ---------------------------------------------------------------------------
// The round's selection pass with the kernel rows recomputed: f_j += sum_k c_k
// K(k, j) over the changed rows k, then each workgroup's kWsCand1 smallest keys
// per side.  Workgroup g owns selection group g's columns (ws_select's
// geometry: rpt x 256 of them), so its lists are ws_select's — the top keys of
// the same columns.  The changed rows (M <= q_max <= 192: nrb blocks of 32)
// are staged in LDS once; each wave then walks 32-column blocks of the group on
// its own (no barrier until the lists), all nrb row blocks of a column block
// by the split MFMA, with the next block's operands loading into the other of
// two register sets.  Per column: each lane sums its rows (row blocks in
// order, 16 rows each in order), the two half-waves add (a + b == b + a: both
// lanes the same bits); each lane keeps its columns' 4 smallest keys a side.
// ---------------------------------------------------------------------------
constexpr int kFupdThreads = 512;  // 8 waves: two per SIMD, up to 256 registers each (no spills)

// keep the 4 smallest of l (ascending) and k
__device__ __forceinline__ void top4_insert(uint64_t (&l)[kWsCand1], uint64_t k) {
#pragma unroll
  for (int i = 0; i < kWsCand1; ++i) {
    const uint64_t lo = l[i] < k ? l[i] : k, hi = l[i] < k ? k : l[i];
    l[i] = lo;
    k = hi;
  }
}

template <int NKB>
__global__ __launch_bounds__(kFupdThreads) void ws_fupdate_split_kernel(WsArgs a, const u4* __restrict__ xs,
                                                                        const int32_t* __restrict__ xsh,
                                                                        const float* __restrict__ xsq, float gamma) {
  constexpr int CPR = NKB * 8;   // u4 per split row
  constexpr int W = kFupdThreads / 64;
  __shared__ u4 s_a[192 * CPR];  // the changed rows, chunk c of row r at c ^ ((r >> 1) & 7) within its k block
  __shared__ float s_coef[192], s_asq[192];
  __shared__ int32_t s_ash[192];
  __shared__ uint64_t s_wc[W][2][kWsCand1];
  WsCtrl* c = a.ctrl;
  const int M = c->n_apply;  // uniform
  const int done = c->done;
  if (M == 0 && done != kRunning) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(6);
  const int nrb = (M + 31) / 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5;
  for (int id = tid; id < nrb * 32 * CPR; id += kFupdThreads) {
    const int r = id / CPR, ch = id % CPR, kb = ch >> 3, cc = ch & 7;
    const int64_t g = c->apply_idx[min(r, M - 1)];
    s_a[r * CPR + kb * 8 + (cc ^ ((r >> 1) & 7))] = xs[g * CPR + ch];
  }
  if (tid < nrb * 32) {
    const int64_t g = c->apply_idx[min(tid, M - 1)];
    s_coef[tid] = tid < M ? c->apply_coef[tid] : 0.f;  // padding rows add exactly zero
    s_asq[tid] = xsq[g];
    s_ash[tid] = xsh[g];
  }
  __syncthreads();
  const int64_t N = a.nl;
  const int64_t g0 = (int64_t)blockIdx.x * a.rpt * kWsSelThreads;  // this group's columns [g0, g1)
  const int64_t g1 = min(N, g0 + (int64_t)a.rpt * kWsSelThreads);
  const int64_t nblk = (g1 - g0 + 31) / 32;
  const int sw = ((lane & 31) >> 1) & 7;
  struct Cols {
    u4 b[NKB * 4];
    float sq, f, al, y;
    int sh;
  };
  // operands of the group's column block t (past the last block: re-read a valid one)
  auto load = [&](int64_t t, Cols& o) {
    const int64_t j = min(g0 + min(t, nblk - 1) * 32 + (lane & 31), g1 - 1);
    const u4* br = xs + (a.off + j) * CPR;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        o.b[kb * 4 + 2 * ks] = br[kb * 8 + 2 * ks + hl];
        o.b[kb * 4 + 2 * ks + 1] = br[kb * 8 + 4 + 2 * ks + hl];
      }
    o.sq = xsq[a.off + j];
    o.sh = xsh[a.off + j];
    o.f = a.f[j];
    o.al = a.alpha[a.off + j];
    o.y = a.y[a.off + j];
  };
  bool bad = false;
  uint64_t lu[kWsCand1], ll[kWsCand1];
#pragma unroll
  for (int r = 0; r < kWsCand1; ++r) lu[r] = ll[r] = kKeyNone;
  auto block = [&](int64_t t, const Cols& o) {
    float acc = 0.f;
    for (int rb = 0; rb < nrb; ++rb) {
      f16v H, P, Q;
#pragma unroll
      for (int r = 0; r < 16; ++r) H[r] = P[r] = Q[r] = 0.f;
      const int ra = (rb * 32 + (lane & 31)) * CPR;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int ch = kb * 8 + ((2 * ks + hl) ^ sw), cl = kb * 8 + ((4 + 2 * ks + hl) ^ sw);
          const h8 ah = __builtin_bit_cast(h8, s_a[ra + ch]), al = __builtin_bit_cast(h8, s_a[ra + cl]);
          const h8 bh = __builtin_bit_cast(h8, o.b[kb * 4 + 2 * ks]);
          const h8 bl = __builtin_bit_cast(h8, o.b[kb * 4 + 2 * ks + 1]);
          H = mfma32_f16(ah, bh, H);
          P = mfma32_f16(ah, bl, P);
          Q = mfma32_f16(al, bh, Q);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const float dot = ldexpf(H[r] + (P[r] + Q[r]), -(s_ash[lr] + o.sh));
        const float v = rbf_split_value(s_asq[lr], o.sq, dot, gamma);
        {
#pragma clang fp contract(off)
          acc = acc + s_coef[lr] * v;
        }
      }
    }
    float fj = o.f;
    if (nrb > 0) {
#pragma clang fp contract(off)
      const float sum = acc + __shfl_xor(acc, 32);  // the two half-waves: a + b == b + a
      fj = o.f + sum;
    }
    const int64_t j = g0 + t * 32 + (lane & 31);
    if (t < nblk && hl == 0 && j < g1) {
      if (nrb > 0) {
        a.f[j] = fj;
        bad |= !isfinite(fj);
      }
      if (done == kRunning) {
        if (in_up(o.al, o.y, a.C)) top4_insert(lu, make_key(fj, (uint32_t)(a.off + j)));
        if (in_low(o.al, o.y, a.C)) top4_insert(ll, make_key(-fj, (uint32_t)(a.off + j)));
      }
    }
  };
  int64_t blk = wave;
  if (blk < nblk) {
    Cols c0, c1;
    load(blk, c0);
    for (; blk < nblk; blk += 2 * W) {
      load(blk + W, c1);
      __builtin_amdgcn_sched_barrier(0);  // the prefetch is issued before the block's work
      block(blk, c0);
      load(blk + 2 * W, c0);
      __builtin_amdgcn_sched_barrier(0);
      block(blk + W, c1);
    }
  }
  if (bad) atomicOr(&c->nonfinite, 1);
  if (blockIdx.x == 0 && tid == 0) c->rows_computed += M;  // kernel rows evaluated this round (none stored)
  if (done != kRunning) return;  // uniform: no lists
  // the wave's kWsCand1 smallest keys a side (the lane holding a winner pops
  // it: keys are unique), then wave 0 merges the W lists
  for (int rr = 0; rr < kWsCand1; ++rr) {
    const uint64_t mu = wave_min_u64(lu[0]), ml = wave_min_u64(ll[0]);
    if (lane == 0) {
      s_wc[wave][0][rr] = mu;
      s_wc[wave][1][rr] = ml;
    }
    if (lu[0] == mu) {
#pragma unroll
      for (int r = 0; r + 1 < kWsCand1; ++r) lu[r] = lu[r + 1];
      lu[kWsCand1 - 1] = kKeyNone;
    }
    if (ll[0] == ml) {
#pragma unroll
      for (int r = 0; r + 1 < kWsCand1; ++r) ll[r] = ll[r + 1];
      ll[kWsCand1 - 1] = kKeyNone;
    }
  }
  __syncthreads();
  if (wave == 0) {
    const bool hv = lane < W * kWsCand1;
    uint64_t eu = hv ? s_wc[lane / kWsCand1][0][lane % kWsCand1] : kKeyNone;
    uint64_t el = hv ? s_wc[lane / kWsCand1][1][lane % kWsCand1] : kKeyNone;
    uint64_t* out = a.cand_out + (size_t)blockIdx.x * 2 * kWsCand;
    for (int rr = 0; rr < kWsCand1; ++rr) {
      const uint64_t mu = wave_min_u64(eu), ml = wave_min_u64(el);
      if (lane == 0) {
        out[rr] = mu;
        out[kWsCand + rr] = ml;
      }
      if (eu == mu) eu = kKeyNone;
      if (el == ml) el = kKeyNone;
    }
  }
  if (blockIdx.x == 0 && tid == 0) WS_STAMP(7);
}

}  // namespace dev

namespace launch {

// (one-block rounds only: a multi-block ws-cache engine runs its multi-block
// rounds on the row cache and its one-block rounds — after the adaptive count
// reached 1 — without it)
bool ws_recompute_supported(const WsArgs& a, int dp) {
  return dp <= 64 && a.world == 1 && a.xpeer == nullptr && a.off == 0 && a.q_max <= kWsMax;
}

void ws_subgram_split(const WsArgs& a, const void* xs, const int32_t* xsh, const float* xsq, int dp, float gamma,
                      hipStream_t s) {
  const int tn = (a.q_max + 63) / 64;
  const dim3 grid((unsigned)(tn * tn));
  auto fn = (dp + 31) / 32 <= 1 ? dev::ws_subgram_split_kernel<1> : dev::ws_subgram_split_kernel<2>;
  fn<<<grid, dev::kWsGatherThreads, 0, s>>>(a, (const dev::u4*)xs, xsh, xsq, gamma);
  post_launch("ws_subgram_split", s);
}

void ws_fupdate_split(const WsArgs& a, const void* xs, const int32_t* xsh, const float* xsq, int dp, float gamma,
                      hipStream_t s) {
  static const int cus = [] {
    int dev = 0, n = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    return std::max(1, n);
  }();
  // one workgroup per selection group (the group's lists are ws_select's); a
  // group's 8 waves walk its 32-column blocks
  (void)cus;
  const int64_t grid = a.G;
  auto fn = (dp + 31) / 32 <= 1 ? dev::ws_fupdate_split_kernel<1> : dev::ws_fupdate_split_kernel<2>;
  fn<<<dim3((unsigned)grid), dev::kFupdThreads, 0, s>>>(a, (const dev::u4*)xs, xsh, xsq, gamma);
  post_launch("ws_fupdate_split", s);
}

}  // namespace launch
}  // namespace dpsvm
