// SMO iteration kernels for the kernel-row-cache ("LRU") mode, MI355X (gfx950).
// QUARANTINED (the "chain" engine: pair-at-a-time with X partitioned): built
// into the pair-cache plugin (dpsvm_amd/_pairq, solver/gpu_engines_pairq.hip),
// not into the production module; engines="all" loads it.
// (The Gram-resident dense mode uses the single fused kernel in smo_fused.hip.)
//
//   smo_rows      fill this iteration's cache lines: (1) spill victims' old
//                 contents to the pinned host tier, (2) fetch host-tier hits back
//                 (zero-copy PCIe loads), (3) ONE X pass computing up to 16 new
//                 kernel rows on fp32 MFMA 16x16x4 (exact f32), query vectors in
//                 LDS, fused expansion + exp epilogue.  Replaces the reference's
//                 per-miss cublasSgemv x2 on two streams (svmTrain.cu:212-249,
//                 K3/K4) and the functor turning dot products into RBF values (K5).
//   smo_step      pending f update (svmTrain.cu:98-137) fused with I-set
//                 classification and the argmin/argmax selection
//                 (svmTrain.cu:41-95 + 400-483): per-workgroup u64 keys.
//   smo_finalize  one workgroup: global pair, eta on device (was host CBLAS,
//                 svmTrain.cu:696-714), alpha update + clip
//                 (svmTrainMain.cpp:282-299), stop test, the cache policy and
//                 next iteration's row requests, host-mapped status record.
//
// Cache policy: CLOCK (second chance) instead of the reference's host-side
// std::map + std::list LRU (cache.cu:62-105, O(L) lookup, host sync every
// iteration).  Hits set a reference bit (one store); allocating up to 16 lines
// is ONE parallel pass over a 1024-line window (ballot + prefix ranks), so the
// policy costs a constant number of dependent global round trips.  Optional
// pinned host tier = FIFO victim cache (SURVEY §5.7 spill tier).
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// ---------------------------------------------------------------------------
// smo_rows
// Grid: G workgroups x 256 threads, 128 local rows per workgroup; each wave
// owns two 16-row MFMA tiles.  MFMA 16x16x4 f32 operand map: A lane l ->
// (row l&15, k l>>4), B lane l -> (k l>>4, query l&15).  Each lane loads a
// float4 of X (16 contiguous columns per 16 rows and wave-instruction);
// component c of the float4 feeds MFMA c — a permutation of k that the query
// operand (LDS, same float4) mirrors.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kStepThreads) void smo_rows_kernel(SmoArgs a) {
  const SmoCtrl* c = a.ctrl;
  const int nq = c->nq;
  if (nq == 0 || (c->done != kRunning && c->final_applied)) return;
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t blk_row0 = (int64_t)blockIdx.x * kStepRows;

  // (1) spill the victims' old contents to the host tier, (2) fetch host hits.
  //     Each workgroup touches only its own 128 rows of every line.
  if (a.hlines) {
    const int half = tid >> 7, r = tid & 127;
    if (c->n_spill > 0) {
      for (int q = half; q < nq; q += 2) {
        const int h = c->q_hspill[q];
        if (h >= 0) {
          const int64_t col = blk_row0 + r;
          a.hlines[(int64_t)h * a.ldl + col] = a.lines[(int64_t)c->q_line[q] * a.ldl + col];
        }
      }
      __syncthreads();  // old contents read before any new value lands
    }
    for (int q = half; q < nq; q += 2) {
      if (c->q_op[q] == kOpFetch) {
        const int64_t col = blk_row0 + r;
        a.lines[(int64_t)c->q_line[q] * a.ldl + col] = a.hlines[(int64_t)c->q_hsrc[q] * a.ldl + col];
      }
    }
  }
  if (c->n_compute == 0) return;

  // (3) X pass for the kOpCompute queries
  const int64_t row0 = blk_row0 + wave * 32;
  const int64_t xbase = a.off - a.x_row0;  // local row -> device X row
  const int dp = a.dp;
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const float* xr0 = a.x + (xbase + row0 + (lane & 15)) * dp + 4 * (lane >> 4);
  const float* xr1 = xr0 + 16 * (int64_t)dp;

  for (int kc = 0; kc < dp; kc += kRowsKC) {
    const int kcl = min(kRowsKC, dp - kc);
    const int ldw = kcl + 4;  // +4 floats: 16 query rows hit distinct 16-B bank slots
    const int k4n = kcl >> 2;
    for (int i = tid; i < kNQ * k4n; i += kStepThreads) {
      const int q = i / k4n, k4 = i - q * k4n;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (q < nq && c->q_op[q] == kOpCompute) v = *(const f4*)(c->q_ptr[q] + kc + 4 * k4);
      *(f4*)(wsm + q * ldw + 4 * k4) = v;
    }
    __syncthreads();
    const float* wr = wsm + (lane & 15) * ldw + 4 * (lane >> 4);
#pragma unroll 2
    for (int k0 = 0; k0 < kcl; k0 += 16) {
      const f4 xa = *(const f4*)(xr0 + kc + k0);
      const f4 xb = *(const f4*)(xr1 + kc + k0);
      const f4 wv = *(const f4*)(wr + k0);
      acc0 = mfma16(xa.x, wv.x, acc0);
      acc1 = mfma16(xb.x, wv.x, acc1);
      acc0 = mfma16(xa.y, wv.y, acc0);
      acc1 = mfma16(xb.y, wv.y, acc1);
      acc0 = mfma16(xa.z, wv.z, acc0);
      acc1 = mfma16(xb.z, wv.z, acc1);
      acc0 = mfma16(xa.w, wv.w, acc0);
      acc1 = mfma16(xb.w, wv.w, acc1);
    }
    __syncthreads();
  }
  // epilogue: lane holds rows (lane>>4)*4 + r of each tile for query lane&15
  const int q = lane & 15;
  if (q < nq && c->q_op[q] == kOpCompute) {
    const int64_t line = c->q_line[q];
    const float wsq = c->q_sq[q];
    float* out = a.lines + line * a.ldl;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f4 acc = t == 0 ? acc0 : acc1;
      const int64_t base = row0 + t * 16 + (lane >> 4) * 4;
      f4 kv;
#pragma unroll
      for (int r = 0; r < 4; ++r) kv[r] = rbf_from_dot(a.xsq[a.off + base + r], wsq, acc[r], a.gamma);
      *(f4*)(out + base) = kv;
    }
  }
}

// ---------------------------------------------------------------------------
// smo_step: apply the pending f update, classify, per-workgroup argmin/argmax.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kStepThreads) void smo_step_kernel(SmoArgs a) {
  const SmoCtrl* c = a.ctrl;
  const int done = c->done;
  if (done != kRunning && c->final_applied) return;
  __shared__ uint64_t scratch[2 * (kStepThreads / 64)];
  const int tid = threadIdx.x;
  const float ch = c->c_hi, cl = c->c_lo;
  uint64_t kh = kKeyNone, kl = kKeyNone;
  if (tid < kStepRows) {
    const int64_t j = (int64_t)blockIdx.x * kStepRows + tid;
    if (j < a.nl) {
      float fj = a.f[j];
      if (ch != 0.f || cl != 0.f) {
        const float khv = ch != 0.f ? a.lines[(int64_t)c->line_hi * a.ldl + j] : 0.f;
        const float klv = cl != 0.f ? a.lines[(int64_t)c->line_lo * a.ldl + j] : 0.f;
        fj = f_apply(fj, ch, khv, cl, klv);
        a.f[j] = fj;
      }
      if (done == kRunning) {
        const int64_t g = a.off + j;
        const float av = a.alpha[g], yv = a.y[g];
        if (in_up(av, yv, a.C)) kh = make_key(fj, (uint32_t)g);
        if (in_low(av, yv, a.C)) kl = make_key(-fj, (uint32_t)g);
      }
    }
  }
  if (done != kRunning) return;  // uniform
  block_min2_u64<kStepThreads>(kh, kl, scratch);
  if (tid == 0) {
    a.partials[2 * blockIdx.x] = kh;
    a.partials[2 * blockIdx.x + 1] = kl;
  }
}

// ---------------------------------------------------------------------------
// smo_local_record (partitioned X): reduce this rank's partials and package the
// two winning rows for the all-gather (SURVEY §5.8 alternative A).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void smo_local_record_kernel(SmoArgs a) {
  __shared__ uint64_t scratch[8];
  const SmoCtrl* c = a.ctrl;
  if (c->done != kRunning && c->final_applied) return;
  uint64_t kh = kKeyNone, kl = kKeyNone;
  if (c->done == kRunning) {
    for (int b = threadIdx.x; b < a.G; b += 256) {
      uint64_t h = a.partials[2 * b], l = a.partials[2 * b + 1];
      kh = h < kh ? h : kh;
      kl = l < kl ? l : kl;
    }
  }
  block_min2_u64<256>(kh, kl, scratch);
  CandRecord* rec = (CandRecord*)a.my_record;
  float* rows = (float*)(a.my_record + sizeof(CandRecord));
  if (threadIdx.x == 0) {
    rec->key_hi = kh;
    rec->key_lo = kl;
  }
  const float* xh = kh != kKeyNone ? a.x + ((int64_t)key_index(kh) - a.x_row0) * a.dp : nullptr;
  const float* xl = kl != kKeyNone ? a.x + ((int64_t)key_index(kl) - a.x_row0) * a.dp : nullptr;
  for (int k = threadIdx.x; k < a.dp; k += 256) {
    rows[k] = xh ? xh[k] : 0.f;
    rows[a.dp + k] = xl ? xl[k] : 0.f;
  }
}

// ---------------------------------------------------------------------------
// smo_finalize: one workgroup (16 waves), identical on every rank.
// ---------------------------------------------------------------------------
__device__ void write_status(const SmoArgs& a, const SmoCtrl* c) {
  SmoStatus* st = a.status;
  if (!st) return;
  st->iter = c->iter;
  st->done = c->done != kRunning ? (c->final_applied ? c->done : 0) : 0;
  st->b_hi = c->b_hi;
  st->b_lo = c->b_lo;
  st->hits = c->hits;
  st->misses = c->misses;
  st->rows_computed = c->rows_computed;
  st->x_passes = c->x_passes;
  st->spec_rows = c->spec_rows;
  st->host_hits = c->host_hits;
  st->spills = c->spills;
  __atomic_store_n(&st->seq, c->iter, __ATOMIC_RELEASE);
}

// exclusive prefix rank of `pred` over the workgroup (1024 threads); *total set
__device__ __forceinline__ int block_rank(bool pred, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(pred);
  if (lane == 0) wsum[wave] = __popcll(m);
  __syncthreads();
  int before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kFinThreads / 64; ++w) {
    before += w < wave ? wsum[w] : 0;
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return before + __popcll(m & ((1ull << lane) - 1ull));
}

__global__ __launch_bounds__(kFinThreads) void smo_finalize_kernel(SmoArgs a) {
  __shared__ uint64_t kscr[2 * (kFinThreads / 64)];
  __shared__ int wsum[kFinThreads / 64];
  __shared__ int s_i[32];
  __shared__ float s_f[4];
  __shared__ int32_t s_keys[kNQ];
  __shared__ int32_t s_lines[kNQ];
  __shared__ int32_t s_hsrc[kNQ];
  SmoCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  const int done_in = c->done;
  if (done_in != kRunning) {
    __syncthreads();
    if (tid == 0 && !c->final_applied) {
      c->final_applied = 1;
      c->nq = 0;
      c->n_compute = 0;
      c->n_spill = 0;
      c->c_hi = 0.f;
      c->c_lo = 0.f;
      write_status(a, c);
    }
    return;
  }

  // ---- 1. global selection (+ this thread's partial as a speculation candidate) ----
  uint64_t kh = kKeyNone, kl = kKeyNone, my_h = kKeyNone, my_l = kKeyNone;
  if (a.partitioned) {
    for (int r = tid; r < a.world; r += kFinThreads) {
      const CandRecord* rec = (const CandRecord*)(a.records + (int64_t)r * a.rec_bytes);
      kh = rec->key_hi < kh ? rec->key_hi : kh;
      kl = rec->key_lo < kl ? rec->key_lo : kl;
    }
  } else {
    for (int b = tid; b < a.G; b += kFinThreads) {
      const uint64_t h = a.partials[2 * b], l = a.partials[2 * b + 1];
      if (b == tid) {
        my_h = h;
        my_l = l;
      }
      kh = h < kh ? h : kh;
      kl = l < kl ? l : kl;
    }
  }
  block_min2_u64<kFinThreads>(kh, kl, kscr);
  if (kh == kKeyNone || kl == kKeyNone) {
    if (tid == 0) {
      c->done = kNoPair;
      c->final_applied = 1;
      c->nq = 0;
      c->n_compute = 0;
      c->n_spill = 0;
      c->c_hi = c->c_lo = 0.f;
      write_status(a, c);
    }
    return;
  }
  const int i_hi = (int)key_index(kh), i_lo = (int)key_index(kl);
  const float b_hi = key_value(kh), b_lo = -key_value(kl);

  // ---- 2. |x_hi - x_lo|^2 on device (explicit difference, svmTrain.cu:696-714) ----
  const float* xh = nullptr;
  const float* xl = nullptr;
  if (a.partitioned) {
    for (int r = 0; r < a.world; ++r) {
      const uint8_t* rb = a.records + (int64_t)r * a.rec_bytes;
      const CandRecord* rec = (const CandRecord*)rb;
      if (rec->key_hi == kh) xh = (const float*)(rb + sizeof(CandRecord));
      if (rec->key_lo == kl) xl = (const float*)(rb + sizeof(CandRecord)) + a.dp;
    }
  } else {
    xh = a.x + ((int64_t)i_hi - a.x_row0) * a.dp;
    xl = a.x + ((int64_t)i_lo - a.x_row0) * a.dp;
  }
  // wave 0 (thread 0 applies the update): same arithmetic as the fused kernels
  const float dist2 = tid < 64 ? wave_dist2(xh, xl, a.dp, tid) : 0.f;

  // ---- 3. alpha update and stop test (one lane) ----
  if (tid == 0) {
    int done = kRunning;
    float c_hi = 0.f, c_lo = 0.f;
    if (!isfinite(b_hi) || !isfinite(b_lo)) {
      done = kNonFinite;
    } else {
      const float k_hl = expf(-a.gamma * dist2);
      const float a_hi_old = a.alpha[i_hi], a_lo_old = a.alpha[i_lo];
      const PairUpdate u = pair_update(a_hi_old, a_lo_old, a.y[i_hi], a.y[i_lo], b_hi, b_lo, k_hl,
                                       a.C, a.tau, a.clip, i_hi == i_lo);
      a.alpha[i_lo] = u.a_lo_new;
      a.alpha[i_hi] = u.a_hi_new;
      c_hi = u.c_hi;
      c_lo = u.c_lo;
      c->iter = c->iter + 1;
      if (!gap_open(b_hi, b_lo, a.eps)) done = kConverged;
      else if (c->iter >= a.max_iter) done = kMaxIter;
    }
    s_i[0] = done;
    s_f[0] = c_hi;
    s_f[1] = c_lo;
  }
  __syncthreads();
  const int done = s_i[0];
  const float c_hi = s_f[0], c_lo = s_f[1];
  if (done == kNonFinite) {
    if (tid == 0) {
      c->done = kNonFinite;
      c->final_applied = 1;
      c->nq = 0;
      c->n_compute = 0;
      c->n_spill = 0;
      c->c_hi = c->c_lo = 0.f;
      c->b_hi = b_hi;
      c->b_lo = b_lo;
      write_status(a, c);
    }
    return;
  }

  // ---- 4. rows needed by the pending f update: hits set the CLOCK bit ----
  if (tid < 2) {
    int key = -1;
    if (tid == 0 && c_hi != 0.f) key = i_hi;
    if (tid == 1 && c_lo != 0.f && !(i_lo == i_hi && c_hi != 0.f)) key = i_lo;
    int line = -1;
    if (key >= 0) {
      line = a.slot_of[key];
      if (line >= 0) a.ref[line] = 1;
    }
    s_i[2 + tid] = key;
    s_i[4 + tid] = line;
  }
  __syncthreads();
  const int need_hi = s_i[2], need_lo = s_i[3];
  const int hit_line_hi = s_i[4], hit_line_lo = s_i[5];
  int m = 0;
  if (need_hi >= 0 && hit_line_hi < 0) ++m;
  if (need_lo >= 0 && hit_line_lo < 0) ++m;
  if (tid == 0) {
    int k = 0;
    if (need_hi >= 0 && hit_line_hi < 0) s_keys[k++] = need_hi;
    if (need_lo >= 0 && hit_line_lo < 0) s_keys[k++] = need_lo;
  }

  // ---- 5. speculation: the X pass is paid anyway -> add the best uncached
  //         workgroup winners (parallel cache check, then ordered rounds) ----
  if (!a.partitioned && a.spec > 0 && m > 0) {
    const int budget = min(min(a.spec, kNQ - m), max(0, a.L / 2 - m));
    if (budget > 0) {
      uint64_t ch = my_h, cl = my_l;
      if (ch != kKeyNone) {
        const int idx = (int)key_index(ch);
        if (idx == i_hi || idx == i_lo || a.slot_of[idx] >= 0) ch = kKeyNone;
      }
      if (cl != kKeyNone) {
        const int idx = (int)key_index(cl);
        if (idx == i_hi || idx == i_lo || a.slot_of[idx] >= 0) cl = kKeyNone;
      }
      int cnt = m;  // thread 0's view of the list length
      if (tid == 0) s_i[6] = m;
      for (int r = 0; r < (budget + 1) / 2; ++r) {
        uint64_t bh = ch, bl = cl;
        block_min2_u64<kFinThreads>(bh, bl, kscr);
        if (bh == kKeyNone && bl == kKeyNone) break;
        if (ch == bh) ch = kKeyNone;
        if (cl == bl) cl = kKeyNone;
        if (tid == 0) {
          const uint64_t cand[2] = {bh, bl};
          for (int s = 0; s < 2; ++s) {
            if (cand[s] == kKeyNone || cnt >= m + budget) continue;
            const int idx = (int)key_index(cand[s]);
            bool dup = false;
            for (int q = 0; q < cnt; ++q) dup |= s_keys[q] == idx;
            if (!dup) s_keys[cnt++] = idx;
          }
          s_i[6] = cnt;
        }
      }
      __syncthreads();
      if (s_i[6] > m) m = s_i[6];
      __syncthreads();
    }
  }
  const int M = m;  // lines to allocate (needed misses first, then speculative)

  // ---- 6. CLOCK allocation of M lines in one parallel window scan ----
  int hand = c->hand;
  if (M > 0) {
    const int W = min(kFinThreads, a.L);
    const int p = (int)(((int64_t)hand + tid) % a.L);
    const bool in_win = tid < W;
    const bool pin = p == hit_line_hi || p == hit_line_lo;
    const int r = in_win ? (int)a.ref[p] : 1;
    const bool elig = in_win && r == 0 && !pin;
    int total = 0;
    const int rank = block_rank(elig, wsum, &total);
    if (elig && rank < M) s_lines[rank] = p;
    if (elig && rank == M - 1) s_i[7] = tid;  // cut: position of the M-th victim
    __syncthreads();
    const int cut = total >= M ? s_i[7] : W - 1;
    if (in_win && tid <= cut && r != 0 && !pin) a.ref[p] = 0;  // second chance consumed
    if (total < M) {
      // every window line was referenced: take the first unpinned, unchosen ones
      const bool chosen = elig && rank < M;
      const bool e2 = in_win && !pin && !chosen;
      int tot2 = 0;
      const int r2 = block_rank(e2, wsum, &tot2);
      if (e2 && total + r2 < M) s_lines[total + r2] = p;
    }
    hand = (int)(((int64_t)hand + cut + 1) % a.L);
    __syncthreads();
  }

  // ---- 7. install the M keys; host-tier fetch / spill decisions ----
  // (wave 0, one lane per query; keys are misses, victims are cached rows, so
  //  no key is both inserted and evicted here)
  int n_spill = 0, n_fetch = 0;
  int hhand = c->hhand;
  if (tid < kNQ) s_hsrc[tid] = (tid < M && a.H > 0) ? a.hslot_of[s_keys[tid]] : -1;
  __syncthreads();
  if (tid < 64) {
    const bool act = tid < M;
    int l = -1, k = -1, old = -1, hsrc = -1;
    if (act) {
      l = s_lines[tid];
      k = s_keys[tid];
      old = a.key_of[l];
      hsrc = s_hsrc[tid];
    }
    const bool want_spill = act && a.H > 0 && old >= 0 && a.hslot_of[old] < 0;
    const uint64_t sm = __ballot(want_spill);
    const int srank = __popcll(sm & ((1ull << tid) - 1ull));
    n_spill = __popcll(sm);
    n_fetch = __popcll(__ballot(hsrc >= 0));
    int hspill = -1;
    if (want_spill && srank < a.H) {  // distinct host lines even when H < kNQ
      const int hl = (int)(((int64_t)hhand + srank) % a.H);
      bool clash = false;  // never overwrite a host line this iteration fetches from
      for (int q = 0; q < M; ++q) clash |= s_hsrc[q] == hl;
      if (!clash) {
        const int prev = a.hkey_of[hl];
        if (prev >= 0) a.hslot_of[prev] = -1;
        a.hkey_of[hl] = old;
        a.hslot_of[old] = hl;
        hspill = hl;
      }
    }
    if (act) {
      if (old >= 0) a.slot_of[old] = -1;
      a.key_of[l] = k;
      a.slot_of[k] = l;
      a.ref[l] = 1;
      c->q_idx[tid] = k;
      c->q_line[tid] = l;
      c->q_op[tid] = hsrc >= 0 ? kOpFetch : kOpCompute;
      c->q_hsrc[tid] = hsrc;
      c->q_hspill[tid] = hspill;
      c->q_sq[tid] = a.xsq[k];
      c->q_ptr[tid] = (a.partitioned ? (k == i_hi ? xh : xl) : a.x + ((int64_t)k - a.x_row0) * a.dp);
    }
    if (a.H > 0) hhand = (int)(((int64_t)hhand + n_spill) % a.H);
    if (tid == 0) {
      s_i[8] = n_spill;
      s_i[9] = n_fetch;
    }
  }
  __syncthreads();

  // ---- 8. publish the control record ----
  if (tid == 0) {
    n_spill = s_i[8];
    n_fetch = s_i[9];
    int line_hi = -1, line_lo = -1, q = 0;
    if (need_hi >= 0) line_hi = hit_line_hi >= 0 ? hit_line_hi : s_lines[q++];
    if (c_lo != 0.f) {
      if (i_lo == i_hi && c_hi != 0.f) line_lo = line_hi;
      else line_lo = hit_line_lo >= 0 ? hit_line_lo : s_lines[q++];
    }
    const int n_need = (need_hi >= 0) + (need_lo >= 0);
    const int n_miss = (need_hi >= 0 && hit_line_hi < 0) + (need_lo >= 0 && hit_line_lo < 0);
    c->done = done;
    c->final_applied = 0;
    c->i_hi = i_hi;
    c->i_lo = i_lo;
    c->c_hi = c_hi;
    c->c_lo = c_lo;
    c->line_hi = line_hi;
    c->line_lo = line_lo;
    c->b_hi = b_hi;
    c->b_lo = b_lo;
    c->nq = M;
    c->n_compute = M - n_fetch;
    c->n_spill = n_spill;
    c->hand = hand;
    c->hhand = hhand;
    c->hits += n_need - n_miss;
    c->misses += n_miss;
    c->rows_computed += M - n_fetch;
    c->x_passes += (M - n_fetch) > 0 ? 1 : 0;
    c->spec_rows += M - n_miss;
    c->host_hits += n_fetch;
    c->spills += n_spill;
    write_status(a, c);
  }
}

// Dense mode in the 3-kernel pipeline is not used (smo_fused covers it).

}  // namespace dev

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
namespace launch {

size_t smo_rows_lds_bytes(int dp) {
  const int kcl = dp < kRowsKC ? dp : kRowsKC;
  return (size_t)kNQ * (kcl + 4) * sizeof(float);
}

void smo_rows(const SmoArgs& a, hipStream_t s) {
  const size_t lds = smo_rows_lds_bytes(a.dp);
  dev::smo_rows_kernel<<<dim3(a.G), kStepThreads, lds, s>>>(a);
  post_launch("smo_rows", s);
}

void smo_step(const SmoArgs& a, hipStream_t s) {
  dev::smo_step_kernel<<<dim3(a.G), kStepThreads, 0, s>>>(a);
  post_launch("smo_step", s);
}

void smo_local_record(const SmoArgs& a, hipStream_t s) {
  dev::smo_local_record_kernel<<<dim3(1), 256, 0, s>>>(a);
  post_launch("smo_local_record", s);
}

void smo_finalize(const SmoArgs& a, hipStream_t s) {
  dev::smo_finalize_kernel<<<dim3(1), kFinThreads, 0, s>>>(a);
  post_launch("smo_finalize", s);
}

}  // namespace launch
}  // namespace dpsvm
