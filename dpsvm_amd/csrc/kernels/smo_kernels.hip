// SMO iteration kernels for MI355X (gfx950, wave64).
//
//   smo_rows      LRU cache misses: K rows of up to 16 query vectors over the
//                 local shard in ONE pass over X, fp32 MFMA 16x16x4 (exact f32),
//                 query vectors staged in LDS, fused expansion + exp epilogue.
//                 Replaces the reference's per-miss cublasSgemv x2 on two
//                 streams (svmTrain.cu:212-249, K3/K4) and the Thrust functor
//                 that turned dot products into RBF values (K5).
//   smo_step      pending f update (svmTrain.cu:98-137) fused with I-set
//                 classification and the argmin/argmax selection
//                 (svmTrain.cu:41-95 + 400-483): per-workgroup u64 keys.
//   smo_finalize  one workgroup: global pair, eta from the two sample rows on
//                 device (was host CBLAS, svmTrain.cu:696-714), alpha update and
//                 clip (svmTrainMain.cpp:282-299), stop test, device LRU
//                 bookkeeping (was host std::map/list, cache.cu:62-105), next
//                 iteration's row requests, host-mapped status record.
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// ---------------------------------------------------------------------------
// setup kernels
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void row_sqnorm_kernel(const float* __restrict__ x, int64_t n,
                                                         int d, int ld, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* r = x + row * (int64_t)ld;
  float s = 0.f;
  for (int k = lane; k < d; k += 64) s += r[k] * r[k];
  s = wave_sum(s);
  if (lane == 0) out[row] = s;
}

__global__ void init_f_kernel(const float* __restrict__ y, int64_t off, int64_t nl,
                              float* __restrict__ f) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nl) f[j] = -y[off + j];  // f = -y (svmTrain.cu:380)
}

__global__ void fill_i32_kernel(int32_t* p, int64_t n, int32_t v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// ---------------------------------------------------------------------------
// smo_rows: K(q, j) for the ctrl->nq requested rows q and every local row j.
// Grid: G workgroups x 256 threads; each wave owns two 16-row tiles.
// MFMA 16x16x4 f32 operand map: A lane l -> (row l&15, k l>>4), B lane l ->
// (k l>>4, query l&15).  Each lane loads a float4 of X (16 contiguous columns
// per 16 rows and wave-instruction); component c of the float4 feeds MFMA c, a
// permutation of k that the query operand (LDS, same float4) mirrors.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kStepThreads) void smo_rows_kernel(SmoArgs a) {
  const SmoCtrl* c = a.ctrl;
  const int nq = c->nq;
  if (nq == 0 || (c->done != kRunning && c->final_applied)) return;
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t row0 = (int64_t)blockIdx.x * kStepRows + wave * 32;
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
      if (q < nq) v = *(const f4*)(c->q_ptr[q] + kc + 4 * k4);
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
  if (q < nq) {
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
        float delta;
        if (ch != 0.f && cl != 0.f)
          delta = (ch * a.lines[(int64_t)c->line_hi * a.ldl + j]) +
                  (cl * a.lines[(int64_t)c->line_lo * a.ldl + j]);
        else if (ch != 0.f)
          delta = ch * a.lines[(int64_t)c->line_hi * a.ldl + j];
        else
          delta = cl * a.lines[(int64_t)c->line_lo * a.ldl + j];
        fj += delta;
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
// smo_finalize: one workgroup, identical on every rank.
// ---------------------------------------------------------------------------
struct Lru {
  int32_t head, tail, used;
};

__device__ void lru_unlink(const SmoArgs& a, Lru& s, int l) {
  const int p = a.lru_prev[l], nx = a.lru_next[l];
  if (p >= 0) a.lru_next[p] = nx; else s.head = nx;
  if (nx >= 0) a.lru_prev[nx] = p; else s.tail = p;
}
__device__ void lru_push_front(const SmoArgs& a, Lru& s, int l) {
  a.lru_prev[l] = -1;
  a.lru_next[l] = s.head;
  if (s.head >= 0) a.lru_prev[s.head] = l;
  s.head = l;
  if (s.tail < 0) s.tail = l;
}
// returns line; *hit set; on miss the line is (re)assigned to `key` (LRU victim)
__device__ int lru_get(const SmoArgs& a, Lru& s, int key, bool* hit) {
  int l = a.slot_of[key];
  if (l >= 0) {
    *hit = true;
    if (s.head != l) {
      lru_unlink(a, s, l);
      lru_push_front(a, s, l);
    }
    return l;
  }
  *hit = false;
  if (s.used < a.L) {
    l = s.used++;
  } else {
    l = s.tail;
    lru_unlink(a, s, l);
    const int old = a.key_of[l];
    if (old >= 0) a.slot_of[old] = -1;
  }
  a.key_of[l] = key;
  a.slot_of[key] = l;
  lru_push_front(a, s, l);
  return l;
}

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
  st->spec_hits = c->spec_hits;
  __atomic_store_n(&st->seq, c->iter, __ATOMIC_RELEASE);
}

__global__ __launch_bounds__(kFinThreads) void smo_finalize_kernel(SmoArgs a) {
  __shared__ uint64_t kscratch[2 * (kFinThreads / 64)];
  __shared__ float fscratch[kFinThreads / 64];
  __shared__ int s_nq;
  __shared__ int32_t s_qidx[kNQ];
  SmoCtrl* c = a.ctrl;
  const int tid = threadIdx.x;
  const int done_in = c->done;
  if (done_in != kRunning) {
    __syncthreads();
    if (tid == 0 && !c->final_applied) {
      c->final_applied = 1;
      c->nq = 0;
      c->c_hi = 0.f;
      c->c_lo = 0.f;
      write_status(a, c);
    }
    return;
  }

  // ---- 1. global selection ----
  uint64_t kh = kKeyNone, kl = kKeyNone;
  if (a.partitioned) {
    for (int r = tid; r < a.world; r += kFinThreads) {
      const CandRecord* rec = (const CandRecord*)(a.records + (int64_t)r * a.rec_bytes);
      kh = rec->key_hi < kh ? rec->key_hi : kh;
      kl = rec->key_lo < kl ? rec->key_lo : kl;
    }
  } else {
    for (int b = tid; b < a.G; b += kFinThreads) {
      const uint64_t h = a.partials[2 * b], l = a.partials[2 * b + 1];
      kh = h < kh ? h : kh;
      kl = l < kl ? l : kl;
    }
  }
  block_min2_u64<kFinThreads>(kh, kl, kscratch);

  if (kh == kKeyNone || kl == kKeyNone) {
    if (tid == 0) {
      c->done = kNoPair;
      c->final_applied = 1;
      c->nq = 0;
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
  float part = 0.f;
  for (int k = tid; k < a.d; k += kFinThreads) {
    const float t = xh[k] - xl[k];
    part += t * t;
  }
  const float dist2 = block_sum<kFinThreads>(part, fscratch);

  // ---- 3. alpha update, stop test, cache requests (one lane) ----
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
      const int iter = c->iter + 1;
      c->iter = iter;
      if (!gap_open(b_hi, b_lo, a.eps)) done = kConverged;
      else if (iter >= a.max_iter) done = kMaxIter;
    }
    int nq = 0;
    int line_hi = -1, line_lo = -1;
    int64_t hits = c->hits, misses = c->misses;
    if (done != kNonFinite) {
      if (a.cache_mode == kCacheDense) {
        if (c_hi != 0.f) { line_hi = i_hi; ++hits; }
        if (c_lo != 0.f) { line_lo = i_lo; ++hits; }
      } else {
        Lru s{c->lru_head, c->lru_tail, c->lines_used};
        bool hit;
        if (c_hi != 0.f) {
          line_hi = lru_get(a, s, i_hi, &hit);
          if (hit) ++hits;
          else {
            ++misses;
            c->q_idx[nq] = i_hi;
            c->q_line[nq] = line_hi;
            c->q_ptr[nq] = xh;
            c->q_sq[nq] = a.xsq[i_hi];
            ++nq;
          }
        }
        if (c_lo != 0.f) {
          if (i_lo == i_hi && line_hi >= 0) {
            line_lo = line_hi;
          } else {
            line_lo = lru_get(a, s, i_lo, &hit);
            if (hit) ++hits;
            else {
              ++misses;
              c->q_idx[nq] = i_lo;
              c->q_line[nq] = line_lo;
              c->q_ptr[nq] = xl;
              c->q_sq[nq] = a.xsq[i_lo];
              ++nq;
            }
          }
        }
        c->lru_head = s.head;
        c->lru_tail = s.tail;
        c->lines_used = s.used;
      }
    } else {
      c_hi = c_lo = 0.f;
    }
    c->done = done;
    c->final_applied = (done == kNonFinite) ? 1 : 0;
    c->i_hi = i_hi;
    c->i_lo = i_lo;
    c->c_hi = c_hi;
    c->c_lo = c_lo;
    c->line_hi = line_hi;
    c->line_lo = line_lo;
    c->b_hi = b_hi;
    c->b_lo = b_lo;
    c->hits = hits;
    c->misses = misses;
    if (nq > 0) {
      c->rows_computed += nq;
      c->x_passes += 1;
    }
    c->nq = nq;
    s_nq = nq;
    for (int q = 0; q < nq; ++q) s_qidx[q] = c->q_idx[q];
  }
  __syncthreads();

  // ---- 4. speculative rows (LRU, replicated X): the X pass is paid anyway,
  //      so fill the idle MFMA columns with the best uncached block winners ----
  int nq = s_nq;
  if (a.cache_mode == kCacheLRU && !a.partitioned && a.spec > 0 && nq > 0) {
    const int budget = min(min(a.spec, kNQ - nq), a.L / 2 - nq);
    // each thread holds the partial keys of its blocks (both sides, as copies)
    int rounds = 0;
    uint64_t mine_h = kKeyNone, mine_l = kKeyNone;  // min over this thread's untaken keys
    // thread owns blocks tid, tid+1024, ...; G is typically <= 1024 per rank
    auto recompute = [&](uint64_t taken_h, uint64_t taken_l) {
      uint64_t h = kKeyNone, l = kKeyNone;
      for (int b = tid; b < a.G; b += kFinThreads) {
        const uint64_t ph = a.partials[2 * b], pl = a.partials[2 * b + 1];
        if (ph > taken_h && ph < h) h = ph;
        if (pl > taken_l && pl < l) l = pl;
      }
      mine_h = h;
      mine_l = l;
    };
    // keys are distinct; "taken" = every key <= the last selected one on that side
    uint64_t last_h = kh, last_l = kl;  // the current pair is already handled
    int added = 0;
    while (added < budget && rounds < 2 * kNQ) {
      ++rounds;
      recompute(last_h, last_l);
      uint64_t bh = mine_h, bl = mine_l;
      block_min2_u64<kFinThreads>(bh, bl, kscratch);
      if (bh == kKeyNone && bl == kKeyNone) break;
      if (tid == 0) {
        Lru s{c->lru_head, c->lru_tail, c->lines_used};
        const uint64_t cand[2] = {bh, bl};
        for (int side = 0; side < 2 && added < budget; ++side) {
          if (cand[side] == kKeyNone) continue;
          const int idx = (int)key_index(cand[side]);
          if (a.slot_of[idx] >= 0) continue;  // cached already
          bool dup = false;
          for (int q = 0; q < s_nq; ++q) dup |= (s_qidx[q] == idx);
          if (dup) continue;
          bool hit;
          const int line = lru_get(a, s, idx, &hit);
          c->q_idx[s_nq] = idx;
          c->q_line[s_nq] = line;
          c->q_ptr[s_nq] = a.x + ((int64_t)idx - a.x_row0) * a.dp;
          c->q_sq[s_nq] = a.xsq[idx];
          s_qidx[s_nq] = idx;
          ++s_nq;
          ++added;
        }
        c->lru_head = s.head;
        c->lru_tail = s.tail;
        c->lines_used = s.used;
      }
      last_h = bh;
      last_l = bl;
      __syncthreads();
    }
    if (tid == 0 && added > 0) {
      c->nq = s_nq;
      c->rows_computed += added;
      c->spec_rows += added;
    }
  }
  if (tid == 0) write_status(a, c);
}

// ---------------------------------------------------------------------------
// SV compaction (K11 replacement: thrust::remove_if over a 4-zip)
// ---------------------------------------------------------------------------
constexpr int kCompactBlock = 1024;

__global__ __launch_bounds__(kCompactBlock) void compact_count_kernel(const float* alpha, int64_t n,
                                                                      int32_t* counts) {
  __shared__ int32_t wc[kCompactBlock / 64];
  const int64_t i = (int64_t)blockIdx.x * kCompactBlock + threadIdx.x;
  const bool p = i < n && alpha[i] > 0.f;
  const uint64_t m = __ballot(p);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t s = 0;
    for (int w = 0; w < kCompactBlock / 64; ++w) s += wc[w];
    counts[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(1024) void compact_scan_kernel(int32_t* counts, int nb, int32_t* total) {
  // single workgroup exclusive scan (sequential chunks per thread + LDS scan)
  __shared__ int32_t part[1024];
  const int per = (nb + 1023) / 1024;
  const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
  int32_t s = 0;
  for (int b = b0; b < b1; ++b) s += counts[b];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t run = 0;
    for (int t = 0; t < 1024; ++t) {
      int32_t v = part[t];
      part[t] = run;
      run += v;
    }
    *total = run;
  }
  __syncthreads();
  int32_t run = part[threadIdx.x];
  for (int b = b0; b < b1; ++b) {
    int32_t v = counts[b];
    counts[b] = run;
    run += v;
  }
}

__global__ __launch_bounds__(kCompactBlock) void compact_scatter_kernel(const float* alpha, int64_t n,
                                                                        const int32_t* offsets,
                                                                        int32_t* idx_out) {
  __shared__ int32_t wc[kCompactBlock / 64];
  const int64_t i = (int64_t)blockIdx.x * kCompactBlock + threadIdx.x;
  const bool p = i < n && alpha[i] > 0.f;
  const uint64_t m = __ballot(p);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) wc[wave] = __popcll(m);
  __syncthreads();
  int32_t base = offsets[blockIdx.x];
  for (int w = 0; w < wave; ++w) base += wc[w];
  const int32_t rank = __popcll(m & ((1ull << lane) - 1ull));
  if (p) idx_out[base + rank] = (int32_t)i;
}

__global__ void gather_sv_kernel(const float* x, int64_t x_row0, const float* xsq, const float* alpha,
                                 const float* y, const int32_t* idx, int64_t nsv, int dp, float* sv,
                                 float* svsq, float* coef) {
  const int64_t r = blockIdx.x;
  if (r >= nsv) return;
  const int64_t g = idx[r];
  const float* src = x + (g - x_row0) * dp;
  for (int k = threadIdx.x; k < dp; k += blockDim.x) sv[r * dp + k] = src[k];
  if (threadIdx.x == 0) {
    svsq[r] = xsq[g];
    coef[r] = alpha[g] * y[g];
  }
}

}  // namespace dev

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
namespace launch {

void row_sqnorm(const float* x, int64_t n, int d, int ld, float* out, hipStream_t s) {
  if (n <= 0) return;
  dev::row_sqnorm_kernel<<<dim3((unsigned)((n + 3) / 4)), 256, 0, s>>>(x, n, d, ld, out);
  post_launch("row_sqnorm", s);
}

void init_f(const float* y, int64_t off, int64_t nl, float* f, hipStream_t s) {
  if (nl <= 0) return;
  dev::init_f_kernel<<<dim3((unsigned)((nl + 255) / 256)), 256, 0, s>>>(y, off, nl, f);
  post_launch("init_f", s);
}

void fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t s) {
  if (n <= 0) return;
  dev::fill_i32_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, s>>>(p, n, v);
  post_launch("fill_i32", s);
}

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

int64_t compact_scratch_ints(int64_t n) { return (n + dev::kCompactBlock - 1) / dev::kCompactBlock + 1; }

void compact_positive(const float* alpha, int64_t n, int32_t* idx_out, int32_t* count_dev,
                      int32_t* scratch, hipStream_t s) {
  const int nb = (int)((n + dev::kCompactBlock - 1) / dev::kCompactBlock);
  dev::compact_count_kernel<<<dim3(nb), dev::kCompactBlock, 0, s>>>(alpha, n, scratch);
  post_launch("compact_count", s);
  dev::compact_scan_kernel<<<dim3(1), 1024, 0, s>>>(scratch, nb, count_dev);
  post_launch("compact_scan", s);
  dev::compact_scatter_kernel<<<dim3(nb), dev::kCompactBlock, 0, s>>>(alpha, n, scratch, idx_out);
  post_launch("compact_scatter", s);
}

void gather_sv(const float* x, int64_t x_row0, const float* xsq, const float* alpha,
               const float* y, const int32_t* idx, int64_t nsv, int dp, float* sv, float* svsq,
               float* coef, hipStream_t s) {
  if (nsv <= 0) return;
  dev::gather_sv_kernel<<<dim3((unsigned)nsv), 256, 0, s>>>(x, x_row0, xsq, alpha, y, idx, nsv, dp,
                                                           sv, svsq, coef);
  post_launch("gather_sv", s);
}

}  // namespace launch
}  // namespace dpsvm
