// Fused SMO iteration for the dense (Gram-resident) mode: ONE launch per
// iteration, no finalize kernel and no in-kernel grid synchronisation.
//
// Kernel t:
//   1. every workgroup reads the previous kernel's per-workgroup selection keys
//      (all-reduced across ranks when world > 1) and reduces them to the same
//      global pair (i_hi, i_lo, b_hi, b_lo) — redundantly, deterministically;
//   2. every workgroup computes eta from |x_hi - x_lo|^2 and the alpha update
//      (identical arithmetic everywhere; common.hpp pair_update);
//   3. the f update of its own rows from the resident Gram rows K[i_hi][.],
//      K[i_lo][.] (svmTrain.cu:98-137), I-set classification and the
//      per-workgroup argmin/argmax keys for iteration t+1;
//   4. workgroup 0 commits the PREVIOUS pair's alphas (lazy: nobody reads those
//      two entries from memory in this launch — readers take them from the
//      record) and publishes this pair's record + the host status.
// Reference per-iteration path: svmTrainMain.cpp:235-310 (>= 7 blocking host
// round trips + a TCP Allgather); two kernels + host in the CUDA build.
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

__device__ __forceinline__ void publish_status(SmoStatus* st, int iter, int done, float b_hi, float b_lo) {
  if (!st) return;
  st->iter = iter;
  st->done = done;
  st->b_hi = b_hi;
  st->b_lo = b_lo;
  __atomic_store_n(&st->seq, iter, __ATOMIC_RELEASE);
}

__global__ __launch_bounds__(kFusedThreads) void smo_fused_kernel(SmoArgs a, int mode,
                                                                  const uint64_t* __restrict__ p_in,
                                                                  uint64_t* __restrict__ p_out,
                                                                  const FusedRec* __restrict__ r_in,
                                                                  FusedRec* __restrict__ r_out) {
  __shared__ uint64_t kscr[2 * (kFusedThreads / 64)];
  __shared__ float fscr[kFusedThreads / 64];
  const int tid = threadIdx.x;
  const bool lead = blockIdx.x == 0 && tid == 0;
  const int64_t row0 = (int64_t)blockIdx.x * a.fused_rows;
  const int64_t row_end = min((int64_t)a.nl, row0 + (int64_t)a.fused_rows);

  if (mode == 0) {  // initial selection over the current f / alpha
    uint64_t kh = kKeyNone, kl = kKeyNone;
    for (int64_t j = row0 + tid; j < row_end; j += kFusedThreads) {
      const int64_t g = a.off + j;
      const float fj = a.f[j], av = a.alpha[g], yv = a.y[g];
      if (in_up(av, yv, a.C)) { const uint64_t k = make_key(fj, (uint32_t)g); kh = k < kh ? k : kh; }
      if (in_low(av, yv, a.C)) { const uint64_t k = make_key(-fj, (uint32_t)g); kl = k < kl ? k : kl; }
    }
    block_min2_u64<kFusedThreads>(kh, kl, kscr);
    if (tid == 0) {
      p_out[2 * blockIdx.x] = kh;
      p_out[2 * blockIdx.x + 1] = kl;
    }
    return;
  }

  const FusedRec rin = *r_in;
  if (rin.done != kRunning) {
    if (lead) {
      if (rin.i_hi >= 0) {
        a.alpha[rin.i_lo] = rin.a_lo;
        a.alpha[rin.i_hi] = rin.a_hi;
      }
      FusedRec o = rin;
      o.i_hi = o.i_lo = -1;
      *r_out = o;
      publish_status(a.status, rin.iter, rin.done, rin.b_hi, rin.b_lo);
    }
    return;
  }

  // ---- 1. global pair (redundant in every workgroup) ----
  uint64_t kh = kKeyNone, kl = kKeyNone;
  for (int b = tid; b < a.fused_G; b += kFusedThreads) {
    const uint64_t h = p_in[2 * b], l = p_in[2 * b + 1];
    kh = h < kh ? h : kh;
    kl = l < kl ? l : kl;
  }
  block_min2_u64<kFusedThreads>(kh, kl, kscr);
  if (kh == kKeyNone || kl == kKeyNone) {
    if (lead) {
      if (rin.i_hi >= 0) {
        a.alpha[rin.i_lo] = rin.a_lo;
        a.alpha[rin.i_hi] = rin.a_hi;
      }
      FusedRec o = rin;
      o.i_hi = o.i_lo = -1;
      o.done = kNoPair;
      *r_out = o;
      publish_status(a.status, rin.iter, kNoPair, rin.b_hi, rin.b_lo);
    }
    return;
  }
  const int i_hi = (int)key_index(kh), i_lo = (int)key_index(kl);
  const float b_hi = key_value(kh), b_lo = -key_value(kl);

  // issue the Gram-row loads of this thread's first row early (dense: line = row)
  const int64_t j0 = row0 + tid;
  const float* line_hi = a.lines + (int64_t)i_hi * a.ldl;
  const float* line_lo = a.lines + (int64_t)i_lo * a.ldl;
  float kh0 = 0.f, kl0 = 0.f, f0 = 0.f;
  if (j0 < row_end) {
    kh0 = line_hi[j0];
    kl0 = line_lo[j0];
    f0 = a.f[j0];
  }

  // ---- 2. eta and the alpha update (identical arithmetic in every workgroup) ----
  const float* xh = a.x + ((int64_t)i_hi - a.x_row0) * a.dp;
  const float* xl = a.x + ((int64_t)i_lo - a.x_row0) * a.dp;
  float part = 0.f;
  for (int k = tid; k < a.d; k += kFusedThreads) {
    const float t = xh[k] - xl[k];
    part += t * t;
  }
  const float dist2 = block_sum<kFusedThreads>(part, fscr);
  auto alpha_now = [&](int i) -> float {
    if (i == rin.i_hi) return rin.a_hi;  // pending commit of the previous pair (hi wins)
    if (i == rin.i_lo) return rin.a_lo;
    return a.alpha[i];
  };
  const float a_hi_old = alpha_now(i_hi), a_lo_old = alpha_now(i_lo);
  int done = kRunning;
  float c_hi = 0.f, c_lo = 0.f, a_hi_new = a_hi_old, a_lo_new = a_lo_old;
  const int iter = rin.iter + 1;
  if (!isfinite(b_hi) || !isfinite(b_lo)) {
    done = kNonFinite;
  } else {
    const float k_hl = expf(-a.gamma * dist2);
    const PairUpdate u = pair_update(a_hi_old, a_lo_old, a.y[i_hi], a.y[i_lo], b_hi, b_lo, k_hl, a.C, a.tau,
                                     a.clip, i_hi == i_lo);
    a_hi_new = u.a_hi_new;
    a_lo_new = u.a_lo_new;
    c_hi = u.c_hi;
    c_lo = u.c_lo;
    if (!gap_open(b_hi, b_lo, a.eps)) done = kConverged;
    else if (iter >= a.max_iter) done = kMaxIter;
  }

  // ---- 4. commit previous pair, publish this one ----
  if (lead) {
    if (rin.i_hi >= 0) {
      a.alpha[rin.i_lo] = rin.a_lo;
      a.alpha[rin.i_hi] = rin.a_hi;
    }
    FusedRec o;
    const bool upd = done != kNonFinite;
    o.i_hi = upd ? i_hi : -1;
    o.i_lo = upd ? i_lo : -1;
    o.a_hi = a_hi_new;
    o.a_lo = a_lo_new;
    o.iter = upd ? iter : rin.iter;
    o.done = done;
    o.b_hi = b_hi;
    o.b_lo = b_lo;
    *r_out = o;
    if (done != kRunning || iter % kStatusEvery == 0) publish_status(a.status, o.iter, done, b_hi, b_lo);
  }

  // ---- 3. f update + classification of this workgroup's rows ----
  uint64_t nh = kKeyNone, nlk = kKeyNone;
  for (int64_t j = j0; j < row_end; j += kFusedThreads) {
    float fj, khv, klv;
    if (j == j0) {
      fj = f0; khv = kh0; klv = kl0;
    } else {
      fj = a.f[j]; khv = line_hi[j]; klv = line_lo[j];
    }
    if (c_hi != 0.f || c_lo != 0.f) {
      float delta;
      if (c_hi != 0.f && c_lo != 0.f) delta = (c_hi * khv) + (c_lo * klv);
      else if (c_hi != 0.f) delta = c_hi * khv;
      else delta = c_lo * klv;
      fj += delta;
      a.f[j] = fj;
    }
    if (done == kRunning) {
      const int64_t g = a.off + j;
      float av;
      if (g == i_hi) av = a_hi_new;
      else if (g == i_lo) av = a_lo_new;
      else if (g == rin.i_hi) av = rin.a_hi;
      else if (g == rin.i_lo) av = rin.a_lo;
      else av = a.alpha[g];
      const float yv = a.y[g];
      if (in_up(av, yv, a.C)) { const uint64_t k = make_key(fj, (uint32_t)g); nh = k < nh ? k : nh; }
      if (in_low(av, yv, a.C)) { const uint64_t k = make_key(-fj, (uint32_t)g); nlk = k < nlk ? k : nlk; }
    }
  }
  if (done != kRunning) return;  // uniform
  block_min2_u64<kFusedThreads>(nh, nlk, kscr);
  if (tid == 0) {
    p_out[2 * blockIdx.x] = nh;
    p_out[2 * blockIdx.x + 1] = nlk;
  }
}

}  // namespace dev

namespace launch {

void smo_fused(const SmoArgs& a, int mode, const uint64_t* p_in, uint64_t* p_out, const FusedRec* r_in,
               FusedRec* r_out, hipStream_t s) {
  dev::smo_fused_kernel<<<dim3(a.fused_G), kFusedThreads, 0, s>>>(a, mode, p_in, p_out, r_in, r_out);
  post_launch("smo_fused", s);
}

}  // namespace launch
}  // namespace dpsvm
