// Persistent dense SMO (Gram resident): ONE launch runs up to `steps` SMO
// iterations.  Every workgroup stays resident (grid <= 256 workgroups of 256
// threads, one per CU) and keeps its rows' f, alpha and y in registers; the
// only per-iteration traffic between workgroups is the selection keys,
// exchanged as tagged granules (xch.hpp) — each workgroup publishes its two
// keys to every rank, every workgroup polls all of them.  This replaces the
// kernel boundary (~1.5 us) and the reload of row state of the one-launch-per-
// iteration kernel (smo_fused.hip) with one all-to-all poll.
//
// Iteration t in workgroup b (identical arithmetic to smo_fused.hip, so the
// two paths are bit-identical):
//   1. wave 0 polls the publications tagged t of every workgroup of every rank
//      (each lane watches kB of them, all loads of a round in flight together,
//      a short sleep between rounds): the minima, with the alphas of the rows
//      behind them, broadcast through LDS (barrier 1);
//   2. pair (i_hi, i_lo), eta from the two sample rows, alpha update — the
//      pair's current alphas arrive with the keys from their owners'
//      registers, so alpha memory is never read during the run (a plain or
//      sc1 load could hit a stale line in this XCD's L2);
//   3. f / alpha update of the own rows in registers from the Gram rows
//      K[i_hi][.], K[i_lo][.], classification, per-workgroup keys with their
//      alphas (barrier 2), published tagged t+1.
// Workgroup 0 stores every pair's new alphas as it goes (every rank computes
// every pair: the full alpha vector on every rank; nobody reads it before the
// launch ends); at exit every workgroup writes its own rows' f.
// Reference per-iteration path: svmTrainMain.cpp:235-310.
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "xch.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

constexpr int kPersistMaxRows = 12;  // rows per thread (fused_rows <= 3072); kR = 4 up to 1024 rows

// kSys: system-scope exchange (ranks on other devices / processes); kB: poll
// batch, publications watched per lane per round (xch.hpp).  One poll loop per
// instantiation: no dispatch inside the iteration.
template <bool kSys, int kB, int kR>
__global__ __launch_bounds__(kFusedThreads) void smo_persist_kernel(SmoArgs a, FusedRec* __restrict__ st, int steps) {
  static_assert(kFusedThreads == 256, "4 waves assumed");
  __shared__ uint64_t kscr[8];
  __shared__ float kfs[8];
  __shared__ XKeys pair_s;
  __shared__ int fail_s;
  __shared__ float d2_s;
  if (steps < 0) {  // residency census (setup): this kernel, this grid
    census_arrive(a.census, a.census_ticks);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool lead = blockIdx.x == 0 && tid == 0;
  const int rpt = a.fused_rows / kFusedThreads;  // rows per thread
  const int64_t row0 = (int64_t)blockIdx.x * a.fused_rows;
  const int64_t row_end = min((int64_t)a.nl, row0 + (int64_t)a.fused_rows);

  float f[kR], al[kR], yv[kR];
  bool has[kR];
#pragma unroll
  for (int k = 0; k < kR; ++k) {
    const int64_t j = row0 + tid + (int64_t)k * kFusedThreads;
    has[k] = k < rpt && j < row_end;
    f[k] = has[k] ? a.f[j] : 0.f;
    al[k] = has[k] ? a.alpha[a.off + j] : 0.f;
    yv[k] = has[k] ? a.y[a.off + j] : 0.f;
  }
  const FusedRec s0 = *st;
  if (s0.done != kRunning) return;
  // exchange endpoints, loaded once (wave 0 polls and publishes)
  const uint64_t* my_buf = a.xpeer[a.xrank];
  uint64_t* peer_buf = wave == 0 ? xch_peer(a, lane) : nullptr;
  int t = s0.iter, done = kRunning;
  float b_hi = s0.b_hi, b_lo = s0.b_lo;

  // diagnostics (DPSVM_STAMPS): thread 0 of workgroups 0 and G-1 keeps 6
  // s_memrealtime stamps per iteration in registers and stores them after
  // publishing (0 poll start, 1 pair known, 2 alpha update, 3 f update,
  // 4 keys reduced, 5 published)
  const bool stamping = a.stamps != nullptr && tid == 0 && (blockIdx.x == 0 || blockIdx.x == a.fused_G - 1);
  uint64_t stv[6] = {0, 0, 0, 0, 0, 0};
#define PSTAMP(i) \
  if (stamping) stv[i] = __builtin_amdgcn_s_memrealtime()
  for (int step = 0; step < steps; ++step) {
    PSTAMP(0);
    // ---- 1. publications tagged t+1 (produced by iteration t) ----
    const uint32_t tag = (uint32_t)t + 1u;
    if (wave == 0) {
      XKeys m = xk_none();
      const bool ok = xch_poll_wave_t<kSys, kB>(a, my_buf, (int)(tag & 1u), tag, m, lane);
      m = wave_min_xk(m);
      if (lane == 0) {
        pair_s = m;
        fail_s = ok ? 0 : 1;
      }
    }
    __syncthreads();
    const XKeys pk = pair_s;
    if (fail_s) {
      done = kCommFail;
      break;
    }
    if (pk.kh == kKeyNone || pk.kl == kKeyNone) {
      done = kNoPair;
      break;
    }
    const int i_hi = (int)key_index(pk.kh), i_lo = (int)key_index(pk.kl);
    const float bh = key_value(pk.kh), bl = -key_value(pk.kl);
    PSTAMP(1);

    // ---- 2. one round trip: Gram rows of the own rows, sample rows ----
    const float* line_hi = a.lines + (int64_t)i_hi * a.ldl;
    const float* line_lo = a.lines + (int64_t)i_lo * a.ldl;
    // unconditional loads (absent rows read the first own row): no exec-mask
    // branches between them, so every load of the round trip is in flight together
    float khv[kR], klv[kR];
#pragma unroll
    for (int k = 0; k < kR; ++k) {
      const int64_t j = has[k] ? row0 + tid + (int64_t)k * kFusedThreads : row0;
      khv[k] = line_hi[j];
      klv[k] = line_lo[j];
    }
    const float y_hi = a.y[i_hi], y_lo = a.y[i_lo];  // read-only during the run
    float k_hl;
    if (a.eta_gram) {
      // K(hi, lo) straight from the resident Gram (every column local): one
      // more load of the same round trip, no sample-row reads, no barrier.
      // The GEMM's |x|^2 expansion rounds differently from the explicit
      // difference below, so the trajectory matches to tolerance, not bits.
      k_hl = line_hi[i_lo - a.off];
    } else {
      const float* xh = a.x + ((int64_t)i_hi - a.x_row0) * a.dp;
      const float* xl = a.x + ((int64_t)i_lo - a.x_row0) * a.dp;
      // wave 0 alone reads the two sample rows (one copy of their traffic per
      // workgroup instead of four: with every workgroup on the same two rows the
      // replicated loads delayed the slowest publisher) and shares |x_hi - x_lo|^2
      // through LDS; the other waves' Gram-row loads are in flight meanwhile
      if (wave == 0) {
        const float d2 = wave_dist2(xh, xl, a.dp, lane);  // same tree as every other engine
        if (lane == 0) d2_s = d2;
      }
      __syncthreads();
      k_hl = expf(-a.gamma * d2_s);
    }
    const float a_hi_old = pk.ah, a_lo_old = pk.al;     // the owners' current values
    float c_hi = 0.f, c_lo = 0.f, a_hi_new = a_hi_old, a_lo_new = a_lo_old;
    const int iter = t + 1;
    if (!isfinite(bh) || !isfinite(bl)) {
      done = kNonFinite;
    } else {
      const PairUpdate u =
          pair_update(a_hi_old, a_lo_old, y_hi, y_lo, bh, bl, k_hl, a.C, a.tau, a.clip, i_hi == i_lo);
      a_hi_new = u.a_hi_new;
      a_lo_new = u.a_lo_new;
      c_hi = u.c_hi;
      c_lo = u.c_lo;
      if (!gap_open(bh, bl, a.eps)) done = kConverged;
      else if (iter >= a.max_iter) done = kMaxIter;
    }
    b_hi = bh;
    b_lo = bl;
    PSTAMP(2);
    if (done == kNonFinite) break;
    if (lead) {  // alpha memory is write-only during the run (read after the launch)
      a.alpha[i_lo] = a_lo_new;
      a.alpha[i_hi] = a_hi_new;  // hi written last (svmTrainMain.cpp:298-299)
    }
    t = iter;

    // ---- 3. f update + classification of the own rows ----
    const bool upd_f = c_hi != 0.f || c_lo != 0.f;
    XKeys nk = xk_none();
#pragma unroll
    for (int k = 0; k < kR; ++k) {
      if (!has[k]) continue;
      const int64_t g = a.off + row0 + tid + (int64_t)k * kFusedThreads;
      if (upd_f) f[k] = f_apply(f[k], c_hi, khv[k], c_lo, klv[k]);
      if (g == i_lo) al[k] = a_lo_new;
      if (g == i_hi) al[k] = a_hi_new;  // hi wins when i_hi == i_lo
      if (in_up(al[k], yv[k], a.C)) xk_min(nk, XKeys{make_key(f[k], (uint32_t)g), kKeyNone, al[k], 0.f});
      if (in_low(al[k], yv[k], a.C)) xk_min(nk, XKeys{kKeyNone, make_key(-f[k], (uint32_t)g), 0.f, al[k]});
    }
    PSTAMP(3);
    if (done != kRunning) break;  // uniform: the last update is applied, no keys needed

    nk = wave_min_xk(nk);
    if (lane == 0) {
      kscr[wave] = nk.kh;
      kscr[4 + wave] = nk.kl;
      kfs[wave] = nk.ah;
      kfs[4 + wave] = nk.al;
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int w = 1; w < kFusedThreads / 64; ++w) xk_min(nk, XKeys{kscr[w], kscr[4 + w], kfs[w], kfs[4 + w]});
      PSTAMP(4);
      const uint32_t otag = (uint32_t)t + 1u;
      xch_push(a, peer_buf, (int)(otag & 1u), blockIdx.x, nk, otag, lane);
      PSTAMP(5);
      if (stamping) {
        uint64_t* dst = a.stamps + ((size_t)(t % kStampRing) * 2 + (blockIdx.x == 0 ? 0 : 1)) * kStampSlots;
#pragma unroll
        for (int i = 0; i < 6; ++i) dst[i] = stv[i];
      }
    }
  }
#undef PSTAMP

  // ---- exit: own rows' f back to memory; workgroup 0 writes the state ----
#pragma unroll
  for (int k = 0; k < kR; ++k) {
    const int64_t j = row0 + tid + (int64_t)k * kFusedThreads;
    if (has[k]) a.f[j] = f[k];
  }
  if (lead) {
    FusedRec o;
    o.i_hi = o.i_lo = -1;
    o.a_hi = o.a_lo = 0.f;
    o.iter = t;
    o.done = done;
    o.b_hi = b_hi;
    o.b_lo = b_lo;
    *st = o;
    if (a.status) {
      SmoStatus* s = a.status;
      s->iter = t;
      s->done = done;
      s->b_hi = b_hi;
      s->b_lo = b_lo;
      __atomic_store_n(&s->seq, t, __ATOMIC_RELEASE);
    }
  }
}

}  // namespace dev

namespace launch {

void preload_persist_kernel(hipStream_t s) {
  // trivial launch (no rows, state "done"): loads the code object and exits
  FusedRec* st = nullptr;
  HIP_CHECK(hipMalloc((void**)&st, sizeof(FusedRec)));
  FusedRec h{};
  h.done = kConverged;
  HIP_CHECK(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, s));
  SmoArgs z{};
  z.fused_G = 1;
  z.fused_rows = kFusedThreads;
  dev::smo_persist_kernel<false, 1, 4><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<false, 2, 4><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<false, 4, 4><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<true, 1, 4><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<true, 2, 4><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<true, 4, 4><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<false, 1, dev::kPersistMaxRows><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<false, 2, dev::kPersistMaxRows><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<false, 4, dev::kPersistMaxRows><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<true, 1, dev::kPersistMaxRows><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<true, 2, dev::kPersistMaxRows><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  dev::smo_persist_kernel<true, 4, dev::kPersistMaxRows><<<1, kFusedThreads, 0, s>>>(z, st, 0);
  HIP_CHECK(hipStreamSynchronize(s));
  HIP_CHECK(hipGetLastError());
  (void)hipFree(st);
}

// The instantiation a launch of `a` runs: (scope, poll batch, register rows).
using PersistFn = void (*)(SmoArgs, FusedRec*, int);
template <int kR>
static PersistFn persist_fn_r(bool sys, int kb) {
  if (sys) return kb == 1 ? dev::smo_persist_kernel<true, 1, kR> : kb == 2 ? dev::smo_persist_kernel<true, 2, kR>
                                                                           : dev::smo_persist_kernel<true, 4, kR>;
  return kb == 1 ? dev::smo_persist_kernel<false, 1, kR> : kb == 2 ? dev::smo_persist_kernel<false, 2, kR>
                                                                   : dev::smo_persist_kernel<false, 4, kR>;
}
static PersistFn persist_fn(const SmoArgs& a) {
  const int E = a.xworld * a.fused_G;
  const int kb = a.xpoll_kb > 0 ? a.xpoll_kb : (E <= 64 ? 1 : E <= 128 ? 2 : 4);
  // rows per thread: 4 (<= 1024 rows per workgroup, the headline geometry) or 12
  return a.fused_rows <= 4 * kFusedThreads ? persist_fn_r<4>(a.xworld > 1, kb)
                                           : persist_fn_r<dev::kPersistMaxRows>(a.xworld > 1, kb);
}

int poll_batch(const SmoArgs& a) {
  const int E = a.xworld * a.fused_G;
  return a.xpoll_kb > 0 ? a.xpoll_kb : (E <= 64 ? 1 : E <= 128 ? 2 : 4);
}

int smo_persist_blocks_per_cu(const SmoArgs& a) {
  int nb = 0;
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)persist_fn(a), kFusedThreads, 0));
  return nb;
}

void smo_persist_census(const SmoArgs& a, int groups, hipStream_t s) {
  PersistFn fn = persist_fn(a);
  fn<<<dim3(groups), kFusedThreads, 0, s>>>(a, nullptr, -1);
  post_launch("smo_persist census", s);
}

void smo_persist(const SmoArgs& a, FusedRec* st, int steps, hipStream_t s) {
  DPSVM_CHECK(a.xworld >= 1 && a.fused_G <= 256 && a.fused_rows <= dev::kPersistMaxRows * kFusedThreads,
              "persistent SMO needs the key exchange and <= 256 resident workgroups");
  PersistFn fn = persist_fn(a);
  fn<<<dim3(a.fused_G), kFusedThreads, 0, s>>>(a, st, steps);
  post_launch("smo_persist", s);
}

}  // namespace launch
}  // namespace dpsvm
