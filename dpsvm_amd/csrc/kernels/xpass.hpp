// One workgroup's share of an X pass: K(x_q, x_j) for up to kNQ query rows q
// against the workgroup's own rows j, written into the query rows' cache lines.
// Shared by the fused cache engine (smo_fused_lru.hip) and the persistent cache
// engine (smo_persist_lru.hip): one arithmetic (same k order as smo_rows), so
// every engine produces bit-identical kernel rows.
// Reference: one cublasSgemv per missed row over the local rows
// (svmTrain.cu:212-249) + the exp of update_functor (svmTrain.cu:128-130).
#pragma once

#include <hip/hip_runtime.h>

#include "dpsvm/device_state.hpp"
#include "device_util.hpp"

namespace dpsvm {
namespace dev {

// LDS floats of an X pass: kNQ staged query vectors (k-chunks of kRowsKC) +
// |x_j|^2 of up to fused_rows own rows
__host__ __device__ constexpr size_t xpass_lds_floats(int dp, int fused_rows) {
  return (size_t)kNQ * ((dp < kRowsKC ? dp : kRowsKC) + 4) + (size_t)fused_rows;
}

// Fill rows [row0, row_end) of lines line[q] for every q < n_new with
// op[q] == kOpCompute (key / line / op: uniform, e.g. LDS).  wsm: xpass_lds_floats
// of dynamic LDS; its tail holds the own rows' |x_j|^2, staged here unless
// xsq_staged.  16 query rows per pass on v_mfma_f32_16x16x4_f32, X loads in
// batches of 4 k-steps x 4 tiles (16 KiB per wave in flight: one workgroup per
// CU, the pass is HBM-latency bound without deep prefetch).  No trailing
// barrier: callers synchronise before reading the new segments.
__device__ __forceinline__ void xpass_fill(const SmoArgs& a, int64_t row0, int64_t row_end, int n_new,
                                           const int* key, const int* line, const int* op, float* wsm,
                                           bool xsq_staged) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int dp = a.dp;
  const int q = lane & 15;
  const bool qv = q < n_new && op[q] == kOpCompute;
  const float wsq = qv ? a.xsq[key[q]] : 0.f;
  const int64_t xbase = a.off - a.x_row0;
  const int npass = (int)((row_end - row0 + 255) / 256);
  float* xsq_s = wsm + kNQ * ((dp < kRowsKC ? dp : kRowsKC) + 4);  // [fused_rows] |x_j|^2 of own rows
  // sched_barrier keeps the scheduler from sinking the loads back next to
  // their MFMAs.  Same k order as smo_rows: bit-identical rows.
  f4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = (f4){0.f, 0.f, 0.f, 0.f};
  auto xrow = [&](int pass) {
    return a.x + (xbase + row0 + (int64_t)pass * 256 + wave * 64 + (lane & 15)) * dp + 4 * (lane >> 4);
  };
  auto load = [&](f4 (&v)[4][4], const float* xk, int k) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) v[s][t] = *(const f4*)(xk + (int64_t)t * 16 * dp + k + 16 * s);
  };
  auto comp = [&](const f4 (&v)[4][4], const float* wr, int k) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f4 wv = *(const f4*)(wr + k + 16 * s);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[t] = mfma16(v[s][t].x, wv.x, acc[t]);
        acc[t] = mfma16(v[s][t].y, wv.y, acc[t]);
        acc[t] = mfma16(v[s][t].z, wv.z, acc[t]);
        acc[t] = mfma16(v[s][t].w, wv.w, acc[t]);
      }
    }
  };
  auto comp16 = [&](const float* xk, const float* wr, int k0, int k1) {  // 16-wide k-steps [k0, k1)
    for (int k = k0; k < k1; k += 16) {
      const f4 wv = *(const f4*)(wr + k);
      f4 xv[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) xv[t] = *(const f4*)(xk + (int64_t)t * 16 * dp + k);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[t] = mfma16(xv[t].x, wv.x, acc[t]);
        acc[t] = mfma16(xv[t].y, wv.y, acc[t]);
        acc[t] = mfma16(xv[t].z, wv.z, acc[t]);
        acc[t] = mfma16(xv[t].w, wv.w, acc[t]);
      }
    }
  };
  auto epilogue = [&](int pass) {  // K values of this pass's 256 rows -> the new lines
    if (qv) {
      float* out = a.lines + (int64_t)line[q] * a.ldl + row0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int rel = pass * 256 + wave * 64 + t * 16 + (lane >> 4) * 4;
        f4 kv;
#pragma unroll
        for (int r = 0; r < 4; ++r) kv[r] = rbf_from_dot(xsq_s[rel + r], wsq, acc[t][r], a.gamma);
        *(f4*)(out + rel) = kv;
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = (f4){0.f, 0.f, 0.f, 0.f};
  };
  // own rows' |x|^2 staged once (one round trip instead of one per pass)
  if (!xsq_staged)
    for (int i = tid; i < npass * 256; i += kFusedThreads) xsq_s[i] = a.xsq[a.off + row0 + i];
  if (dp <= kRowsKC) {
    // single staged chunk: the batch sequence runs across passes, so the
    // next pass's first X batch is in flight during this pass's epilogue
    const int ldw = dp + 4, k4n = dp >> 2;
    for (int i = tid; i < kNQ * k4n; i += kFusedThreads) {
      const int qq = i / k4n, k4 = i - qq * k4n;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (qq < n_new && op[qq] == kOpCompute) v = *(const f4*)(a.x + ((int64_t)key[qq] - a.x_row0) * dp + 4 * k4);
      *(f4*)(wsm + qq * ldw + 4 * k4) = v;
    }
    __syncthreads();
    const float* wr = wsm + q * ldw + 4 * (lane >> 4);
    const int nb = dp >> 6, S = npass * nb;
    auto finish = [&](int pass) {
      comp16(xrow(pass), wr, nb * 64, dp);  // remainder k-steps (dp % 64)
      epilogue(pass);
    };
    if (nb == 0) {
      for (int pass = 0; pass < npass; ++pass) finish(pass);
    } else {
      f4 xa[4][4], xb[4][4];
      load(xa, xrow(0), 0);
      for (int st = 0; st < S; st += 2) {
        if (st + 1 < S) load(xb, xrow((st + 1) / nb), ((st + 1) % nb) * 64);
        __builtin_amdgcn_sched_barrier(0);
        comp(xa, wr, (st % nb) * 64);
        if ((st + 1) % nb == 0) finish(st / nb);
        if (st + 1 < S) {
          if (st + 2 < S) load(xa, xrow((st + 2) / nb), ((st + 2) % nb) * 64);
          __builtin_amdgcn_sched_barrier(0);
          comp(xb, wr, ((st + 1) % nb) * 64);
          if ((st + 2) % nb == 0) finish((st + 1) / nb);
        }
      }
    }
  } else {
    // wide rows: query vectors restaged per k-chunk of kRowsKC
    for (int pass = 0; pass < npass; ++pass) {
      const float* xr = xrow(pass);
      for (int kc = 0; kc < dp; kc += kRowsKC) {
        const int kcl = min(kRowsKC, dp - kc), ldw = kcl + 4, k4n = kcl >> 2;
        __syncthreads();  // previous readers of the staged chunk are done
        for (int i = tid; i < kNQ * k4n; i += kFusedThreads) {
          const int qq = i / k4n, k4 = i - qq * k4n;
          f4 v = {0.f, 0.f, 0.f, 0.f};
          if (qq < n_new && op[qq] == kOpCompute)
            v = *(const f4*)(a.x + ((int64_t)key[qq] - a.x_row0) * dp + kc + 4 * k4);
          *(f4*)(wsm + qq * ldw + 4 * k4) = v;
        }
        __syncthreads();
        const float* wr = wsm + q * ldw + 4 * (lane >> 4) - kc;  // indexed with absolute k
        const int nb = kcl >> 6;
        f4 xa[4][4], xb[4][4];
        if (nb > 0) load(xa, xr, kc);
        for (int bb = 0; bb < nb; bb += 2) {
          if (bb + 1 < nb) load(xb, xr, kc + (bb + 1) * 64);
          __builtin_amdgcn_sched_barrier(0);
          comp(xa, wr, kc + bb * 64);
          if (bb + 1 < nb) {
            if (bb + 2 < nb) load(xa, xr, kc + (bb + 2) * 64);
            __builtin_amdgcn_sched_barrier(0);
            comp(xb, wr, kc + (bb + 1) * 64);
          }
        }
        comp16(xr, wr, kc + nb * 64, kc + kcl);
      }
      epilogue(pass);
    }
  }
}

}  // namespace dev
}  // namespace dpsvm
