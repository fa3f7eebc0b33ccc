// Working-set engine, the sub-problem solve (ws_solve): the q x q sub-Gram in
// LDS and the reference's pair rule on wave 0 (svmTrainMain.cpp:255-299), the
// round's commit of the alphas and the changed rows.  Round structure and
// shared helpers: ws_common.hpp.
#include <hip/hip_runtime.h>

#include <atomic>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "ws_common.hpp"
#include "ws_solve.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// peer exchange: sub-Gram granules in flight per solve thread and poll batch
constexpr int kWsSolvePollBatch = 10;

// the sub-Gram load of one launch per round; the loop: ws_solve.hpp
template <bool kBox, bool kFull, bool kMulti, bool kW2, int NS = 3>
__global__ __launch_bounds__(kWsSolveThreads) void ws_solve_kernel(WsArgs a) {
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
  bool xok = true;
  if (a.xpeer != nullptr) {
    // peer exchange: block blk's rows a < q from this rank's receive buffer,
    // entries (a, b < q) and f (last column) pushed by their owners (the gather
    // kernels push and return: the solve is the round's only sub-Gram consumer);
    // columns q .. q_max - 1 are zeros.  A thread's granules are loaded in
    // batches of kB (all in flight: one latency of the uncached buffer per
    // batch), then only the ones not yet tagged are re-polled.
    const int64_t R = c->outer;
    const uint64_t t = xtag((uint32_t)R + 1u);
    const uint64_t* rows = a.xpeer[a.xrank] + ws_xrow(a, par, ib);  // row ra at + ra * (ldk + 1)
    const int w = ldk + 1, n_e = q * w;
    constexpr int kB = kWsSolvePollBatch;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int e0 = 0; e0 < n_e && xok; e0 += kB * kWsSolveThreads) {
      uint64_t v[kB];
      uint32_t need = 0;  // bit k: entry e0 + tid + k * threads still to land
#pragma unroll
      for (int k = 0; k < kB; ++k) {
        const int e = e0 + tid + k * kWsSolveThreads;
        const int col = e - (e / w) * w;
        const bool want = e < n_e && (col < q || col == ldk);
        v[k] = want ? xch_load<true>(rows + e) : t;
        need |= want ? 1u << k : 0u;
      }
      while (true) {
#pragma unroll
        for (int k = 0; k < kB; ++k)
          if (((need >> k) & 1u) && ws_tag_ok(v[k], t)) need &= ~(1u << k);
        if (need == 0) break;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.xtimeout_ticks) {
          xok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < kB; ++k)
          if ((need >> k) & 1u) v[k] = xch_load<true>(rows + e0 + tid + k * kWsSolveThreads);
      }
#pragma unroll
      for (int k = 0; k < kB; ++k) {
        const int e = e0 + tid + k * kWsSolveThreads;
        if (e >= n_e) break;
        const int ra = e / w, col = e - ra * w;
        if (col < ldk) K[ra * ldk + col] = col < q ? __uint_as_float((uint32_t)v[k]) : 0.f;
        else s_f[ra] = __uint_as_float((uint32_t)v[k]);
      }
    }
    if (tid < q) {
      s_a[tid] = aux[a.aux_stride + tid];
      s_y[tid] = aux[2 * a.aux_stride + tid];
      s_idx[tid] = c->idx[par][ib + tid];
      s_line[tid] = c->line[par][ib + tid];
    }
  } else if (a.direct_sub) {
    // blocks of <= 64 rows at world 1 (dense): the entries straight from the
    // resident Gram (K(i, j) at gram[i ldg + j]) instead of a ws_gather launch
    // of P q workgroups, its launch gap and a second copy through global
    // memory.  Each entry is a random 128-B line of HBM, so only the upper
    // triangle is loaded (the split Gram is bitwise symmetric) and mirrored in
    // LDS: 1,176 loads for a 48-row block, all in flight at once
    int32_t gi = 0;
    if (tid < q) {
      gi = c->idx[par][ib + tid];
      s_idx[tid] = gi;
      s_line[tid] = c->line[par][ib + tid];
    }
    __syncthreads();
    // the rows' f / alpha / y in flight with the entries (one memory round trip
    // for both, stored after)
    float fv = 0.f, av = 0.f, yv = 0.f;
    if (tid < q) {
      fv = a.f[gi];  // one rank: local row = global row
      av = a.alpha[gi];
      yv = a.y[gi];
    }
    const int n = q * ldk;
    constexpr int U = 4;  // n <= 64 x 64 = U x threads: one pass
    for (int e0 = tid; e0 < n; e0 += U * kWsSolveThreads) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * kWsSolveThreads;
        const int ra = e / ldk, col = e - ra * ldk;
        v[u] = e < n && ra <= col && col < q ? a.gram[(int64_t)s_idx[ra] * a.ldg + s_idx[col]] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * kWsSolveThreads;
        const int ra = e / ldk, col = e - ra * ldk;
        if (e < n && ra <= col) {
          K[e] = v[u];                                    // columns q .. q_max - 1: zeros
          if (col < q && col != ra) K[col * ldk + ra] = v[u];  // the mirrored entry
        }
      }
    }
    if (tid < q) {
      s_f[tid] = fv;
      s_a[tid] = av;
      s_y[tid] = yv;
    }
  } else {
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
  bool xfail = false;
  if (a.xpeer != nullptr) xfail = !__syncthreads_and(xok);
  else __syncthreads();
  // a rank stopped publishing: this block takes no step; its commit below still
  // counts it, and the round's last block keeps kCommFail
  if (xfail && tid == 0) ws_comm_fail_thread(a, c);
  if (tid == 0) WS_STAMP(3);
  if (wave != 0) return;

  ws_solve_run<kBox, kFull, kMulti, kW2, NS>(a, c, K, s_a, s_y, s_f, s_idx, s_line, q, blk, ib, it0, b_hi, b_lo,
                                             xfail);
}

}  // namespace dev

namespace launch {

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
  // one slot per lane when q_max <= 64 (blocks of the 64-block rounds)
#define WS_SOLVE_FNS1(W2)                                                                                        \
  dev::ws_solve_kernel<false, false, false, W2, 1>, dev::ws_solve_kernel<true, false, false, W2, 1>,            \
      dev::ws_solve_kernel<false, false, true, W2, 1>, dev::ws_solve_kernel<true, false, true, W2, 1>
  static const Fn fns1[8] = {WS_SOLVE_FNS1(false), WS_SOLVE_FNS1(true)};
#undef WS_SOLVE_FNS1
  const int v = (w2 ? 8 : 0) + (multi ? 4 : 0) + (box ? 2 : 0) + (full ? 1 : 0);
  const int v2 = (w2 ? 4 : 0) + (multi ? 2 : 0) + (box ? 1 : 0);
  const bool one = a.q_max <= 64, two = !one && a.q_max <= 128;
  const Fn fn = one ? fns1[v2] : two ? fns2[v2] : fns[v];
  // dynamic LDS above 64 KiB needs the attribute (160 KiB on gfx950); the
  // largest size set so far per device and kernel (rank threads of one process
  // launch on different devices concurrently)
  static std::atomic<size_t> attr[kMaxDevices][32];
  std::atomic<size_t>& at = attr[current_device()][one ? 24 + v2 : two ? 16 + v2 : v];
  size_t cur = at.load(std::memory_order_relaxed);
  if (lds > 64 * 1024 && lds > cur) {
    HIP_CHECK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    while (lds > cur && !at.compare_exchange_weak(cur, lds)) {
    }
  }
  fn<<<multi ? a.blocks : 1, kWsSolveThreads, lds, s>>>(a);
  post_launch("ws_solve", s);
}

}  // namespace launch
}  // namespace dpsvm
