// Working-set engine, persistent small-problem rounds (ws_persist): ONE launch
// runs up to `rounds` one-block rounds of the resident-Gram engine on a grid of
// G co-resident workgroups (one per CU, checked by a census at setup), with
// the round's kernel boundaries replaced by two one-way signals:
//
//   every group   waits for the G selection arrivals of the previous round
//                 (psync[0]), merges the candidate lists (stop test + next
//                 working set, ws_merge.hpp — redundantly, as ws_gather does),
//                 gathers rows grp, grp + G, ... of the q x q sub-Gram into
//                 global memory and arrives (psync[4]);
//   workgroup 0   waits for those G arrivals, loads the sub-Gram into LDS, runs
//                 the pair loop on wave 0 and the commit (ws_solve.hpp), then
//                 releases the round (psync[1] = rounds released);
//   every group   waits for the release, applies the round's alpha changes to
//                 its 256 columns of f and publishes its candidate lists (the
//                 ws_select arithmetic: the same four list partitions summed in
//                 the same order, so f, the candidates and the trajectory are
//                 bit-identical to the graph of launches), then arrives.
//
// The graph path spends ~29 us of a ~74 us round of the covtype-shape 7.5k-row
// sub-problem outside the solve (four launches: select 9.3, merge 8.0, gather
// and sub-Gram load 4.4, launch gaps ~6; profiles/r4_ws_stamps_cov7500*.json);
// here a round boundary is an agent-scope fence pair plus an atomic per
// signal (three per round).  Cross-workgroup data (f rows of the set, alpha, candidate
// lists, the control record) moves under release / acquire fences at agent
// scope (the XCDs' L2s are not coherent with each other).  Every wait is
// bounded (a.xtimeout_ticks): a grid that is not co-resident ends the run with
// kCommFail instead of hanging.  Stamps (DPSVM_STAMPS, workgroup 0): [0] round
// start, [1] arrivals seen, [2] merged, [8] gather arrivals seen, [3] sub-Gram
// in LDS, [4] solved, [6] release seen, [10] f updated, [7] candidates published.  Reference round:
// svmTrainMain.cpp:235-310.
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "ws_common.hpp"
#include "ws_merge.hpp"
#include "ws_solve.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

constexpr int kWpThreads = kWsGatherThreads;  // the merge's block (256 threads)
static_assert(kWpThreads == kWsSelThreads, "one selection group of 256 columns per workgroup");

__device__ __forceinline__ int32_t wp_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0 waits until *p >= target (false: timed out); the caller's barrier
// then publishes the outcome to the workgroup
__device__ __forceinline__ bool wp_wait(const int32_t* p, int32_t target, int64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (wp_load(p) < target) {
    if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > ticks) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// the run ends (a wait timed out: the grid is not co-resident after all)
__device__ __forceinline__ void wp_fail(const WsArgs& a, WsCtrl* c) {
  __hip_atomic_store(&c->done, (int32_t)kCommFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  c->n_apply = 0;
  ws_status(a.status, c);
}

// LDS of one workgroup: the union (merge scratch | sub-Gram | the round's change
// list) is dynamic, q_max^2 floats at least
template <bool kBox, bool kFull, bool kW2, int NS>
__global__ __launch_bounds__(kWpThreads, 1) void ws_persist_kernel(WsArgs a, int rounds) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ float s_a[kWsMax + 128], s_y[kWsMax], s_f[kWsMax];  // s_a: + 2 x 64 scratch words (the solve)
  __shared__ int32_t s_set[kWsMax], s_line[kWsMax];
  __shared__ uint64_t s_wc[kWpThreads / 64][2][kWsCand1];
  __shared__ int s_word[2];
  int32_t* const sync = a.psync;
  if (rounds < 0) {  // residency census (setup): this kernel, this grid, these resources
    census_arrive(sync + 2, a.xtimeout_ticks);
    return;
  }
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = (int)gridDim.x, grp = (int)blockIdx.x;
  const bool wg0 = grp == 0;
  const bool lead = wg0 && tid == 0;
  if (tid == 0) s_word[0] = wp_load(sync + 1);  // rounds released before this launch (nobody moves it yet)
  __syncthreads();
  const int32_t gen0 = s_word[0];
  int32_t* s_list = (int32_t*)lds;              // the change list: lines, then coefficients
  float* s_coef = lds + kWsMax;
  const int64_t j = (int64_t)grp * kWpThreads + tid;  // this thread's column (rpt = 1)
  const bool has = j < a.nl;

  for (int r = 0; r < rounds; ++r) {
    const int32_t gen = gen0 + r;  // rounds released before this one
    // ---- every group: the previous round's selections are in (r = 0: the
    // launch boundary), then the merge — redundantly, identical inputs and
    // arithmetic, as in ws_gather: no group waits for a published set ----
    if (wg0 && tid == 0) WS_STAMP(0);
    if (tid == 0) s_word[1] = r == 0 || wp_wait(sync, G * gen, a.xtimeout_ticks) ? 1 : 0;
    __syncthreads();
    if (!s_word[1]) {
      if (tid == 0) wp_fail(a, c);
      break;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every group's f and candidate lists
    if (lead) WS_STAMP(1);
    int q = 0;
    float b_hi = 0.f, b_lo = 0.f;
    const bool go = ws_merge(a, c, s_set, &q, &b_hi, &b_lo, *(WsMergeLds*)lds);  // ends with a barrier
    const int par = (int)(c->outer & 1);
    const int ldk = a.q_max;
    if (go) {
      if (lead) WS_STAMP(2);
      if (wg0) {
        for (int t = tid; t < q; t += kWpThreads) {
          c->idx[par][t] = s_set[t];
          c->line[par][t] = s_set[t];  // the resident Gram: line i is row i
        }
        if (tid == 0) {
          c->q[par] = q;
          c->b_hi = b_hi;
          c->b_lo = b_lo;
        }
      }
      // the sub-Gram rows ra = grp, grp + G, ... (q random columns of member
      // ra's Gram row; columns q .. q_max - 1 zero) and their f / alpha / y,
      // through global memory to workgroup 0 (the scattered reads of one CU
      // would take ~30 us: the whole grid issues them)
      const int my_rows = q > grp ? (q - grp + G - 1) / G : 0;
      const int n = my_rows * ldk;
      constexpr int U = 8;
      for (int e0 = tid; e0 < n; e0 += U * kWpThreads) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = e0 + u * kWpThreads;
          const int k = e / ldk, col = e - k * ldk;
          const bool in = e < n && col < q;
          v[u] = in ? a.gram[(int64_t)s_set[grp + k * G] * a.ldg + s_set[col]] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = e0 + u * kWpThreads;
          const int k = e / ldk, col = e - k * ldk;
          if (e < n) a.subg[(size_t)(grp + k * G) * ldk + col] = v[u];
        }
      }
      for (int k = tid; k < my_rows; k += kWpThreads) {
        const int ra = grp + k * G;
        const int32_t gi = s_set[ra];
        a.aux[ra] = a.f[gi];  // one rank: local row = global row
        a.aux[a.aux_stride + ra] = a.alpha[gi];
        a.aux[2 * a.aux_stride + ra] = a.y[gi];
      }
    }
    // every group arrives (also when the run stopped: the counts stay G per round)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(sync + 4, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);

    // ---- workgroup 0: the sub-Gram into LDS, the pair loop, the commit ----
    if (wg0) {
      if (go) {
        if (tid == 0) s_word[1] = wp_wait(sync + 4, G * (gen + 1), a.xtimeout_ticks) ? 1 : 0;
        __syncthreads();
        if (!s_word[1]) {
          if (tid == 0) wp_fail(a, c);
          break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (lead) WS_STAMP(8);
        const int64_t it0 = c->iter;
        float* K = lds;
        if ((ldk & 3) == 0) {  // q rows x q_max: 16-B loads, four in flight per thread
          const f4* src = (const f4*)a.subg;
          f4* dst = (f4*)K;
          const int n4 = q * ldk / 4;
          for (int e = tid; e < n4; e += 4 * kWpThreads) {
            f4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int k = e + u * kWpThreads;
              v[u] = src[k < n4 ? k : 0];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (e + u * kWpThreads < n4) dst[e + u * kWpThreads] = v[u];
          }
        } else {
          for (int e = tid; e < q * ldk; e += kWpThreads) K[e] = a.subg[e];
        }
        for (int t = tid; t < q; t += kWpThreads) {
          s_line[t] = s_set[t];
          s_f[t] = a.aux[t];
          s_a[t] = a.aux[a.aux_stride + t];
          s_y[t] = a.aux[2 * a.aux_stride + t];
        }
        __syncthreads();
        if (lead) WS_STAMP(3);
        if (wave == 0)
          ws_solve_run<kBox, kFull, false, kW2, NS>(a, c, K, s_a, s_y, s_f, s_set, s_line, q, 0, 0, it0, b_hi, b_lo,
                                                    false);
      }
      // release: every wave's stores (control record, alphas, change list) out
      // of this XCD's L2 before the round count moves
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(sync + 1, gen + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (tid == 0) s_word[1] = wp_wait(sync + 1, gen + 1, a.xtimeout_ticks) ? 1 : 0;
      __syncthreads();
      if (!s_word[1]) {
        if (tid == 0) wp_fail(a, c);
        break;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }

    // ================= every group: f update of its columns + candidates =================
    if (wg0 && tid == 0) WS_STAMP(6);
    const int na = __hip_atomic_load(&c->n_apply, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int done = __hip_atomic_load(&c->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // workgroup 0: the sub-Gram (aliased by the list) is dead
    for (int k = tid; k < na; k += kWpThreads) {
      s_list[k] = c->apply_line[k];
      s_coef[k] = c->apply_coef[k];
    }
    __syncthreads();
    float f = has ? a.f[j] : 0.f;
    if (na > 0) {
      // ws_select MODE 0 at RPT 1: four partitions of the list, each summed in
      // list order, combined in partition order (ws_select.hip)
      const int per = (na + 3) / 4;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      constexpr int CH = 15;  // x 4 partitions: 60 Gram loads in flight per thread (vmcnt <= 63)
      for (int s0 = 0; s0 < per; s0 += CH) {
        float kv[4][CH];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            const int k = min(p * per + s0 + u, na - 1);
            kv[p][u] = has ? a.gram[(int64_t)s_list[k] * a.ldg + j] : 0.f;
          }
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int k_hi = min(na, (p + 1) * per);
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            const int k = p * per + s0 + u;
            if (k < k_hi) acc[p] = f_add1(acc[p], s_coef[k], kv[p][u]);
          }
        }
      }
      float d;
      {
#pragma clang fp contract(off)
        d = ((acc[0] + acc[1]) + acc[2]) + acc[3];
        f = f + d;
      }
      if (has) a.f[j] = f;
      if (has && !isfinite(f)) atomicOr(&c->nonfinite, 1);
    }
    if (wg0 && tid == 0) WS_STAMP(10);
    if (done == kRunning) {
      uint64_t ku = kKeyNone, kl = kKeyNone;
      if (has) {
        const float av = a.alpha[j], yv = a.y[j];
        if (in_up(av, yv, a.C)) ku = make_key(f, (uint32_t)j);
        if (in_low(av, yv, a.C)) kl = make_key(-f, (uint32_t)j);
      }
      // each wave's kWsCand1 smallest keys per side, then wave 0 merges the four
      // lists (the owner of a winner drops it: keys are unique)
      for (int rr = 0; rr < kWsCand1; ++rr) {
        const uint64_t mu = wave_min_u64(ku), ml = wave_min_u64(kl);
        if (lane == 0) {
          s_wc[wave][0][rr] = mu;
          s_wc[wave][1][rr] = ml;
        }
        if (ku == mu) ku = kKeyNone;
        if (kl == ml) kl = kKeyNone;
      }
      __syncthreads();
      if (wave == 0) {
        const bool hv = lane < (kWpThreads / 64) * kWsCand1;
        uint64_t eu = hv ? s_wc[lane / kWsCand1][0][lane % kWsCand1] : kKeyNone;
        uint64_t el = hv ? s_wc[lane / kWsCand1][1][lane % kWsCand1] : kKeyNone;
        uint64_t* out = a.cand_out + (size_t)grp * 2 * kWsCand;
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
    }
    if (wg0 && tid == 0) WS_STAMP(7);
    // arrive: this group's f and lists out of its XCD's L2 first
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(sync, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (done != kRunning) break;  // uniform: every group read the same record
  }
}

}  // namespace dev

namespace launch {

using WsPersistFn = void (*)(WsArgs, int);

static WsPersistFn ws_persist_fn(const WsArgs& a) {
  const bool box = a.clip == (int)ClipMode::Box, full = a.q_max == kWsMax, w2 = a.wss == 2;
  // slots per lane as ws_solve: 3 (q_max > 128), 2 (<= 128), 1 (<= 64)
#define WP(B, F, W, S) dev::ws_persist_kernel<B, F, W, S>
  static const WsPersistFn f3[8] = {WP(false, false, false, 3), WP(false, true, false, 3), WP(true, false, false, 3),
                                    WP(true, true, false, 3),   WP(false, false, true, 3), WP(false, true, true, 3),
                                    WP(true, false, true, 3),   WP(true, true, true, 3)};
  static const WsPersistFn f2[4] = {WP(false, false, false, 2), WP(true, false, false, 2), WP(false, false, true, 2),
                                    WP(true, false, true, 2)};
  static const WsPersistFn f1[4] = {WP(false, false, false, 1), WP(true, false, false, 1), WP(false, false, true, 1),
                                    WP(true, false, true, 1)};
#undef WP
  if (a.q_max <= 64) return f1[(w2 ? 2 : 0) + (box ? 1 : 0)];
  if (a.q_max <= 128) return f2[(w2 ? 2 : 0) + (box ? 1 : 0)];
  return f3[(w2 ? 4 : 0) + (box ? 2 : 0) + (full ? 1 : 0)];
}

size_t ws_persist_lds(const WsArgs& a) {
  return std::max(sizeof(dev::WsMergeLds), (size_t)a.q_max * a.q_max * sizeof(float));
}

static WsPersistFn ws_persist_prepared(const WsArgs& a) {
  WsPersistFn fn = ws_persist_fn(a);
  const size_t lds = ws_persist_lds(a);
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return fn;
}

int ws_persist_blocks_per_cu(const WsArgs& a) {
  WsPersistFn fn = ws_persist_prepared(a);
  int nb = 0;
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)fn, dev::kWpThreads, ws_persist_lds(a)));
  return nb;
}

bool ws_persist_supported(const WsArgs& a) {
  // one rank, one block, the resident Gram, 256 columns per workgroup, and a
  // change list that fits the LDS union (q_max <= kWsMax: 2 q_max words)
  return a.world == 1 && a.blocks == 1 && a.cache == 0 && a.xpeer == nullptr && a.rpt == 1 && a.G >= 1 &&
         a.G <= kWsMaxGroups && a.psync != nullptr && 2 * a.q_max * 4 <= (int64_t)ws_persist_lds(a);
}

void ws_persist_census(const WsArgs& a, hipStream_t s) {
  WsPersistFn fn = ws_persist_prepared(a);
  fn<<<dim3((unsigned)a.G), dev::kWpThreads, ws_persist_lds(a), s>>>(a, -1);
  post_launch("ws_persist census", s);
}

void ws_persist(const WsArgs& a, int rounds, hipStream_t s) {
  DPSVM_CHECK(ws_persist_supported(a), "ws_persist: one rank, one block, resident Gram, rpt 1");
  WsPersistFn fn = ws_persist_prepared(a);
  fn<<<dim3((unsigned)a.G), dev::kWpThreads, ws_persist_lds(a), s>>>(a, rounds);
  post_launch("ws_persist", s);
}

}  // namespace launch
}  // namespace dpsvm
