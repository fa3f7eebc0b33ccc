// Persistent SMO for the kernel-row-cache mode (replicated X, the Gram shard
// does not fit in HBM): ONE launch runs up to `steps` iterations, like
// smo_persist.hip, over a CLOCK cache of kernel-row lines.
//
// Every workgroup only ever reads and writes ITS OWN rows' segments of the
// lines, and every workgroup takes the same cache decisions from the same
// inputs (the pair, the publications, its copy of the metadata).  So each
// workgroup keeps a PRIVATE copy of the cache metadata (slot_of / key_of / ref
// bits / hand) in HBM and no cache state is shared between workgroups: the
// only per-iteration traffic between workgroups stays the key exchange
// (xch.hpp), exactly as in the dense persistent engine.
//
// Iteration t in workgroup b:
//   0. the CLOCK window's bits and owners (pair independent) load during the
//      poll;
//   1. wave 0 polls the publications tagged t: the pair with its alphas, and
//      every lane keeps its best candidate per side (speculation);
//   2. one round trip: the pair's slots and labels; wave 0 also the sample rows
//      for eta and the candidates' slots, then plans: alpha update, the rows
//      the f update needs, hits / misses, speculative rows (the policy of
//      smo_fused_lru.hip);
//   3. on a miss: block-wide CLOCK victim scan of the window, metadata update,
//      X pass over the own rows for the new lines (xpass.hpp);
//   4. f / alpha update of the own rows (registers) from the two lines,
//      classification, keys published tagged t+1.
// Same arithmetic as smo_fused_lru / smo_rows (one X pass, one f_apply, one
// eta), so every cache engine follows the same trajectory bit for bit.
// Reference: svmTrainMain.cpp:235-310 with the host LRU of cache.cu:62-105 and
// one cublasSgemv per missed row (svmTrain.cu:212-249).
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "plan_util.hpp"
#include "xch.hpp"
#include "xpass.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

constexpr int kPLMaxRows = 12;  // rows per thread (fused_rows <= 3072)

// decisions of one iteration, shared by the waves of a workgroup (LDS)
struct PLPlan {
  int n_new, n_miss, need_hi, need_lo, hit_hi, hit_lo, miss_hi, span;
  int key[kNQ], line[kNQ], old[kNQ], op[kNQ];
};

template <bool kSys, int kB>
__global__ __launch_bounds__(kFusedThreads) void smo_persist_lru_kernel(SmoArgs a, FusedRec* __restrict__ st,
                                                                        int steps, int64_t* __restrict__ stats) {
  static_assert(kFusedThreads == 256, "4 waves assumed");
  extern __shared__ __attribute__((aligned(16))) float wsm[];  // X pass: query vectors + own |x|^2
  __shared__ uint64_t kscr[8];
  __shared__ float kfs[8];
  __shared__ XKeys pair_s;
  __shared__ int fail_s;
  __shared__ float d2_s;
  __shared__ PLPlan pl;
  __shared__ int kscan[kFusedThreads / 64];
  if (steps < 0) {  // residency census (setup): this kernel, this grid, this LDS
    census_arrive(a.census, a.census_ticks);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool lead = blockIdx.x == 0 && tid == 0;
  const int rpt = (a.fused_rows + kFusedThreads - 1) / kFusedThreads;
  const int64_t row0 = (int64_t)blockIdx.x * a.fused_rows;
  const int64_t row_end = min((int64_t)a.nl, row0 + (int64_t)a.fused_rows);

  float f[kPLMaxRows], al[kPLMaxRows], yv[kPLMaxRows];
  bool has[kPLMaxRows];
#pragma unroll
  for (int k = 0; k < kPLMaxRows; ++k) {
    const int64_t j = row0 + tid + (int64_t)k * kFusedThreads;
    has[k] = k < rpt && j < row_end;
    f[k] = has[k] ? a.f[j] : 0.f;
    al[k] = has[k] ? a.alpha[a.off + j] : 0.f;
    yv[k] = has[k] ? a.y[a.off + j] : 0.f;
  }
  const FusedRec s0 = *st;
  if (s0.done != kRunning) return;
  int32_t* meta = a.plru_meta + (int64_t)blockIdx.x * a.plru_stride;
  int32_t* slot = meta + 4;
  int32_t* keyo = slot + a.n;
  uint8_t* refb = (uint8_t*)(keyo + a.L);
  int hand = meta[0];
  const int L = a.L, W = min(1024, a.L);
  // own rows' |x|^2 for the X pass, staged once per launch (ordered by the
  // first barrier of the loop)
  float* xsq_s = wsm + kNQ * ((a.dp < kRowsKC ? a.dp : kRowsKC) + 4);
  const int npass = (int)((row_end - row0 + 255) / 256);
  for (int i = tid; i < npass * 256; i += kFusedThreads) xsq_s[i] = a.xsq[a.off + row0 + i];
  const uint64_t* my_buf = a.xpeer[a.xrank];
  uint64_t* peer_buf = wave == 0 ? xch_peer(a, lane) : nullptr;
  int t = s0.iter, done = kRunning;
  float b_hi = s0.b_hi, b_lo = s0.b_lo;
  int64_t c_hits = 0, c_miss = 0, c_rows = 0, c_pass = 0, c_spec = 0;
  // diagnostics (DPSVM_STAMPS): thread 0 of workgroups 0 and G-1 stamps 0 poll
  // start, 1 pair known, 2 plan broadcast, 3 lines filled, 4 f update, 5
  // published; slot 6 = rows filled this iteration
  const bool stamping = a.stamps != nullptr && tid == 0 && (blockIdx.x == 0 || blockIdx.x == a.fused_G - 1);
  uint64_t stv[7] = {0, 0, 0, 0, 0, 0, 0};
#define PLSTAMP(i) \
  if (stamping) stv[i] = __builtin_amdgcn_s_memrealtime()

  for (int step = 0; step < steps; ++step) {
    // ---- 0. the CLOCK window (pair independent): in flight during the poll ----
    int wp[4], wref[4], wkey[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pos = 4 * tid + j;
      const int pp = hand + pos;  // hand < L, pos < W <= L
      wp[j] = pp >= L ? pp - L : pp;
      wref[j] = 1;
      wkey[j] = -1;
      if (pos < W) {
        wref[j] = refb[wp[j]];
        wkey[j] = keyo[wp[j]];
      }
    }

    // ---- 1. publications tagged t+1 (produced by iteration t) ----
    PLSTAMP(0);
    const uint32_t tag = (uint32_t)t + 1u;
    uint64_t ch = kKeyNone, cl = kKeyNone;  // wave 0: the lane's best candidate per side
    if (wave == 0) {
      XKeys m = xk_none();
      const bool ok = xch_poll_wave_t<kSys, kB>(a, my_buf, (int)(tag & 1u), tag, m, lane);
      ch = m.kh;
      cl = m.kl;
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
    const int iter = t + 1;
    PLSTAMP(1);

    // ---- 2. one round trip: the pair's slots and labels; wave 0: eta's
    //         sample rows and the candidates' slots ----
    const int s_hi = slot[i_hi], s_lo = slot[i_lo];
    const float y_hi = a.y[i_hi], y_lo = a.y[i_lo];  // read-only during the run
    const int ih_c = ch != kKeyNone ? (int)key_index(ch) : 0, il_c = cl != kKeyNone ? (int)key_index(cl) : 0;
    const float a_hi_old = pk.ah, a_lo_old = pk.al;  // the owners' current values
    float c_hi = 0.f, c_lo = 0.f, a_hi_new = a_hi_old, a_lo_new = a_lo_old;
    auto alpha_update = [&](float dist2) {
      if (!isfinite(bh) || !isfinite(bl)) {
        done = kNonFinite;
      } else {
        const float k_hl = expf(-a.gamma * dist2);
        const PairUpdate u =
            pair_update(a_hi_old, a_lo_old, y_hi, y_lo, bh, bl, k_hl, a.C, a.tau, a.clip, i_hi == i_lo);
        a_hi_new = u.a_hi_new;
        a_lo_new = u.a_lo_new;
        c_hi = u.c_hi;
        c_lo = u.c_lo;
        if (!gap_open(bh, bl, a.eps)) done = kConverged;
        else if (iter >= a.max_iter) done = kMaxIter;
      }
    };
    if (wave == 0) {
      const int cs_h = slot[ih_c], cs_l = slot[il_c];
      const float* xh = a.x + ((int64_t)i_hi - a.x_row0) * a.dp;
      const float* xl = a.x + ((int64_t)i_lo - a.x_row0) * a.dp;
      const float d2 = wave_dist2(xh, xl, a.dp, lane);  // same tree as every other engine
      alpha_update(d2);
      // rows the f update needs, hits and misses (uniform)
      const int need_hi = c_hi != 0.f ? i_hi : -1;
      const int need_lo = (c_lo != 0.f && !(i_lo == i_hi && c_hi != 0.f)) ? i_lo : -1;
      const int hit_hi = need_hi >= 0 ? s_hi : -1;
      const int hit_lo = need_lo >= 0 ? s_lo : -1;
      const int miss_hi = need_hi >= 0 && hit_hi < 0, miss_lo = need_lo >= 0 && hit_lo < 0;
      const int n_miss = miss_hi + miss_lo;
      const int budget = n_miss > 0 ? min(min(a.spec, kNQ - n_miss), max(0, L / 2 - n_miss)) : 0;
      int n_new = n_miss;
      if (budget > 0) {  // uniform: the best uncached candidates, t per side (ballot radix select)
        const bool ok_h = ch != kKeyNone && ih_c != i_hi && ih_c != i_lo && cs_h < 0;
        const bool ok_l = cl != kKeyNone && il_c != i_hi && il_c != i_lo && cs_l < 0;
        const uint64_t vch = ok_h ? ch : kKeyNone, vcl = ok_l ? cl : kKeyNone;
        const uint64_t valid_h = __ballot(ok_h), valid_l = __ballot(ok_l);
        const int vh = __popcll(valid_h), vl = __popcll(valid_l);
        int take_h = min(vh, (budget + 1) / 2);
        const int take_l = min(vl, budget - take_h);
        take_h = min(vh, budget - take_l);  // an exhausted low side leaves room
        const uint64_t sel_h = wave_smallest(vch, take_h, valid_h);
        uint64_t sel_l = wave_smallest(vcl, take_l, valid_l);
        // a free SV can win on both sides: keep one copy
        bool dup = false;
        for (uint64_t mm = sel_h; mm; mm &= mm - 1) {
          const int src = __ffsll((unsigned long long)mm) - 1;
          dup |= __builtin_amdgcn_readlane(ih_c, src) == il_c;
        }
        sel_l &= ~__ballot(dup);
        const uint64_t below = (1ull << lane) - 1ull;
        if ((sel_h >> lane) & 1ull) pl.key[n_miss + __popcll(sel_h & below)] = ih_c;
        if ((sel_l >> lane) & 1ull) pl.key[n_miss + __popcll(sel_h) + __popcll(sel_l & below)] = il_c;
        n_new = n_miss + __popcll(sel_h) + __popcll(sel_l);
      }
      if (lane == 0) {
        d2_s = d2;
        if (n_miss > 0) pl.key[0] = miss_hi ? need_hi : need_lo;  // misses first (hi before lo)
        if (n_miss > 1) pl.key[1] = need_lo;
        pl.n_new = n_new;
        pl.n_miss = n_miss;
        pl.need_hi = need_hi;
        pl.need_lo = need_lo;
        pl.hit_hi = hit_hi;
        pl.hit_lo = hit_lo;
        pl.miss_hi = miss_hi;
        pl.span = 0;
      }
      if (lane < kNQ) pl.op[lane] = kOpCompute;
    }
    __syncthreads();
    if (wave != 0) alpha_update(d2_s);
    PLSTAMP(2);
    b_hi = bh;
    b_lo = bl;
    if (done == kNonFinite) break;  // uniform (no rows needed: nothing planned)
    if (lead) {  // alpha memory is write-only during the run (read after the launch)
      a.alpha[i_lo] = a_lo_new;
      a.alpha[i_hi] = a_hi_new;  // hi written last (svmTrainMain.cpp:298-299)
    }
    t = iter;
    const int M = pl.n_new, n_miss = pl.n_miss;
    const int hit_hi = pl.hit_hi, hit_lo = pl.hit_lo;
    c_hits += (pl.need_hi >= 0) + (pl.need_lo >= 0) - n_miss;
    c_miss += n_miss;
    c_rows += M;
    c_pass += M > 0;
    c_spec += M - n_miss;

    // ---- 3. misses: CLOCK victims from the window, metadata, X pass ----
    if (M > 0) {  // uniform
      bool e[4], unp[4];
      int cnt = 0, cnt2 = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        unp[j] = 4 * tid + j < W && wp[j] != hit_hi && wp[j] != hit_lo;
        e[j] = unp[j] && wref[j] == 0;
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
            pl.old[r] = wkey[j];
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
              pl.old[total + r2] = wkey[j];
            }
            ++r2;
          }
        }
        if (tid == 0) pl.span = W;
      }
      __syncthreads();
      // metadata (this workgroup's copy): scanned window bits get their final
      // value (1 for new / hit lines), new lines take their rows
      const int span = pl.span;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (4 * tid + j < span) {
          bool keep = wp[j] == hit_hi || wp[j] == hit_lo;
          for (int q = 0; q < M; ++q) keep |= pl.line[q] == wp[j];
          refb[wp[j]] = keep ? 1 : 0;
        }
      }
      if (tid == 1 || tid == 2) {  // hit lines outside the scanned part of the window
        const int l = tid == 1 ? hit_hi : hit_lo;
        int off = l - hand;
        if (off < 0) off += L;
        if (l >= 0 && off >= span) refb[l] = 1;
      }
      if (tid >= 16 && tid < 16 + M) {
        const int q = tid - 16;
        const int l = pl.line[q], k = pl.key[q], o = pl.old[q];
        if (o >= 0) slot[o] = -1;  // evicted rows are cached rows, new rows uncached: disjoint
        keyo[l] = k;
        slot[k] = l;
      }
      hand = hand + span >= L ? hand + span - L : hand + span;
      xpass_fill(a, row0, row_end, M, pl.key, pl.line, pl.op, wsm, true);
      __syncthreads();  // the new segments are visible to every wave of the workgroup
    } else if (tid == 0) {
      if (hit_hi >= 0) refb[hit_hi] = 1;
      if (hit_lo >= 0) refb[hit_lo] = 1;
    }

    PLSTAMP(3);
    if (stamping) stv[6] = (uint64_t)M;
    // ---- 4. f update + classification of the own rows ----
    const int need_hi = pl.need_hi;
    int line_hi = -1, line_lo = -1;
    if (need_hi >= 0) line_hi = hit_hi >= 0 ? hit_hi : pl.line[0];
    if (c_lo != 0.f) {
      if (i_lo == i_hi && c_hi != 0.f) line_lo = line_hi;
      else line_lo = hit_lo >= 0 ? hit_lo : (pl.miss_hi ? pl.line[1] : pl.line[0]);
    }
    // absent lines read f (finite) through a dummy pointer; their coefficient is 0
    const float* lh = line_hi >= 0 ? a.lines + (int64_t)line_hi * a.ldl + row0 : a.f + row0;
    const float* ll = line_lo >= 0 ? a.lines + (int64_t)line_lo * a.ldl + row0 : a.f + row0;
    float khv[kPLMaxRows], klv[kPLMaxRows];
#pragma unroll
    for (int k = 0; k < kPLMaxRows; ++k) {
      const int64_t j = has[k] ? tid + (int64_t)k * kFusedThreads : 0;
      khv[k] = lh[j];
      klv[k] = ll[j];
    }
    const bool upd_f = c_hi != 0.f || c_lo != 0.f;
    XKeys nk = xk_none();
#pragma unroll
    for (int k = 0; k < kPLMaxRows; ++k) {
      if (!has[k]) continue;
      const int64_t g = a.off + row0 + tid + (int64_t)k * kFusedThreads;
      if (upd_f) f[k] = f_apply(f[k], c_hi, c_hi != 0.f ? khv[k] : 0.f, c_lo, c_lo != 0.f ? klv[k] : 0.f);
      if (g == i_lo) al[k] = a_lo_new;
      if (g == i_hi) al[k] = a_hi_new;  // hi wins when i_hi == i_lo
      if (in_up(al[k], yv[k], a.C)) xk_min(nk, XKeys{make_key(f[k], (uint32_t)g), kKeyNone, al[k], 0.f});
      if (in_low(al[k], yv[k], a.C)) xk_min(nk, XKeys{kKeyNone, make_key(-f[k], (uint32_t)g), 0.f, al[k]});
    }
    PLSTAMP(4);
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
      const uint32_t otag = (uint32_t)t + 1u;
      xch_push(a, peer_buf, (int)(otag & 1u), blockIdx.x, nk, otag, lane);
      PLSTAMP(5);
      if (stamping) {
        uint64_t* dst = a.stamps + ((size_t)(t % kStampRing) * 2 + (blockIdx.x == 0 ? 0 : 1)) * kStampSlots;
#pragma unroll
        for (int i = 0; i < 7; ++i) dst[i] = stv[i];
      }
    }
  }
#undef PLSTAMP

  // ---- exit: own rows' f back to memory, the hand to the private metadata;
  //      workgroup 0 writes the state and the statistics ----
#pragma unroll
  for (int k = 0; k < kPLMaxRows; ++k) {
    const int64_t j = row0 + tid + (int64_t)k * kFusedThreads;
    if (has[k]) a.f[j] = f[k];
  }
  if (tid == 0) meta[0] = hand;
  if (lead) {
    FusedRec o;
    o.i_hi = o.i_lo = -1;
    o.a_hi = o.a_lo = 0.f;
    o.iter = t;
    o.done = done;
    o.b_hi = b_hi;
    o.b_lo = b_lo;
    *st = o;
    const int64_t hits = stats[0] + c_hits, misses = stats[1] + c_miss, rows = stats[2] + c_rows,
                  passes = stats[3] + c_pass, spec = stats[4] + c_spec;
    stats[0] = hits;
    stats[1] = misses;
    stats[2] = rows;
    stats[3] = passes;
    stats[4] = spec;
    if (a.status) {
      SmoStatus* s = a.status;
      s->iter = t;
      s->done = done;
      s->b_hi = b_hi;
      s->b_lo = b_lo;
      s->hits = hits;
      s->misses = misses;
      s->rows_computed = rows;
      s->x_passes = passes;
      s->spec_rows = spec;
      __atomic_store_n(&s->seq, t, __ATOMIC_RELEASE);
    }
  }
}

// metadata of every workgroup: hand 0, slot_of / key_of -1, ref bits 0
__global__ void plru_init_kernel(int32_t* meta, int64_t stride, int64_t G, int64_t n, int64_t L) {
  const int64_t words_ref = (L + 3) / 4;
  const int64_t used = 4 + n + L + words_ref;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < G * used; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / used, w = e - b * used;
    meta[b * stride + w] = (w < 4 || w >= 4 + n + L) ? 0 : -1;
  }
}

}  // namespace dev

namespace launch {

int64_t plru_stride_words(int64_t n, int64_t L) { return (4 + n + L + (L + 3) / 4 + 63) / 64 * 64; }

bool smo_persist_lru_supported(int dp, int fused_rows, int fused_G) {
  return dp >= 16 && dp % 16 == 0 && fused_rows <= dev::kPLMaxRows * kFusedThreads && fused_G <= 256 &&
         dev::xpass_lds_floats(dp, fused_rows) * sizeof(float) <= 144 * 1024;
}

void plru_init(int32_t* meta, int64_t stride, int64_t G, int64_t n, int64_t L, hipStream_t s) {
  dev::plru_init_kernel<<<1024, 256, 0, s>>>(meta, stride, G, n, L);
  post_launch("plru_init", s);
}

using PlruFn = void (*)(SmoArgs, FusedRec*, int, int64_t*);
static PlruFn plru_fn(const SmoArgs& a, size_t lds) {
  const int E = a.xworld * a.fused_G;
  const int kb = a.xpoll_kb > 0 ? a.xpoll_kb : (E <= 64 ? 1 : E <= 128 ? 2 : 4);
  PlruFn fn;
  if (a.xworld > 1)
    fn = kb == 1 ? dev::smo_persist_lru_kernel<true, 1> : kb == 2 ? dev::smo_persist_lru_kernel<true, 2>
                                                                  : dev::smo_persist_lru_kernel<true, 4>;
  else
    fn = kb == 1 ? dev::smo_persist_lru_kernel<false, 1> : kb == 2 ? dev::smo_persist_lru_kernel<false, 2>
                                                                   : dev::smo_persist_lru_kernel<false, 4>;
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return fn;
}

int smo_persist_lru_blocks_per_cu(const SmoArgs& a) {
  const size_t lds = dev::xpass_lds_floats(a.dp, a.fused_rows) * sizeof(float);
  int nb = 0;
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)plru_fn(a, lds), kFusedThreads, lds));
  return nb;
}

void smo_persist_lru_census(const SmoArgs& a, int groups, hipStream_t s) {
  const size_t lds = dev::xpass_lds_floats(a.dp, a.fused_rows) * sizeof(float);
  plru_fn(a, lds)<<<dim3(groups), kFusedThreads, lds, s>>>(a, nullptr, -1, nullptr);
  post_launch("smo_persist_lru census", s);
}

void smo_persist_lru(const SmoArgs& a, FusedRec* st, int steps, int64_t* stats, hipStream_t s) {
  DPSVM_CHECK(a.xworld >= 1 && smo_persist_lru_supported(a.dp, a.fused_rows, a.fused_G) && a.plru_meta,
              "persistent cache SMO: needs the key exchange, <= 256 resident workgroups, <= 3072 rows each");
  const size_t lds = dev::xpass_lds_floats(a.dp, a.fused_rows) * sizeof(float);
  plru_fn(a, lds)<<<dim3(a.fused_G), kFusedThreads, lds, s>>>(a, st, steps, stats);
  post_launch("smo_persist_lru", s);
}

void preload_persist_lru_kernel(hipStream_t s) {
  // trivial launches (state "done"): load the code objects and exit
  FusedRec* st = nullptr;
  HIP_CHECK(hipMalloc((void**)&st, sizeof(FusedRec)));
  FusedRec h{};
  h.done = kConverged;
  HIP_CHECK(hipMemcpyAsync(st, &h, sizeof(h), hipMemcpyHostToDevice, s));
  SmoArgs z{};
  z.fused_G = 1;
  z.fused_rows = kFusedThreads;
  z.dp = 16;
  const size_t lds = dev::xpass_lds_floats(16, kFusedThreads) * sizeof(float);
  dev::smo_persist_lru_kernel<false, 1><<<1, kFusedThreads, lds, s>>>(z, st, 0, nullptr);
  dev::smo_persist_lru_kernel<false, 2><<<1, kFusedThreads, lds, s>>>(z, st, 0, nullptr);
  dev::smo_persist_lru_kernel<false, 4><<<1, kFusedThreads, lds, s>>>(z, st, 0, nullptr);
  dev::smo_persist_lru_kernel<true, 1><<<1, kFusedThreads, lds, s>>>(z, st, 0, nullptr);
  dev::smo_persist_lru_kernel<true, 2><<<1, kFusedThreads, lds, s>>>(z, st, 0, nullptr);
  dev::smo_persist_lru_kernel<true, 4><<<1, kFusedThreads, lds, s>>>(z, st, 0, nullptr);
  HIP_CHECK(hipStreamSynchronize(s));
  HIP_CHECK(hipGetLastError());
  (void)hipFree(st);
}

}  // namespace launch
}  // namespace dpsvm

// ---------------------------------------------------------------------------
// Kernel-level test entry of the X pass exactly as both cache engines run it
// (xpass_fill): workgroup b fills rows [b * fused_rows, ...) of lines 0..n_new-1
// with K(x_keys[q], x_j).
// ---------------------------------------------------------------------------
namespace dpsvm {
namespace dev {
__global__ __launch_bounds__(kFusedThreads) void xpass_test_kernel(SmoArgs a, const int* __restrict__ keys,
                                                                   int n_new) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  __shared__ int key_s[kNQ], line_s[kNQ], op_s[kNQ];
  const int tid = threadIdx.x;
  if (tid < kNQ) {
    key_s[tid] = tid < n_new ? keys[tid] : 0;
    line_s[tid] = tid;
    op_s[tid] = kOpCompute;
  }
  __syncthreads();
  const int64_t row0 = (int64_t)blockIdx.x * a.fused_rows;
  const int64_t row_end = min((int64_t)a.nl, row0 + (int64_t)a.fused_rows);
  xpass_fill(a, row0, row_end, n_new, key_s, line_s, op_s, wsm, false);
}
}  // namespace dev

namespace launch {
void xpass_rows(const SmoArgs& a, const int* keys_dev, int n_new, hipStream_t s) {
  DPSVM_CHECK(n_new >= 1 && n_new <= kNQ && a.fused_rows % kFusedThreads == 0 && a.dp % 16 == 0,
              "xpass_rows: 1 <= n_new <= 16, rows a multiple of 256, dp a multiple of 16");
  const size_t lds = dev::xpass_lds_floats(a.dp, a.fused_rows) * sizeof(float);
  DPSVM_CHECK(lds <= 160 * 1024, "xpass_rows: LDS");
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute((const void*)dev::xpass_test_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
  const int G = (int)((a.nl + a.fused_rows - 1) / a.fused_rows);
  dev::xpass_test_kernel<<<dim3(G), kFusedThreads, lds, s>>>(a, keys_dev, n_new);
  post_launch("xpass_rows", s);
}
}  // namespace launch
}  // namespace dpsvm
