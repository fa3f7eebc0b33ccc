// Working-set engine: the LDS sub-problem solve on one wave (the reference's
// pair rule, svmTrainMain.cpp:255-299) and the round's commit, run by
// ws_solve.hip (one launch per round).  Round structure and helpers:
// ws_common.hpp.
#pragma once

#include "ws_common.hpp"

namespace dpsvm {
namespace dev {

// ---------------------------------------------------------------------------
// ws_solve: the sub-problem on wave 0
// ---------------------------------------------------------------------------
// Row `pos` (uniform) took alpha `an` and now has gradient fp (both uniform,
// computed from values every lane holds): its I_up / I_low test
// (svmTrain.cu:56-91) as mask logic on uniform operands, then the owner lane's
// slot registers take the new fu / fl by selects.  No branch (every branch of a
// one-wave loop is a fetch bubble) and no per-lane recomputation.
// per lane: the lanes set in the (uniform) mask m take b, the others keep a
__device__ __forceinline__ float sel_lanes(float a, float b, uint64_t m) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}

template <int NS>
__device__ __forceinline__ void ws_place(int pos, float an, float yv, float fp, int lane, float C, float (&fu)[NS],
                                         float (&fl)[NS]) {
  const float INF = __builtin_inff();
  // the operands are uniform: each test as a wave mask (all ones or zero; wave
  // 0 runs with a full exec mask) keeps the set logic on the scalar unit
  // instead of 0/1 VGPRs (~20 VALU per placement)
  // with alpha in [0, C] (clipped), in_up(a, y) == (y > 0 ? a < C : a > 0) and
  // in_low(a, y) == (y > 0 ? a > 0 : a < C) (common.hpp): three compares
  const uint64_t lt = __ballot(an < C), gt = __ballot(an > 0.f), py = __ballot(yv > 0.f);
  const float nu = (((py & lt) | (~py & gt)) != 0) ? fp : INF;
  const float nl = (((py & gt) | (~py & lt)) != 0) ? -fp : INF;
  // the owner lane of slot pos >> 6 as a scalar lane mask per slot, applied by
  // v_cndmask straight from the SGPR pair (no per-lane compare)
  const uint64_t bit = 1ull << (pos & 63);
  const int s = pos >> 6;
  (void)lane;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const uint64_t w = s == k ? bit : 0ull;
    fu[k] = sel_lanes(fu[k], nu, w);
    fl[k] = sel_lanes(fl[k], nl, w);
  }
}

// The reference's pair update (svmTrainMain.cpp:282-295; pair_update in
// common.hpp, same clipping modes) on uniform operands, with the quotient
// y_lo (b_hi - b_lo) / eta from a refined hardware reciprocal: the sub-problem
// step needs no bit parity with the pair-at-a-time engines (f is updated from
// the alphas actually taken, so it stays consistent), and the IEEE division
// sequence is the longest dependent chain of a step.
template <bool kBox>
__device__ __forceinline__ PairUpdate ws_pair_step(float a_hi, float a_lo, float y_hi, float y_lo, float bh, float bl,
                                                   float khl, float C, float tau, bool same, bool* clipped) {
#pragma clang fp contract(off)
  float eta = (1.0f + 1.0f) - 2.0f * khl;
  eta = eta >= tau ? eta : tau;
  float r = __builtin_amdgcn_rcpf(eta);
  r = r + r * __builtin_fmaf(-eta, r, 1.0f);  // one Newton step: ~0.5 ulp
  const float s = y_lo * y_hi;
  float a_lo_new = a_lo + (y_lo * (bh - bl)) * r;
  float a_hi_new;
  if (kBox) {
    // branch-free (every branch of the one-wave loop is a fetch bubble): both
    // box geometries and the same-row case computed, the pair's uniform
    // labels / positions select — the same values the branches produced
    const float dl = a_lo - a_hi, sm = a_lo + a_hi;
    const bool diff = y_hi != y_lo;
    const float L = diff ? (dl > 0.f ? dl : 0.f) : (sm - C > 0.f ? sm - C : 0.f);
    const float hL = diff ? (dl > 0.f ? 0.f : -1.f) : (sm - C > 0.f ? C : -1.f);
    const float H = diff ? (C + dl < C ? C + dl : C) : (sm < C ? sm : C);
    const float hH = diff ? (C + dl < C ? C : -1.f) : (sm < C ? 0.f : -1.f);
    const bool atL = a_lo_new <= L, atH = !atL && a_lo_new >= H;
    const float lo_box = atL ? L : (atH ? H : a_lo_new);
    const float snap = atL ? hL : (atH ? hH : -1.f);
    const float hi_box = clip01(snap >= 0.f ? snap : a_hi + (s * (a_lo - lo_box)), 0.0f, C);
    const float hi_same = clip01(a_hi + (s * (a_lo - a_lo_new)), 0.0f, C);
    const float lo_same = clip01(a_lo_new, 0.0f, C);
    a_lo_new = same ? lo_same : lo_box;
    a_hi_new = same ? hi_same : hi_box;
  } else {
    a_hi_new = a_hi + (s * (a_lo - a_lo_new));
    const float lo_raw = a_lo_new, hi_raw = a_hi_new;
    a_lo_new = clip01(a_lo_new, 0.0f, C);
    a_hi_new = clip01(a_hi_new, 0.0f, C);
    *clipped = (lo_raw != a_lo_new) | (hi_raw != a_hi_new);  // sum(alpha y) no longer kept
  }
  PairUpdate u;
  u.a_hi_new = a_hi_new;
  u.a_lo_new = a_lo_new;
  u.c_hi = (a_hi_new - a_hi) * y_hi;
  u.c_lo = (a_lo_new - a_lo) * y_lo;
  return u;
}

// lowest working-set position whose value equals the (uniform) minimum v
// (-1: none, i.e. NaN); scalar selects, no branch
// s_ff1 of an SGPR-pair mask: the lowest set bit, 0xFFFFFFFF when none (the
// builtins add a zero test and a select per mask)
__device__ __forceinline__ uint32_t sff1_u64(uint64_t m) {
  uint32_t r;
  asm volatile("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m));
  return r;
}

__device__ __forceinline__ int ws_argpos(const float (&x)[3], float v) {
  const uint64_t m0 = __ballot(x[0] == v), m1 = __ballot(x[1] == v), m2 = __ballot(x[2] == v);
  // slot s's first lane | 64 s (none stays all ones), the lowest valid one wins
  // as an unsigned minimum: 3 compares, 3 s_ff1, 2 s_or, 2 s_min
  const uint32_t r0 = sff1_u64(m0), r1 = sff1_u64(m1) | 64u, r2 = sff1_u64(m2) | 128u;
  uint32_t r;
  asm volatile("s_min_u32 %0, %1, %2\n\ts_min_u32 %0, %0, %3" : "=&s"(r) : "s"(r0), "s"(r1), "s"(r2));
  return (int)r;
}

__device__ __forceinline__ int ws_argpos(const float (&x)[1], float v) {
  return (int)sff1_u64(__ballot(x[0] == v));  // -1 (all ones) when none
}

__device__ __forceinline__ int ws_argpos(const float (&x)[2], float v) {
  const uint64_t m0 = __ballot(x[0] == v), m1 = __ballot(x[1] == v);
  const uint32_t r0 = sff1_u64(m0), r1 = sff1_u64(m1) | 64u;
  uint32_t r;
  asm volatile("s_min_u32 %0, %1, %2" : "=s"(r) : "s"(r0), "s"(r1));
  return (int)r;
}

// kFull: q_max == kWsMax, the three 64-row slots fill a sub-Gram row (stride
// 192): row reads need no clamp (columns q..191 hold zeros) and take immediate
// LDS offsets
// kW2: second-order choice of the low row (Fan, Chen & Lin's WSS2, the rule
// LIBSVM uses): hi = argmin f over I_up as in the reference, then lo = the
// I_low row with f_lo > b_hi that maximises (f_lo - b_hi)^2 / eta(hi, lo) —
// the pair whose step gains the most dual objective — instead of argmax f.
// The stop test stays the reference's first-order one (b_lo = max f over I_low).
// NS: 64-row slots per lane (3 for q_max <= 192, 2 for q_max <= 128 — the
// multi-block rounds' 96-row blocks: a third less work per pair step — and 1
// for blocks of <= 64 rows)
// The sub-problem loop and the round's commit, on wave 0 once the q rows are in
// LDS: K (q rows, stride a.q_max), s_a (+ 128 scratch words), s_y, s_f, s_idx,
// s_line.  blk / ib: the block and its first row (multi-block rounds); it0,
// b_hi, b_lo: the round's pair count and global selection at entry; xfail: the
// peer exchange gave up (no step, kCommFail kept).
template <bool kBox, bool kFull, bool kMulti, bool kW2, int NS>
__device__ __forceinline__ void ws_solve_run(const WsArgs& a, WsCtrl* c, const float* K, float* s_a, const float* s_y,
                                             const float* s_f, const int32_t* s_idx, const int32_t* s_line, int q,
                                             int blk, int ib, int64_t it0, float b_hi, float b_lo, bool xfail) {
  static_assert(NS == 3 || ((NS == 2 || NS == 1) && !kFull), "slots");
  const int lane = threadIdx.x & 63;
  const int ldk = a.q_max;
  const float INF = __builtin_inff();
  const float C = a.C;
  const float eps_in = fmaxf(a.eps_floor, a.rel_local * 0.5f * (b_lo - b_hi));
  float fu[NS], fl[NS], yr[NS], a0[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int p = lane + 64 * s;
    const bool v = p < q;
    const float fv = v ? s_f[p] : 0.f;
    a0[s] = v ? s_a[p] : 0.f;
    yr[s] = v ? s_y[p] : 1.f;
    fu[s] = v && in_up(a0[s], yr[s], C) ? fv : INF;
    fl[s] = v && in_low(a0[s], yr[s], C) ? -fv : INF;
  }
  int64_t room = a.max_iter - it0;
  if (kMulti) {  // the active blocks share max_iter
    const int pa = c->p_round;
    room = blk < pa ? room / pa + (blk < room % pa ? 1 : 0) : 0;
  }
  // uniform: in an SGPR, so the loop test is one scalar compare
  const int cap = xfail ? 0 : __builtin_amdgcn_readfirstlane((int)(room < (int64_t)a.inner_max ? room : (int64_t)a.inner_max));
  int inner = 0;
  bool bad = false, clipped_any = false;
  while (inner < cap) {
    float mu = fu[0], ml = fl[0];
    if constexpr (NS >= 2) {
      mu = fminf(mu, fu[1]);
      ml = fminf(ml, fl[1]);
    }
    if constexpr (NS == 3) {
      mu = fminf(mu, fu[2]);
      ml = fminf(ml, fl[2]);
    }
    wave_min2_f32(mu, ml);
    const float bh = mu;
    float bl = -ml;  // first order: b_lo = max f over I_low (also the stop test's)
    const int ph = ws_argpos(fu, mu);
    int pl = -1;
    float kh[NS], kl[NS];
    if constexpr (!kW2) pl = ws_argpos(fl, ml);
    // one exit test: an empty side, the sub-problem's stop test, or NaN
    const bool open = (mu < INF) & (ml < INF) & (bl > bh + 2.0f * eps_in);
    if constexpr (kW2) {
      if (open && ph >= 0) {
        // hi's sub-Gram row first, then the gain of every violating I_low row
        // as a minimum of -gain (INF: not a candidate)
#pragma unroll
        for (int s = 0; s < NS; ++s) kh[s] = K[ph * ldk + (kFull ? lane + 64 * s : min(lane + 64 * s, q - 1))];
        float g[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const float dv = -fl[s] - bh;
          float eta = (1.0f + 1.0f) - 2.0f * kh[s];
          eta = eta >= a.tau ? eta : a.tau;
          // on every lane, then a select: hipcc made each slot's conditional
          // reciprocal an exec-masked branch (three per step)
          float gv = -(dv * dv) * __builtin_amdgcn_rcpf(eta);
          asm volatile("" : "+v"(gv));
          g[s] = ((fl[s] < INF) & (dv > 0.f)) ? gv : INF;
        }
        float gm = g[0];
        if constexpr (NS >= 2) gm = fminf(gm, g[1]);
        if constexpr (NS == 3) gm = fminf(gm, g[2]);
        float gm2 = gm;
        wave_min2_f32(gm, gm2);
        pl = gm < INF ? ws_argpos(g, gm) : -1;
        if (pl >= 0) {
          const int sl = pl >> 6;
          bl = -readlane_f32(sl == 0 || NS == 1 ? fl[0] : (NS == 2 || sl == 1) ? fl[1] : fl[NS - 1], pl & 63);  // f of the chosen lo
        }
      }
    }
    if (!open || (ph | pl) < 0) {
      bad = open;  // a violating pair exists but no position matches it: NaN
      break;
    }
    // every remaining LDS read of the step in one batch: the pair's alphas /
    // labels, the 2 x 2 block K(hi|lo, hi|lo) and the sub-Gram rows
    const float a_hi = s_a[ph], y_hi = s_y[ph], a_lo = s_a[pl], y_lo = s_y[pl];
    const float khl = K[ph * ldk + pl], klh = K[pl * ldk + ph], khh = K[ph * ldk + ph], kll = K[pl * ldk + pl];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int p = kFull ? lane + 64 * s : min(lane + 64 * s, q - 1);
      if constexpr (!kW2) kh[s] = K[ph * ldk + p];
      kl[s] = K[pl * ldk + p];
    }
    bool clipped = false;
    const PairUpdate up = ws_pair_step<kBox>(a_hi, a_lo, y_hi, y_lo, bh, bl, khl, C, a.tau, ph == pl, &clipped);
    if (kMulti && !kBox) clipped_any |= clipped;
    float f_lo_new, f_hi_new;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float dl;
      {
#pragma clang fp contract(off)
        dl = up.c_hi * kh[s] + up.c_lo * kl[s];  // f_apply's delta (device_util.hpp)
        fu[s] = fu[s] + dl;
        fl[s] = fl[s] - dl;  // -(f + delta): exact negation of the same rounding
      }
    }
    {
      // the pair's own new gradients, uniformly: the owners computed exactly
      // these sums (row ph: kh = K(hi,hi), kl = K(lo,hi); row pl: K(hi,lo), K(lo,lo))
#pragma clang fp contract(off)
      f_lo_new = bl + (up.c_hi * khl + up.c_lo * kll);
      f_hi_new = bh + (up.c_hi * khh + up.c_lo * klh);
    }
    ws_place(pl, up.a_lo_new, y_lo, f_lo_new, lane, C, fu, fl);
    ws_place(ph, up.a_hi_new, y_hi, f_hi_new, lane, C, fu, fl);  // hi written last (svmTrainMain.cpp:298-299)
    // lane 0 writes the pair's alphas, the other lanes a private scratch word
    // each (no exec-mask branch in the loop, no bank conflict)
    s_a[lane == 0 ? pl : kWsMax + lane] = up.a_lo_new;
    s_a[lane == 0 ? ph : kWsMax + 64 + lane] = up.a_hi_new;
    ++inner;
  }
  // ---- commit: alphas, the changed rows for the f update, control, status ----
  int n_apply = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int p = lane + 64 * s;
    const float an = p < q ? s_a[p] : 0.f;
    const bool nz = p < q && an != a0[s];
    const uint64_t mk = __ballot(nz);
    const int at = n_apply + __popcll(mk & ((1ull << lane) - 1ull));
    if (nz) {
      const int32_t gi = s_idx[p];
      a.alpha[gi] = an;
      float dc;
      {
#pragma clang fp contract(off)
        dc = (an - a0[s]) * yr[s];
      }
      c->apply_idx[ib + at] = gi;
      c->apply_line[ib + at] = s_line[p];
      c->apply_coef[ib + at] = dc;
      if (kMulti) a.dalpha[gi] = an - a0[s];
    }
    n_apply += __popcll(mk);
  }
  if (lane == 0 && !kMulti) {
    WS_STAMP(4);
    if (a.stamps) a.stamps[(size_t)(c->outer % kStampRing) * 2 * kStampSlots + 5] = (uint64_t)inner;
    c->iter = it0 + inner;
    c->outer = c->outer + 1;
    if (xfail) {
      c->n_apply = 0;  // the exchange poll gave up (peer exchange): the run ends here, kCommFail kept
    } else {
      c->n_apply = n_apply;
      c->done = bad ? kNonFinite : inner == 0 ? kNoPair : (it0 + inner >= a.max_iter ? kMaxIter : kRunning);
    }
    ws_status(a.status, c);
  }
  if (kMulti) {
    // publish this block's counts; the last block to finish commits the round
    // (threadfence + counter: no workgroup waits for another)
    int prev = 0;
    if (lane == 0) {
      c->nab[blk] = n_apply;
      c->inb[blk] = inner;
      c->badb[blk] = bad ? 1 : 0;
      c->clipb[blk] = clipped_any ? 1 : 0;
      __threadfence();
      prev = atomicAdd(&c->solve_cnt, 1);
    }
    prev = __builtin_amdgcn_readfirstlane(prev);
    int tot_a = 0, tot_i = 0, any_bad = 0, any_clip = 0;
    if (prev == a.blocks - 1) {  // uniform
      __threadfence();
      // the P blocks' counts: every lane loads its blocks' (all loads in flight;
      // one lane walking 128 blocks' agent-scope loads serialised them), then
      // wave sums
      for (int p = lane; p < a.blocks; p += 64) {
        tot_a += __hip_atomic_load(&c->nab[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tot_i += __hip_atomic_load(&c->inb[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        any_bad |= __hip_atomic_load(&c->badb[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        any_clip |= __hip_atomic_load(&c->clipb[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        tot_a += __shfl_xor(tot_a, o);
        tot_i += __shfl_xor(tot_i, o);
        any_bad |= __shfl_xor(any_bad, o);
        any_clip |= __shfl_xor(any_clip, o);
      }
    }
    if (lane == 0 && prev == a.blocks - 1) {
      c->solve_cnt = 0;
      // the reference's independent clipping does not keep sum(alpha y) = 0: once
      // a clip broke it, the blocks' combined steps drift it further (measured:
      // adult-shape P = 8 never converges) — one block per round from here on
      WS_STAMP(4);
      if (a.stamps) a.stamps[(size_t)(c->outer % kStampRing) * 2 * kStampSlots + 5] = (uint64_t)tot_i;
      c->n_apply = tot_a;
      c->iter = it0 + tot_i;
      c->outer = c->outer + 1;
      if (any_clip && a.clip_fallback && c->p_act > 1) {
        c->p_act = 1;
        if (c->p1_round == 0) c->p1_round = c->outer;
      }
      if (__hip_atomic_load(&c->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kCommFail) {
        c->n_apply = 0;  // a block's exchange poll gave up (peer exchange): the run ends here
      } else {
        c->done = any_bad ? kNonFinite : tot_i == 0 ? kNoPair : (it0 + tot_i >= a.max_iter ? kMaxIter : kRunning);
      }
      ws_status(a.status, c);
    }
  }
}

}  // namespace dev
}  // namespace dpsvm
