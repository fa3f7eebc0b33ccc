// Working-set engine, selection pass (ws_select): the round's alpha changes
// applied to every f_j — one pass, or the two passes around the multi-block
// line search — then each workgroup's candidate keys per side.  Round
// structure and shared helpers: ws_common.hpp.
#include <hip/hip_runtime.h>

#include "dpsvm/common.hpp"
#include "dpsvm/device_state.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "ws_common.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

// ---------------------------------------------------------------------------
// ws_select: f update of the last round + per-workgroup candidates
// ---------------------------------------------------------------------------
// Threads of a workgroup: 256 rows (x RPT) times PARTS partitions of the
// changed-row list.  Each partition sums its contiguous slice of the list in
// list order; the slices combine in partition order — the rounding depends on
// the list only (never on the grid or the rank count), and every thread has at
// most ~48 Gram loads of one batch in flight instead of a chain of batches.
template <int RPT>
constexpr int ws_parts() {
  // register budget: <= 4 waves per SIMD at RPT <= 4, 2 up to 16, 1 at 32 (2M rows on one GPU)
  return RPT <= 4 ? 4 : RPT <= 16 ? 2 : 1;
}

// MODE 0: one pass (f += the round's change, then candidates).  Multi-block
// rounds split it: MODE 1 computes the change d_f into a.dfs and per-workgroup
// partial sums of the line search (d'Qd = sum_j c_j d_f_j and g'd = -sum_j c_j
// f_j over the changed rows j, c_j = d_alpha_j y_j), MODE 2 takes
// t = min(1, g'd / d'Qd) from the partials (fixed order: every workgroup the
// same t), applies f += t d_f and alpha = alpha_new - (1 - t) d_alpha, then
// selects the candidates.  Pass 2 walks no list: one partition, 256 threads.
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

template <int RPT, int MODE>
constexpr int ws_sel_parts() {
  return MODE == 2 ? 1 : ws_parts<RPT>();
}

template <int RPT, int MODE>
__global__ __launch_bounds__((kWsSelThreads * ws_sel_parts<RPT, MODE>())) void ws_select_kernel(WsArgs a) {
  constexpr int PARTS = ws_sel_parts<RPT, MODE>();
  constexpr int CH = RPT >= 32 ? 1 : RPT >= 8 ? 4 : 48 / RPT;  // Gram loads in flight per thread (vmcnt <= 63)
  constexpr int LMAX = MODE == 1 ? kWsMaxAll : MODE == 0 ? kWsMax : 1;
  __shared__ int32_t s_idx[LMAX];  // lines of the changed rows
  __shared__ float s_coef[LMAX];
  __shared__ double s_red[2][kWsSelThreads * PARTS / 64];
  __shared__ double s_red_tot[2];
  __shared__ float s_part[PARTS > 1 ? PARTS - 1 : 1][PARTS > 1 ? kWsSelThreads * RPT : 1];
  __shared__ uint64_t s_wc[kWsSelThreads / 64][2][kWsCand];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x & (kWsSelThreads - 1), part = threadIdx.x / kWsSelThreads;
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(MODE == 1 ? 22 : 6);  // pass 1: own slots (22, 23)
  const int na = c->n_apply;
  const int done = c->done;
  if (na == 0 && (done != kRunning || MODE == 1)) return;
  if constexpr (MODE == 0) {
    for (int k = threadIdx.x; k < na; k += kWsSelThreads * PARTS) {
      s_idx[k] = c->apply_line[k];
      s_coef[k] = c->apply_coef[k];
    }
  }
  // a workgroup owns a.rpt x 256 rows (ws_geometry); RPT (>= a.rpt) only sizes the registers.
  // MODE 1 runs KS = a.ks workgroups per row group, each over its KS-th of the
  // changed-row list (pass 1 fills the device when G is small: 30 groups per rank at
  // 8 ranks on the headline); pass 2 sums the KS partial changes in slice order.
  const int KS = MODE == 1 ? max(1, a.ks) : 1;
  const int grp = MODE == 1 ? (int)(blockIdx.x % a.G) : (int)blockIdx.x, ksi = MODE == 1 ? (int)(blockIdx.x / a.G) : 0;
  if constexpr (MODE == 1) {
    // the blocks' apply segments, concatenated in block order; this workgroup
    // loads only its slice [e_lo, e_hi) of the list (at their list positions)
    const int per_wg = PARTS * ((na + PARTS * KS - 1) / (PARTS * KS));
    const int e_lo = min(na, ksi * per_wg), e_hi = min(na, e_lo + per_wg);
    int at = 0;
    for (int p = 0; p < a.blocks && at < e_hi; ++p) {
      const int nb = c->nab[p];
      const int k0 = max(0, e_lo - at), k1 = min(nb, e_hi - at);
      for (int k = k0 + threadIdx.x; k < k1; k += kWsSelThreads * PARTS) {
        s_idx[at + k] = c->apply_line[p * a.q_max + k];
        s_coef[at + k] = c->apply_coef[p * a.q_max + k];
      }
      at += nb;
    }
  }
  __syncthreads();
  const int64_t base = (int64_t)grp * a.rpt * kWsSelThreads + tid;
  float f[RPT];
  bool has[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int64_t j = base + (int64_t)r * kWsSelThreads;
    has[r] = r < a.rpt && j < a.nl;
    f[r] = has[r] && part == 0 ? a.f[j] : 0.f;
  }
  if (na > 0) {
    float acc[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) acc[r] = 0.f;
    if constexpr (MODE != 2) {
    const int per = (na + PARTS * KS - 1) / (PARTS * KS);
    const int k_lo = min(na, (ksi * PARTS + part) * per), k_hi = min(na, k_lo + per);
    for (int k0 = k_lo; k0 < k_hi; k0 += CH) {
      float kv[CH][RPT];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int kk = min(k0 + u, k_hi - 1);
        const float* row = a.gram + (int64_t)s_idx[kk] * a.ldg;
#pragma unroll
        for (int r = 0; r < RPT; ++r) kv[u][r] = has[r] ? row[base + r * kWsSelThreads] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        if (k0 + u < k_hi) {
          const float cc = s_coef[k0 + u];
#pragma unroll
          for (int r = 0; r < RPT; ++r) acc[r] = f_add1(acc[r], cc, kv[u][r]);
        }
      }
    }
    if (PARTS > 1) {
      if (part > 0) {
#pragma unroll
        for (int r = 0; r < RPT; ++r) s_part[part - 1][r * kWsSelThreads + tid] = acc[r];
      }
      __syncthreads();
#pragma unroll
      for (int p = 1; p < PARTS; ++p) {
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
#pragma clang fp contract(off)
          acc[r] = acc[r] + s_part[p - 1][r * kWsSelThreads + tid];
        }
      }
    }
    }  // MODE != 2
    if constexpr (MODE == 1) {
      double sq = 0.0, sg = 0.0;
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        if (has[r] && part == 0) {
          const int64_t j = base + r * kWsSelThreads;
          a.dfs[(int64_t)ksi * a.nl + j] = acc[r];
          const float dj = a.dalpha[a.off + j];
          if (dj != 0.f) {
            const double cj = (double)dj * (double)a.y[a.off + j];
            sq += cj * (double)acc[r];  // d'Qd is linear in the KS partial changes
            if (ksi == 0) sg -= cj * (double)f[r];
          }
        }
      }
      // fixed-order block sums (butterfly per wave, waves in order)
      sq = wave_sum_f64(sq);
      sg = wave_sum_f64(sg);
      const int w = threadIdx.x >> 6;
      if ((threadIdx.x & 63) == 0) {
        s_red[0][w] = sq;
        s_red[1][w] = sg;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        double tq = 0.0, tg = 0.0;
        for (int k = 0; k < kWsSelThreads * PARTS / 64; ++k) {
          tq += s_red[0][k];
          tg += s_red[1][k];
        }
        s_red_tot[0] = tq;
        s_red_tot[1] = tg;
        const int64_t slot = ((int64_t)a.rank * a.p1G + grp) * KS + ksi;
        a.part[2 * slot] = tq;
        a.part[2 * slot + 1] = tg;
        if (blockIdx.x == 0) WS_STAMP(23);
      }
      __syncthreads();  // s_red_tot
      if (a.xpeer != nullptr && threadIdx.x < 64 && (threadIdx.x >> 1) < a.world) {
        // peer exchange: the slot's two doubles to every rank (lanes 2 p, 2 p + 1: rank p)
        const int64_t slot = ((int64_t)a.rank * a.p1G + grp) * KS + ksi;
        const int64_t R = c->outer;  // committed by this round's solve
        const uint64_t t = xtag((uint32_t)R + 1u);
        const int pr = threadIdx.x >> 1, h = threadIdx.x & 1;
        const double v = h ? s_red_tot[1] : s_red_tot[0];
        ws_put64(a.xpeer[pr] + ws_xpart(a, (int)(R & 1), slot) + 2 * h, t, (uint64_t)__double_as_longlong(v));
      }
      return;
    }
    if constexpr (MODE == 2) {
      const int pr = c->p_round;  // written by this round's merge (p_act may change below)
      const float t = ws_line_search(a, pr);
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->t_last = t;
        if (t < 1.f) {
          // strongly coupled blocks: fewer from the next round on (the solve's
          // commit may have set p_act = 1 already: an independent-clip event)
          c->n_damped = c->n_damped + 1;
          const int np = t < a.t_halve ? max(1, pr / 2) : pr;
          if (np < c->p_act) c->p_act = np;
          if (c->p_act == 1 && c->p1_round == 0) c->p1_round = c->outer;
          ws_status(a.status, c);  // p1_round visible with the round that set it (gpu_engines.hip)
        }
      }
      if (a.world > 1 && blockIdx.x == 0) {
        // alpha is global on every rank: the changed rows this rank does not own
        // (its threads below fix the owned ones before classifying them)
        // (the P segments' slots flat over the threads: every count and row load
        // in flight at once, not one block's count after another)
        const int slots = a.blocks * a.q_max;
        for (int i = threadIdx.x; i < slots; i += kWsSelThreads * PARTS) {
          const int p = i / a.q_max, k = i - p * a.q_max;
          if (k >= c->nab[p]) continue;
          const int64_t gi = c->apply_idx[i];
          if (gi >= a.off && gi < a.off + a.nl) continue;
          if (t < 1.f) a.alpha[gi] = clip01(a.alpha[gi] - (1.f - t) * a.dalpha[gi], 0.f, a.C);
          a.dalpha[gi] = 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        if (has[r] && part == 0) {
          const int64_t j = base + r * kWsSelThreads;
          float d = a.dfs[j];
          for (int k = 1; k < a.ks; ++k) {
#pragma clang fp contract(off)
            d = d + a.dfs[(int64_t)k * a.nl + j];
          }
          acc[r] = t == 1.f ? d : t * d;
          const float dj = a.dalpha[a.off + j];
          if (dj != 0.f) {
            if (t < 1.f) a.alpha[a.off + j] = clip01(a.alpha[a.off + j] - (1.f - t) * dj, 0.f, a.C);
            a.dalpha[a.off + j] = 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
#pragma clang fp contract(off)
      f[r] = f[r] + acc[r];
    }
    bool bad = false;
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      if (has[r] && part == 0) a.f[base + r * kWsSelThreads] = f[r];
      bad |= has[r] && part == 0 && !isfinite(f[r]);
    }
    if (bad) atomicOr(&c->nonfinite, 1);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(10);
  if (done != kRunning) return;  // uniform

  // partition 0 (waves 0..3) classifies and extracts; the other waves idle to
  // the one barrier below (no wave leaves before it)
  uint64_t ku[RPT], kl[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    ku[r] = kl[r] = kKeyNone;
    if (has[r] && part == 0) {
      const int64_t gj = a.off + base + r * kWsSelThreads;
      const float av = a.alpha[gj], yv = a.y[gj];
      if (in_up(av, yv, a.C)) ku[r] = make_key(f[r], (uint32_t)gj);
      if (in_low(av, yv, a.C)) kl[r] = make_key(-f[r], (uint32_t)gj);
    }
  }
  // each wave's nc smallest keys per side, then wave 0 merges the four lists.
  // Keys are unique (the global index is in the low bits) except kKeyNone, the
  // largest: a key's place is the count of smaller keys, kKeyNone's the real
  // keys' count plus its order among the lanes holding kKeyNone — a
  // permutation, so every place is written once.  One row per thread (RPT 1,
  // every rank of up to 60,160 rows): each lane counts over its wave's 64 keys
  // (broadcast LDS reads, no barrier) instead of nc rounds of wave minima
  const int lane = tid & 63, wave = tid >> 6;
  // multi-block merges read ws_ncand keys per list (MODE 2: every multi-block
  // round, the seed included; the list's tail is kKeyNone), the one-block
  // merge kWsCand1 (MODE 0)
  constexpr int NC = MODE == 0 ? kWsCand1 : kWsCand;  // register capacity
  const int nc = MODE == 0 ? kWsCand1 : ws_ncand(a.ncand);
  constexpr int W = kWsSelThreads / 64;
  const uint64_t below = (1ull << lane) - 1ull;
  // place of key k among the wave's keys, given the count of smaller ones
  auto place = [&](uint64_t k, int smaller) {
    const uint64_t none = __ballot(k == kKeyNone);
    return k == kKeyNone ? 64 - __popcll(none) + __popcll(none & below) : smaller;
  };
  if constexpr (RPT == 1) {
    __shared__ u64x2 s_kk[W][2][32];  // [wave][side] the wave's 64 keys
    if (part == 0) {
      const uint64_t mu = ku[0], ml = kl[0];
      ((uint64_t*)s_kk[wave][0])[lane] = mu;
      ((uint64_t*)s_kk[wave][1])[lane] = ml;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own stores, read by its lanes
      int cu = 0, cl = 0;
#pragma unroll 8
      for (int m = 0; m < 32; ++m) {
        const u64x2 vu = s_kk[wave][0][m], vl = s_kk[wave][1][m];
        cu += (vu.x < mu ? 1 : 0) + (vu.y < mu ? 1 : 0);
        cl += (vl.x < ml ? 1 : 0) + (vl.y < ml ? 1 : 0);
      }
      const int pu = place(mu, cu), pl = place(ml, cl);
      if (pu < nc) s_wc[wave][0][pu] = mu;
      if (pl < nc) s_wc[wave][1][pl] = ml;
    }
  } else {
    for (int round = 0; round < nc && part == 0; ++round) {
      uint64_t mu = kKeyNone, ml = kKeyNone;
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        mu = ku[r] < mu ? ku[r] : mu;
        ml = kl[r] < ml ? kl[r] : ml;
      }
      mu = wave_min_u64(mu);
      ml = wave_min_u64(ml);
      if (lane == 0) {
        s_wc[wave][0][round] = mu;
        s_wc[wave][1][round] = ml;
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        if (ku[r] == mu) ku[r] = kKeyNone;
        if (kl[r] == ml) kl[r] = kKeyNone;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    // lane l: entry l % kWsCand of wave l / kWsCand's list (W x kWsCand = 64)
    static_assert(W * kWsCand == 64, "one merge entry per lane");
    __shared__ uint64_t s_top[2][NC];
    const bool have = lane % kWsCand < nc;  // the waves' nc entries
    const uint64_t eu = have ? s_wc[lane / kWsCand][0][lane % kWsCand] : kKeyNone;
    const uint64_t el = have ? s_wc[lane / kWsCand][1][lane % kWsCand] : kKeyNone;
    int cu = 0, cl = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        if (r < nc) {  // uniform
          cu += s_wc[w][0][r] < eu ? 1 : 0;
          cl += s_wc[w][1][r] < el ? 1 : 0;
        }
      }
    }
    const int pu = place(eu, cu), pl = place(el, cl);
    if (pu < NC) s_top[0][pu] = pu < nc ? eu : kKeyNone;  // multi-block lists: the tail past nc is kKeyNone
    if (pl < NC) s_top[1][pl] = pl < nc ? el : kKeyNone;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint64_t* out = a.cand_out + (size_t)blockIdx.x * 2 * kWsCand;
    if (lane < NC) out[lane] = s_top[0][lane];
    else if (lane >= 32 && lane < 32 + NC) out[kWsCand + lane - 32] = s_top[1][lane - 32];
    if (a.xpeer != nullptr && lane < a.world) {
      // lane p publishes to rank p: the nc keys per side the merge of this
      // engine reads (slot width a.xcw: up keys at 0, low keys at a.xcw / 2)
      uint64_t* dst = a.xpeer[lane] + ws_xcand(a, (int)(c->outer & 1), a.xrank * a.G + blockIdx.x);
      const uint64_t t = xtag((uint32_t)c->outer + 1u);
      const int lo = a.xcw / 2;
#pragma unroll
      for (int r = 0; r < NC; ++r) {
        if (r < nc) {
          ws_put64(dst + 2 * r, t, s_top[0][r]);
          ws_put64(dst + lo + 2 * r, t, s_top[1][r]);
        }
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(7);
}

// Multi-block pass 1, wide layout (a.p1v4): the same sums as MODE 1 — d_f_j =
// sum_k c_k K(k, j) over the round's changed rows, each partition over a
// contiguous slice of the list in list order, partitions combined in order,
// slices summed in order by pass 2 — but a workgroup owns 1024 columns and a
// thread 4 adjacent ones (16-B row loads): each wave reads 1 KiB of a changed
// Gram row per load instead of 256 B (HBM row-buffer locality of the scattered
// rows), and p1G = ceil(nl_max / 1024) groups x ks list slices fill the device.
// TPP threads per partition x PARTS partitions = 1024 threads; a workgroup owns
// 4 TPP columns (TPP 256: 1024 columns, four partitions — the default; TPP 512:
// 2048 columns, two partitions — A/B, DPSVM_P1_COLS=2048).  NT: the Gram rows
// by non-temporal loads (each changed row is read once a round: no L2 / MALL
// reuse to keep; ws_pass1_nt picks it)
constexpr int kP1Threads = 4 * kWsSelThreads;
template <int TPP, bool NT, int CH = 12>  // CH rows x 16 B in flight per thread
__global__ __launch_bounds__(kP1Threads) void ws_pass1_v4_kernel(WsArgs a) {
  constexpr int PARTS = kP1Threads / TPP;
  constexpr int kP1Cols = 4 * TPP;                  // columns per workgroup
  __shared__ int32_t s_idx[kWsMaxAll];
  __shared__ float s_coef[kWsMaxAll];
  __shared__ f4 s_part[PARTS - 1][TPP];
  __shared__ int s_off[kWsMaxBlocks];
  __shared__ double s_red[2][kP1Threads / 64];
  __shared__ double s_red_tot[2];
  WsCtrl* c = a.ctrl;
  const int tid = threadIdx.x & (TPP - 1), part = threadIdx.x / TPP;
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(22);
  const int na = c->n_apply;
  if (na == 0) return;
  const int KS = max(1, a.ks);
  const int grp = (int)(blockIdx.x % a.p1G), ksi = (int)(blockIdx.x / a.p1G);
  {  // this workgroup's slice [e_lo, e_hi) of the blocks' concatenated apply segments
    const int per_wg = PARTS * ((na + PARTS * KS - 1) / (PARTS * KS));
    const int e_lo = min(na, ksi * per_wg), e_hi = min(na, e_lo + per_wg);
    // the segments' offsets: one wave's prefix scan of the P counts (two blocks
    // a lane) — a walk over 128 blocks' counts, one dependent load after another,
    // held up every workgroup's first row load by ~10 us
    static_assert(kWsMaxBlocks <= 128, "two blocks per lane");
    if (threadIdx.x < 64) {
      const int l = threadIdx.x, P = a.blocks;
      const int n0 = 2 * l < P ? c->nab[2 * l] : 0, n1 = 2 * l + 1 < P ? c->nab[2 * l + 1] : 0;
      int inc = n0 + n1;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o);
        if (l >= o) inc += v;
      }
      s_off[2 * l] = inc - n0 - n1;  // exclusive: block 2 l starts here
      s_off[2 * l + 1] = inc - n1;
    }
    __syncthreads();
    for (int e = e_lo + (int)threadIdx.x; e < e_hi; e += kP1Threads) {
      int lo = 0, hi = a.blocks - 1;  // the last block whose segment starts at or before e
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= e) lo = mid;
        else hi = mid - 1;
      }
      const int k = e - s_off[lo];
      s_idx[e] = c->apply_line[lo * a.q_max + k];
      s_coef[e] = c->apply_coef[lo * a.q_max + k];
    }
  }
  __syncthreads();
  const int64_t j0 = (int64_t)grp * kP1Cols + 4 * tid;
  const bool has = j0 < a.nl;  // j0 + 4 <= round_up(nl, 4) <= ldg: the 16-B load stays in the row
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int per = (na + PARTS * KS - 1) / (PARTS * KS);
  const int k_lo = min(na, (ksi * PARTS + part) * per), k_hi = min(na, k_lo + per);
  for (int k0 = k_lo; k0 < k_hi; k0 += CH) {
    f4 kv[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int kk = min(k0 + u, k_hi - 1);
      const float* row = a.gram + (int64_t)s_idx[kk] * a.ldg;
      if constexpr (NT)
        kv[u] = has ? __builtin_nontemporal_load((const f4*)(row + j0)) : f4{0.f, 0.f, 0.f, 0.f};
      else
        kv[u] = has ? *(const f4*)(row + j0) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      if (k0 + u < k_hi) {
        const float cc = s_coef[k0 + u];
        acc.x = f_add1(acc.x, cc, kv[u].x);
        acc.y = f_add1(acc.y, cc, kv[u].y);
        acc.z = f_add1(acc.z, cc, kv[u].z);
        acc.w = f_add1(acc.w, cc, kv[u].w);
      }
    }
  }
  if (part > 0) s_part[part - 1][tid] = acc;
  __syncthreads();
  double sq = 0.0, sg = 0.0;
  if (part == 0) {
#pragma unroll
    for (int p = 1; p < PARTS; ++p) {
#pragma clang fp contract(off)
      const f4 o = s_part[p - 1][tid];
      acc.x = acc.x + o.x;
      acc.y = acc.y + o.y;
      acc.z = acc.z + o.z;
      acc.w = acc.w + o.w;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t j = j0 + e;
      if (has && j < a.nl) {
        a.dfs[(int64_t)ksi * a.nl + j] = acc[e];
        const float dj = a.dalpha[a.off + j];
        if (dj != 0.f) {
          const double cj = (double)dj * (double)a.y[a.off + j];
          sq += cj * (double)acc[e];  // d'Qd is linear in the KS partial changes
          if (ksi == 0) sg -= cj * (double)a.f[j];
        }
      }
    }
  }
  // fixed-order block sums (butterfly per wave, waves in order)
  sq = wave_sum_f64(sq);
  sg = wave_sum_f64(sg);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_red[0][w] = sq;
    s_red[1][w] = sg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tq = 0.0, tg = 0.0;
    for (int k = 0; k < kP1Threads / 64; ++k) {
      tq += s_red[0][k];
      tg += s_red[1][k];
    }
    s_red_tot[0] = tq;
    s_red_tot[1] = tg;
    const int64_t slot = ((int64_t)a.rank * a.p1G + grp) * KS + ksi;
    a.part[2 * slot] = tq;
    a.part[2 * slot + 1] = tg;
    if (blockIdx.x == 0) WS_STAMP(23);
  }
  __syncthreads();  // s_red_tot
  if (a.xpeer != nullptr && threadIdx.x < 64 && (threadIdx.x >> 1) < a.world) {
    // peer exchange: the slot's two doubles to every rank (lanes 2 p, 2 p + 1: rank p)
    const int64_t slot = ((int64_t)a.rank * a.p1G + grp) * KS + ksi;
    const int64_t R = c->outer;  // committed by this round's solve
    const uint64_t t = xtag((uint32_t)R + 1u);
    const int pr = threadIdx.x >> 1, h = threadIdx.x & 1;
    const double v = h ? s_red_tot[1] : s_red_tot[0];
    ws_put64(a.xpeer[pr] + ws_xpart(a, (int)(R & 1), slot) + 2 * h, t, (uint64_t)__double_as_longlong(v));
  }
}

// Multi-block rounds over the peer exchange: every rank's line-search partials
// (pushed by pass 1 into this rank's receive buffer) into a.part, the layout the
// all-gather leaves — pass 2 then reads them as from the collective.  Runs when
// pass 1 ran (the round applies changes).
__global__ __launch_bounds__(256) void ws_xcollect_part_kernel(WsArgs a) {
  WsCtrl* c = a.ctrl;
  if (c->n_apply == 0) return;  // pass 1 pushed nothing (or the run ended: n_apply = 0)
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(17);
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= ws_nparts(a)) return;
  const int64_t R = c->outer;  // committed by this round's solve, as pass 1 tagged it
  uint64_t v[4];
  if (ws_poll<4>(a, a.xpeer[a.xrank] + ws_xpart(a, (int)(R & 1), k), xtag((uint32_t)R + 1u), v)) {
    a.part[2 * k] = __longlong_as_double((long long)ws_get64(v[0], v[1]));
    a.part[2 * k + 1] = __longlong_as_double((long long)ws_get64(v[2], v[3]));
  } else {
    ws_comm_fail_thread(a, c);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) WS_STAMP(19);
}

}  // namespace dev

namespace launch {

void ws_xcollect_part(const WsArgs& a, hipStream_t s) {
  const int64_t slots = (int64_t)a.world * a.p1G * std::max(1, a.ks);
  dev::ws_xcollect_part_kernel<<<dim3((unsigned)((slots + 255) / 256)), 256, 0, s>>>(a);
  post_launch("ws_xcollect_part", s);
}

int ws_pass1_splits(int G) {
  // about one pass-1 workgroup per CU of the 256-CU device: the selection
  // geometry gives a rank of P only G = ceil(60000 / P / 256) groups on the
  // headline (30 at P = 8), and pass 1 is then bound by the few CUs issuing
  // loads — 3,072 changed rows x 7,500 columns: 114 us with 30 workgroups, 38 us
  // with 240; with 60,000 columns 235 workgroups beat 470 / 705 (158 vs 167 /
  // 189 us; profiles/r3_pass1_probe.txt).  Every rank uses the same G, so the
  // same slice count and the same summation order.
  return std::max(1, std::min(kWsMaxPass1Splits, 256 / std::max(1, G)));
}

void ws_geometry(int64_t nl_max, int world, int32_t* G, int32_t* rpt) {
  // every rank the same geometry (sized for the largest shard); the merge reads
  // world * G <= 1024 candidate lists (kWsListsPerThread per merge thread), so
  // up to 8 ranks keep 128-256 selection workgroups each
  const int64_t gmax = std::max<int64_t>(
      1, std::min<int64_t>(kWsMaxGroups, (int64_t)kWsListsPerThread * 256 / std::max(1, world)));
  const int64_t g = std::max<int64_t>(1, std::min<int64_t>(gmax, (nl_max + kWsSelThreads - 1) / kWsSelThreads));
  const int64_t r = (nl_max + g * kWsSelThreads - 1) / (g * kWsSelThreads);
  *G = (int32_t)g;
  *rpt = (int32_t)std::max<int64_t>(1, r);
}

bool ws_supported(int64_t nl_max, int world, int q_max) {
  int32_t G = 0, rpt = 0;
  ws_geometry(nl_max, world, &G, &rpt);
  return q_max >= 2 && q_max <= kWsMax && rpt <= kWsMaxRPT && nl_max < (int64_t)1 << 31 && world <= kWsMaxGroups;
}

template <int MODE>
static void ws_select_mode(const WsArgs& a, hipStream_t s) {
  const dim3 grid(a.G * (MODE == 1 ? std::max(1, a.ks) : 1));
  auto threads = [](int rpt) { return dim3(MODE == 2 ? kWsSelThreads : kWsSelThreads * (rpt <= 4 ? 4 : rpt <= 16 ? 2 : 1)); };
  if (a.rpt <= 1) dev::ws_select_kernel<1, MODE><<<grid, threads(1), 0, s>>>(a);
  else if (a.rpt <= 2) dev::ws_select_kernel<2, MODE><<<grid, threads(2), 0, s>>>(a);
  else if (a.rpt <= 4) dev::ws_select_kernel<4, MODE><<<grid, threads(4), 0, s>>>(a);
  else if (a.rpt <= 8) dev::ws_select_kernel<8, MODE><<<grid, threads(8), 0, s>>>(a);
  else if (a.rpt <= 16) dev::ws_select_kernel<16, MODE><<<grid, threads(16), 0, s>>>(a);
  else dev::ws_select_kernel<32, MODE><<<grid, threads(32), 0, s>>>(a);
  post_launch("ws_select", s);
}

void ws_select(const WsArgs& a, hipStream_t s) {
  if (a.blocks > 1) {
    ws_select_pass(a, 1, s);  // d_f + line-search partials
    ws_select_mode<2>(a, s);  // f += t d_f, candidates
  } else {
    ws_select_mode<0>(a, s);
  }
}

// columns per wide pass-1 workgroup (A/B: DPSVM_P1_COLS=2048)
int ws_pass1_v4_cols() {
  static const int cols = [] {
    const char* e = std::getenv("DPSVM_P1_COLS");
    return e && atoi(e) == 2048 ? 2048 : 1024;
  }();
  return cols;
}

// the wide pass 1's Gram row loads: non-temporal where the Gram is far larger
// than the 256 MB MALL (> 1 GiB: the rows of a round are not read again before
// they would be evicted) — headline 0.0170 -> 0.0160 s, same trajectory
// (profiles/r6_p1_nt_ab.txt); default policy below, where a small Gram's rows
// stay MALL-resident from round to round.  DPSVM_P1_NT=0 / 1 forces it.
static bool ws_pass1_nt(const WsArgs& a) {
  static const int env = [] {
    const char* e = std::getenv("DPSVM_P1_NT");
    return e ? atoi(e) : -1;
  }();
  if (env == 0 || env == 1) return env == 1;
  const int64_t lines = a.cache ? (int64_t)a.L : a.n;
  return lines * a.ldg * (int64_t)sizeof(float) > (int64_t(1) << 30);
}

// rows in flight per thread of the non-temporal wide pass 1 (A/B: DPSVM_P1_CH=8 / 16)
static int ws_pass1_ch() {
  static const int ch = [] {
    const char* e = std::getenv("DPSVM_P1_CH");
    const int v = e ? atoi(e) : 12;
    return v == 8 || v == 16 ? v : 12;
  }();
  return ch;
}

void ws_select_pass(const WsArgs& a, int pass, hipStream_t s) {
  if (pass == 1 && a.p1v4) {
    const dim3 g(a.p1G * std::max(1, a.ks));
    if (ws_pass1_v4_cols() == 2048)
      dev::ws_pass1_v4_kernel<512, false><<<g, dev::kP1Threads, 0, s>>>(a);
    else if (ws_pass1_nt(a) && ws_pass1_ch() == 16)
      dev::ws_pass1_v4_kernel<256, true, 16><<<g, dev::kP1Threads, 0, s>>>(a);
    else if (ws_pass1_nt(a) && ws_pass1_ch() == 8)
      dev::ws_pass1_v4_kernel<256, true, 8><<<g, dev::kP1Threads, 0, s>>>(a);
    else if (ws_pass1_nt(a))
      dev::ws_pass1_v4_kernel<256, true><<<g, dev::kP1Threads, 0, s>>>(a);
    else
      dev::ws_pass1_v4_kernel<256, false><<<g, dev::kP1Threads, 0, s>>>(a);
    post_launch("ws_pass1_v4", s);
  } else if (pass == 1) {
    ws_select_mode<1>(a, s);
  } else {
    ws_select_mode<2>(a, s);
  }
}

int ws_pass1_v4_groups(int64_t nl_max) {
  const int64_t cols = ws_pass1_v4_cols();
  return (int)std::max<int64_t>(1, (nl_max + cols - 1) / cols);
}

// the wide pass 1's list slices: about one workgroup per CU (the headline at one
// rank: 59 groups x 4 slices; a rank of 8: 8 groups x 32 slices)
int ws_pass1_v4_splits(int p1G) { return std::max(1, std::min(2 * kWsMaxPass1Splits, 256 / std::max(1, p1G))); }

}  // namespace launch
}  // namespace dpsvm
