// RBF GEMM on fp16 MFMA with split operands (v_mfma_f32_32x32x16_f16): the
// fp32 dot products of the Gram at fp32 accuracy for 3/16 of the f32-MFMA time.
//
// Why: the f32-input MFMA (rbf_gemm.hip) runs at 1/16 of the f16 rate, and the
// Gram GEMM is half of the headline solve.  Every X row is scaled by a power of
// two (its largest |x| to [2^14, 2^15)) and split into two fp16 planes,
//     x * 2^s = h + l,   h = fp16(x 2^s),  l = fp16(x 2^s - h)      (22 bits)
// and a . b = 2^-(s_a + s_b) (h_a.h_b + (h_a.l_b + l_a.h_b)), the l_a.l_b term
// (2^-22 relative) dropped.  Each fp16 product is exact in fp32 and the MFMA
// accumulates in fp32, so the error vs fp64 is that of an f32 GEMM
// (tests/test_split_gemm_gpu.py and profiles/r3_split_gemm_*: max relative
// error per sum |a_k b_k| within 1.5x of the f32 MFMA kernel's on MNIST-shape,
// Gaussian and covtype-shape data).
//
// Symmetry: the three products go to three accumulators H = sum h_a h_b,
// P = sum h_a l_b, Q = sum l_a h_b and the result is H + (P + Q).  Swapping the
// operands swaps P and Q bit for bit (the same products in the same k order)
// and leaves H unchanged, so K(i, j) computed with i as the A row equals K(j, i)
// computed with j as the A row, bit for bit.  The symmetric Gram (upper tiles
// mirrored), the sharded Gram (every rank's columns, A = all rows) and the
// working-set cache's indexed rows therefore hold identical values, as the
// f32 kernels do.
//
// Operand layout ("split rows", split_rows_f16 below): row i is dp32/32 blocks
// of 128 B, each 32 h values then the 32 l values of k = 32 b .. 32 b + 31, so
// one 128-B line per row per k-stage (a whole line per load group of 8 lanes).
//
// Tiling: 8 waves, each 32 rows x 64 columns (2 MFMA 32x32 tiles, three
// accumulators each: 96 accumulator registers).  STORE: waves 4 x 2 = 128 x 128
// block tiles; ROWS (a working set's cache misses): 2 x 4 = 64 x 256 (short row
// sets).  BK = 32 per stage (two k16 MFMA steps), LDS double buffered through
// registers; LDS rows are the 128-B row blocks with the 16-B chunk index XORed
// by (row >> 1) & 7, which makes every ds_read_b128 lane group of the operand
// reads (16 rows, one chunk) hit 16 distinct bank quads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "dpsvm/common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "split_util.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

constexpr int kSplitThreads = 512;
constexpr int kSplitShiftTarget = 15;  // largest |x| scaled into [2^14, 2^15)

// One wave per row: shift[r] and the h / l planes of row r (columns past dp
// are zero).  Lane q owns the 8-value chunks q, q + 64, ... (chunk q = columns
// 8 q .. 8 q + 7 = block q / 4, chunk q % 4 of both planes): the row is read
// once, as 16-B loads all in flight, the row max taken from the registers —
// 143 us for the headline's 60000 x 784 as a two-pass kernel with 4-B loads.
constexpr int kSplitRowChunks = 4;  // chunks per lane held in registers (dp <= 2048); longer rows loop
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ x, int64_t rows, int dp, int ldx,
                                                         u4* __restrict__ out, int32_t* __restrict__ shift,
                                                         int nkb) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * (int64_t)ldx;
  const int nq = nkb * 4;  // chunks of the padded row
  const bool vec = ((ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  auto load = [&](int q, f4& lo, f4& hi) {
    const int k0 = 8 * q;
    if (vec && k0 + 8 <= dp) {
      lo = *(const f4*)(xr + k0);
      hi = *(const f4*)(xr + k0 + 4);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo[j] = k0 + j < dp ? xr[k0 + j] : 0.f;
        hi[j] = k0 + 4 + j < dp ? xr[k0 + 4 + j] : 0.f;
      }
    }
  };
  auto emit = [&](int q, const f4& lo, const f4& hi, int s) {
    const int b = q >> 2, c = q & 3;
    h8 hv, lv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = ldexpf(j < 4 ? lo[j] : hi[j - 4], s);
      const _Float16 h = (_Float16)v;
      hv[j] = h;
      lv[j] = (_Float16)(v - (float)h);
    }
    u4* orow = out + r * (int64_t)nkb * 8;
    orow[8 * b + c] = __builtin_bit_cast(u4, hv);
    orow[8 * b + 4 + c] = __builtin_bit_cast(u4, lv);
  };
  f4 vl[kSplitRowChunks], vh[kSplitRowChunks];
  float m = 0.f;  // largest |x| of the row (the wave's max; order-free, exact)
#pragma unroll
  for (int i = 0; i < kSplitRowChunks; ++i) {
    const int q = lane + 64 * i;
    if (q < nq) {
      load(q, vl[i], vh[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) m = fmaxf(m, fmaxf(fabsf(vl[i][j]), fabsf(vh[i][j])));
    }
  }
  for (int q = lane + 64 * kSplitRowChunks; q < nq; q += 64) {  // rows past 2048 columns
    f4 lo, hi;
    load(q, lo, hi);
#pragma unroll
    for (int j = 0; j < 4; ++j) m = fmaxf(m, fmaxf(fabsf(lo[j]), fabsf(hi[j])));
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  int e = 0;
  if (m > 0.f && isfinite(m)) (void)frexpf(m, &e);  // m = f 2^e, f in [0.5, 1)
  const int s = m > 0.f && isfinite(m) ? kSplitShiftTarget - e : 0;
  if (lane == 0) shift[r] = s;
#pragma unroll
  for (int i = 0; i < kSplitRowChunks; ++i) {
    const int q = lane + 64 * i;
    if (q < nq) emit(q, vl[i], vh[i], s);
  }
  for (int q = lane + 64 * kSplitRowChunks; q < nq; q += 64) {
    f4 lo, hi;
    load(q, lo, hi);
    emit(q, lo, hi, s);
  }
}

// XCD-aware tile order (as rbf_gemm.hip): linear workgroup id L runs on XCD
// L % 8; chunks of 64 tiles (8 x 8 tile blocks) are dealt so that an XCD's
// consecutive tiles share panels in its L2.  A bijection on the tm x tn grid.
__device__ __forceinline__ void xcd_tile_of(int64_t L, int64_t tm, int64_t tn, int64_t& tx, int64_t& ty) {
  const int64_t total = tm * tn;
  constexpr int64_t CH = 64, GM = 8;
  const int64_t full = total / (8 * CH) * (8 * CH);
  int64_t T = L;
  if (L < full) {
    const int64_t xcd = L % 8, local = L / 8;
    T = ((local / CH) * 8 + xcd) * CH + local % CH;
  }
  const int64_t first_m = (T / (GM * tn)) * GM;
  const int64_t gm = min(GM, tm - first_m);
  const int64_t in = T - first_m * tn;
  tx = first_m + in % gm;
  ty = in / gm;
}

__device__ __forceinline__ void xcd_tile(int64_t& tx, int64_t& ty) {
  xcd_tile_of(blockIdx.x + (int64_t)blockIdx.y * gridDim.x, gridDim.x, gridDim.y, tx, ty);
}

enum SplitEpi { SPLIT_STORE = 0, SPLIT_ROWS = 1 };

// KB: 32-wide k blocks per LDS stage (1: 128-B LDS rows, chunk index XOR
// (row >> 1) & 7; 2: 256-B rows, XOR row & 15 — both leave every ds_read_b128
// lane group of the operand reads on 16 distinct bank quads).
// ABL (diagnostics only, DPSVM_SPLIT_ABLATE): 1 = no global stores (a runtime
// condition never true, gamma < 0, keeps the epilogue's math), 2 = no mirrored stores
// WM x WN waves (default 8 waves); a workgroup tile of 32 WM rows x 64 WN columns.
template <int EPI, int WM, int KB, int ABL = 0, int WN = 8 / WM>
__global__ __launch_bounds__(64 * WM * WN, 1) void rbf_gemm_split_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq, int64_t M,
    const u4* __restrict__ B, const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int64_t N, int nkb,
    float gamma, float* __restrict__ out, int64_t ldo, int sym, const int32_t* __restrict__ a_rows,
    const int32_t* __restrict__ out_rows, const int32_t* __restrict__ m_dev) {
  constexpr int THREADS = 64 * WM * WN, TM = 32 * WM, TN = 64 * WN, ROWS = TM + TN;
  constexpr int CPR = 8 * KB;                    // 16-B chunks per row and stage
  constexpr int CH = ROWS * CPR;                 // chunks per stage
  constexpr int NL = (CH + THREADS - 1) / THREADS;  // chunks per thread (the last one: a spare LDS slot)
  static_assert((KB == 1 || KB == 2) && THREADS >= TM, "stage geometry");
  int64_t tx, ty;
  xcd_tile(tx, ty);
  if (EPI == SPLIT_ROWS) M = *m_dev;
  if (EPI == SPLIT_STORE && sym && ty < tx) return;
  if (EPI == SPLIT_ROWS && tx * TM >= M) return;  // uniform: no barrier reached
  __shared__ u4 lds[2][CH + 1];  // + a spare slot for the staging remainder
  __shared__ float s_asq[TM];
  __shared__ int32_t s_ash[TM], s_orow[TM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int64_t m0 = tx * TM, n0 = ty * TN;
  const int64_t rstride = (int64_t)nkb * 8;  // u4 per split row
  const int nst = (nkb + KB - 1) / KB;       // stages

  if (tid < TM) {
    const int64_t row = m0 + tid;
    const int64_t ar = EPI == SPLIT_ROWS ? (int64_t)a_rows[min(row, M - 1)] : min(row, M - 1);
    s_asq[tid] = Asq[ar];
    s_ash[tid] = Ash[ar];
    s_orow[tid] = EPI == SPLIT_ROWS ? (row < M ? out_rows[row] : -1) : 0;
  }

  // staging: chunk id = tid + THREADS i -> stage row id / CPR (A rows, then B
  // rows), chunk id % CPR; ids past the stage load a valid chunk into the spare slot
  const u4* src[NL];
  int dst[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int idr = tid + THREADS * i, spare = idr >= CH, id = spare ? 0 : idr, r = id / CPR, c = id % CPR;
    int64_t grow;
    const u4* base;
    if (r < TM) {
      const int64_t row = m0 + r;  // rows past M: read a valid row (never stored)
      grow = EPI == SPLIT_ROWS ? (int64_t)a_rows[min(row, M - 1)] : row;
      base = A;
    } else {
      grow = n0 + (r - TM);
      base = B;
    }
    src[i] = base + grow * rstride + c;
    dst[i] = spare ? CH : r * CPR + (c ^ (KB == 1 ? (r >> 1) & 7 : r & 15));
  }
  // chunk i of a stage belongs to k block (i % CPR) / 8 of it: the last stage
  // of an odd block count computes its first block only, and its chunks of the
  // missing block re-read the block before (an address select, not a branch
  // around the load: hipcc would wait vmcnt(0) at every such branch)
  auto load = [&](u4* st, int kt) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int blk = ((tid + THREADS * i) % CPR) >> 3;
      const int64_t o = (int64_t)kt * CPR - ((KB > 1 && kt * KB + blk >= nkb) ? 8 : 0);
      st[i] = src[i][o];
    }
  };
  u4 st[NL];
  load(st, 0);
#pragma unroll
  for (int i = 0; i < NL; ++i) lds[0][dst[i]] = st[i];
  __syncthreads();

  f16v H[2], P[2], Q[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) H[j][r] = P[j][r] = Q[j][r] = 0.f;

  // operand rows of this lane: A row wm*32 + (lane&31), B rows TM + wn*64 + 32 j + (lane&31)
  const int sw = KB == 1 ? ((lane & 31) >> 1) & 7 : lane & 15, hl = lane >> 5;
  const int ra = (wm * 32 + (lane & 31)) * CPR;
  const int rb0 = (TM + wn * 64 + (lane & 31)) * CPR, rb1 = rb0 + 32 * CPR;
  const bool live = EPI != SPLIT_ROWS || m0 + wm * 32 < M;  // ROWS: a wave whose rows all lie past M only stages
  int cur = 0;
  for (int kt = 0; kt < nst; ++kt) {
    const bool more = kt + 1 < nst;
    if (more) load(st, kt + 1);
    if (live) {
#pragma unroll
      for (int blk = 0; blk < KB; ++blk) {
        if (KB > 1 && kt * KB + blk >= nkb) break;  // uniform
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int ch = (8 * blk + 2 * ks + hl) ^ sw, cl = (8 * blk + 4 + 2 * ks + hl) ^ sw;
          const h8 ah = __builtin_bit_cast(h8, lds[cur][ra + ch]);
          const h8 al = __builtin_bit_cast(h8, lds[cur][ra + cl]);
          const h8 bh0 = __builtin_bit_cast(h8, lds[cur][rb0 + ch]);
          const h8 bl0 = __builtin_bit_cast(h8, lds[cur][rb0 + cl]);
          const h8 bh1 = __builtin_bit_cast(h8, lds[cur][rb1 + ch]);
          const h8 bl1 = __builtin_bit_cast(h8, lds[cur][rb1 + cl]);
          H[0] = mfma32_f16(ah, bh0, H[0]);
          H[1] = mfma32_f16(ah, bh1, H[1]);
          P[0] = mfma32_f16(ah, bl0, P[0]);
          P[1] = mfma32_f16(ah, bl1, P[1]);
          Q[0] = mfma32_f16(al, bh0, Q[0]);
          Q[1] = mfma32_f16(al, bh1, Q[1]);
        }
      }
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < NL; ++i) lds[cur ^ 1][dst[i]] = st[i];
    }
    __syncthreads();
    cur ^= 1;
  }
  if (!live) return;

  // ---- epilogue: K = exp(-g max(|a|^2 + |b|^2 - 2 dot, 0)), dot = 2^-(sa+sb) (H + (P + Q)) ----
  // (all values first, into H; then the stores: unpredicated for interior tiles)
  float asq_r[16];
  int ash_r[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
    asq_r[r] = s_asq[lr];
    ash_r[r] = s_ash[lr];
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
    const int64_t cc = col < N ? col : N - 1;
    const float bsq = Bsq[cc];
    const int bsh = Bsh[cc];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float dot = ldexpf(H[j][r] + (P[j][r] + Q[j][r]), -(ash_r[r] + bsh));
      H[j][r] = rbf_split_value(asq_r[r], bsq, dot, gamma);
    }
  }
  const bool interior = m0 + TM <= M && n0 + TN <= N;
  if (EPI == SPLIT_ROWS) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int32_t orow = s_orow[wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
        if (orow >= 0 && (interior || col < N)) out[(int64_t)orow * ldo + col] = H[j][r];
      }
    }
    return;
  }
  if (ABL != 1 || gamma < 0.f) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
        if (interior || (row < M && col < N)) out[row * ldo + col] = H[j][r];
      }
    }
  }
  if (EPI == SPLIT_STORE && sym && ty != tx && ABL == 0) {
    // transposed tile: a lane holds 4 consecutive rows per group -> 16-B stores out[col][row .. row+3]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = m0 + wm * 32 + 8 * q + 4 * hl;
        float* dst = out + col * ldo + row;
        f4 v;
        v.x = H[j][4 * q + 0];
        v.y = H[j][4 * q + 1];
        v.z = H[j][4 * q + 2];
        v.w = H[j][4 * q + 3];
        if (interior) {
          *(f4*)dst = v;
        } else if (col < M) {
          if (row + 3 < N) {
            *(f4*)dst = v;
          } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (row + c < N) dst[c] = v[c];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// LDS-DMA STORE GEMM: the tile kernel's MFMA sequence (128 x 128 tile, 8 waves
// of 32 x 64, k blocks in order: bit-identical Gram) with the operands staged
// by global_load_lds_dwordx4 into FOUR 32-k buffers, three blocks in flight
// ahead of the one being multiplied.  Per k block: a counted vmcnt retires the
// block's own DMA (never vmcnt(0) inside the loop), one raw s_barrier (the DMA
// has landed everywhere, and every wave is done with the buffer the next DMA
// overwrites), the DMA of block kb + 3, then 2 k16 steps of 6 MFMAs.  The
// register-staged kernels above wait for each stage's loads before the next
// stage can start (one stage of prefetch: a 0.3-0.6 us stage against a 1-2 us
// L2-miss latency).  An LDS-DMA wave instruction writes 1 KiB lane-linearly (8
// rows x 128 B): the bank swizzle of the operand reads (chunk c of row r at
// position c ^ ((r >> 1) & 7)) moves to the per-lane SOURCE address.  All LDS
// in one array (row data after the buffers): a second __shared__ object makes
// hipcc wait vmcnt(0) before the operand reads.
// ---------------------------------------------------------------------------
constexpr int kGldsThreads = 512;
__global__ __launch_bounds__(kGldsThreads, 1) void rbf_gemm_split_glds_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq, int64_t M,
    const u4* __restrict__ B, const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int64_t N, int nkb,
    float gamma, float* __restrict__ out, int64_t ldo, int sym) {
  constexpr int WN = 2, TM = 128, TN = 128, ROWS = TM + TN, CPR = 8, BUF = ROWS * CPR, NB = 4;
  int64_t tx, ty;
  xcd_tile(tx, ty);
  if (sym && ty < tx) return;
  __shared__ u4 lds[NB * BUF + 2 * ROWS / 4];  // 4 operand buffers, then |x|^2 [ROWS] and shifts [ROWS]
  float* s_sq = (float*)(lds + NB * BUF);
  int32_t* s_sh = (int32_t*)(lds + NB * BUF) + ROWS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const int64_t m0 = tx * TM, n0 = ty * TN;
  const int64_t rstride = (int64_t)nkb * 8;  // u4 per split row

  if (tid < ROWS) {
    const int64_t ri = tid < TM ? min(m0 + tid, M - 1) : min(n0 + (tid - TM), N - 1);
    s_sq[tid] = tid < TM ? Asq[ri] : Bsq[ri];
    s_sh[tid] = tid < TM ? Ash[ri] : Bsh[ri];
  }
  // DMA sources: wave w fills rows 32 w + 8 i + (lane >> 3), i = 0..3 (waves 0-3: A rows,
  // 4-7: B rows); lane position p = lane & 7 takes global chunk p ^ ((row >> 1) & 7)
  const u4* src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 32 * wave + 8 * i + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    src[i] = r < TM ? A + (m0 + r) * rstride + c : B + (n0 + (r - TM)) * rstride + c;
  }
  auto dma = [&](int kb) {
    u4* dst = lds + (kb & (NB - 1)) * BUF + 32 * wave * CPR;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + (int64_t)kb * 8),
                                       (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, 0);
  };
  __syncthreads();  // row data written (no DMA in flight yet)
  dma(0);
  if (nkb > 1) dma(1);
  if (nkb > 2) dma(2);

  f16v H[2], P[2], Q[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) H[j][r] = P[j][r] = Q[j][r] = 0.f;
  const int sw = ((lane & 31) >> 1) & 7;
  const int ra = (wm * 32 + (lane & 31)) * CPR;
  const int rb0 = (TM + wn * 64 + (lane & 31)) * CPR, rb1 = rb0 + 32 * CPR;
  for (int kb = 0; kb < nkb; ++kb) {
    // retire block kb's DMA: the blocks after it (up to 2) may stay in flight
    const int ahead = min(2, nkb - 1 - kb);
    if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kb + 3 < nkb) dma(kb + 3);  // into the buffer of block kb - 1 (every wave is past it)
    const u4* buf = lds + (kb & (NB - 1)) * BUF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = (2 * ks + hl) ^ sw, cl = (4 + 2 * ks + hl) ^ sw;
      const h8 ah = __builtin_bit_cast(h8, buf[ra + ch]);
      const h8 al = __builtin_bit_cast(h8, buf[ra + cl]);
      const h8 bh0 = __builtin_bit_cast(h8, buf[rb0 + ch]);
      const h8 bl0 = __builtin_bit_cast(h8, buf[rb0 + cl]);
      const h8 bh1 = __builtin_bit_cast(h8, buf[rb1 + ch]);
      const h8 bl1 = __builtin_bit_cast(h8, buf[rb1 + cl]);
      H[0] = mfma32_f16(ah, bh0, H[0]);
      H[1] = mfma32_f16(ah, bh1, H[1]);
      P[0] = mfma32_f16(ah, bl0, P[0]);
      P[1] = mfma32_f16(ah, bl1, P[1]);
      Q[0] = mfma32_f16(al, bh0, Q[0]);
      Q[1] = mfma32_f16(al, bh1, Q[1]);
    }
  }

  // ---- epilogue (as the tile kernel) ----
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cb = TM + wn * 64 + 32 * j + (lane & 31);
    const float bsq = s_sq[cb];
    const int bsh = s_sh[cb];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
      const float dot = ldexpf(H[j][r] + (P[j][r] + Q[j][r]), -(s_sh[lr] + bsh));
      H[j][r] = rbf_split_value(s_sq[lr], bsq, dot, gamma);
    }
  }
  const bool interior = m0 + TM <= M && n0 + TN <= N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
      if (interior || (row < M && col < N)) out[row * ldo + col] = H[j][r];
    }
  }
  if (sym && ty != tx) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = m0 + wm * 32 + 8 * q + 4 * hl;
        float* dst = out + col * ldo + row;
        f4 v;
        v.x = H[j][4 * q + 0];
        v.y = H[j][4 * q + 1];
        v.z = H[j][4 * q + 2];
        v.w = H[j][4 * q + 3];
        if (interior) {
          *(f4*)dst = v;
        } else if (col < M) {
          if (row + 3 < N) {
            *(f4*)dst = v;
          } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (row + c < N) dst[c] = v[c];
          }
        }
      }
    }
  }
}

// the 32-bit LDS byte address of a __shared__ pointer (asm ds_read operands)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// ---------------------------------------------------------------------------
// LDS-DMA ROWS GEMM: a working-set round's cache misses (up to 192 indexed A
// rows, a_rows[0 .. *m_dev)) against all of this rank's B rows, K written to
// the misses' cache lines.  The register-staged ROWS kernel above waits for
// each 32-k stage's loads before the next can start, so on synthetic-2m
// (K = 1024, 2M B rows: the 8 GB split X panel per round) it ran at 2.3 TB/s of
// B bytes and 3.5 ms per round (profiles/r4_big_inputs).  Here the operands of
// a 192 x 128 tile go through three 32-k LDS buffers by global_load_lds_dwordx4
// (40 KiB each; the row data after them in the same array), the next block's
// DMA in flight while a block is multiplied; the waves are the ROWS kernel's
// (6 x 2, 32 x 64 each) with its MFMA sequence and epilogue, so the rows are
// bit-identical to it (and to the Gram kernels').  Ten waves issue the DMA: 40
// wave instructions of 8 rows x 128 B per block, 4 per wave.
// ---------------------------------------------------------------------------
constexpr int kRowsGldsThreads = 768;
// BAUX: cache policy of the B operand's DMA (2 = nt: streamed once per round,
// kept from evicting the A rows every tile re-reads from L2)
// NBR: B ring depth.  A and B have separate rings: A three deep (block kb + 2
// issued at block kb), B NBR deep (block kb + NBR - 1 issued at kb); the waves
// that stage A (0-5) and B (6-9) wait on their own DMA counts.  Measured at the
// synthetic-2m round shape (bench/rows_probe.py, profiles/r6_rows_kernel.txt):
// NBR 5 does not beat 3, B read from L2 instead of HBM saves only ~10%, and
// the operand reads one MFMA group ahead (the Gram's SP 2) change nothing —
// the k loop runs at ~46% MFMA with the chip at ~1.57 GHz.
// ST: diagnostics build with per-workgroup stamps (entry, first block landed,
// k loop done, stores issued, stores done; s_memrealtime at entry / end) at
// stamps[8 (blockIdx.y gridDim.x + blockIdx.x) ..] (bench/rows_probe.py --stamps)
template <int BAUX, int NBR = 3, bool ST = false>
__global__ __launch_bounds__(kRowsGldsThreads, 1) void rbf_rows_split_glds_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq,
    const int32_t* __restrict__ a_rows, const int32_t* __restrict__ m_dev, const u4* __restrict__ B,
    const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int64_t N, int nkb, float gamma,
    float* __restrict__ out, int64_t ldo, const int32_t* __restrict__ out_rows, uint64_t* __restrict__ stamps) {
  uint64_t st[5] = {0, 0, 0, 0, 0}, rt0 = 0;
  if constexpr (ST) {
    st[0] = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  constexpr int WN = 2, TM = 192, TN = 128, CPR = 8, NA = 3;
  constexpr int BUFA = TM * CPR, BUFB = TN * CPR;
  constexpr int DMA_WAVES = (TM + TN) / 32;  // 10: each fills 32 rows (4 instructions of 8 rows)
  static_assert(NA * BUFA * 16 + NBR * BUFB * 16 + (3 * TM + 2 * TN) * 4 <= 160 * 1024, "LDS");
  int64_t tx, ty;
  xcd_tile(tx, ty);
  const int M = *m_dev;
  if (tx * TM >= M) return;  // uniform: no barrier reached
  __shared__ u4 lds[NA * BUFA + NBR * BUFB + (3 * TM + 2 * TN) / 4];
  u4* const ldsA = lds;
  u4* const ldsB = lds + NA * BUFA;
  float* s_asq = (float*)(lds + NA * BUFA + NBR * BUFB);
  int32_t* s_ash = (int32_t*)(s_asq + TM);
  int32_t* s_orow = s_ash + TM;
  float* s_bsq = (float*)(s_orow + TM);
  int32_t* s_bsh = (int32_t*)(s_bsq + TN);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const int64_t m0 = tx * TM, n0 = ty * TN;
  const int64_t rstride = (int64_t)nkb * 8;  // u4 per split row
  if (tid < TM) {
    const int64_t row = m0 + tid;
    const int64_t ar = a_rows[min(row, (int64_t)M - 1)];
    s_asq[tid] = Asq[ar];
    s_ash[tid] = Ash[ar];
    s_orow[tid] = row < M ? out_rows[row] : -1;
  } else if (tid < TM + TN) {
    const int64_t cc = min(n0 + (tid - TM), N - 1);
    s_bsq[tid - TM] = Bsq[cc];
    s_bsh[tid - TM] = Bsh[cc];
  }
  // DMA sources: wave w < 10 fills stage rows 32 w + 8 i + (lane >> 3) (rows
  // >= TM: B row r - TM of its own ring); lane position p = lane & 7 takes
  // global chunk p ^ ((row >> 1) & 7) (the read swizzle; TM is a multiple of
  // 16, so B rows keep it re-based at 0); A rows past M re-read a valid row
  // (never stored)
  const u4* src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = min(32 * wave + 8 * i + (lane >> 3), TM + TN - 1);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int64_t grow = r < TM ? (int64_t)a_rows[min(m0 + r, (int64_t)M - 1)] : n0 + (r - TM);
    src[i] = (r < TM ? A : B) + grow * rstride + c;
  }
  const bool dma_wave = wave < DMA_WAVES;
  const bool b_wave = 32 * wave >= TM;  // waves 6 .. 9 stage B rows only (TM = 192 = 6 x 32)
  auto dma = [&](int kb) {
    if (b_wave) {
      u4* dst = ldsB + (kb % NBR) * BUFB + (32 * wave - TM) * CPR;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(src[i] + (int64_t)kb * 8),
                                         (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, BAUX);
    } else {
      u4* dst = ldsA + (kb % NA) * BUFA + 32 * wave * CPR;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(src[i] + (int64_t)kb * 8),
                                         (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, 0);
    }
  };
  const int ahead = b_wave ? NBR - 1 : NA - 1;  // blocks a staging wave keeps issued past the current one
  __syncthreads();  // row data written (no DMA in flight yet)
  if (dma_wave) {
    for (int b = 0; b < ahead && b < nkb; ++b) dma(b);
  }

  f16v H[2], P[2], Q[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) H[j][r] = P[j][r] = Q[j][r] = 0.f;
  const int sw = ((lane & 31) >> 1) & 7;
  const int ra = (wm * 32 + (lane & 31)) * CPR;
  const int rb0 = (wn * 64 + (lane & 31)) * CPR, rb1 = rb0 + 32 * CPR;
  const bool live = m0 + wm * 32 < M;  // a wave whose rows all lie past M only stages
  for (int kb = 0; kb < nkb; ++kb) {
    // retire block kb's DMA: a staging wave's younger blocks kb + 1 .. (4
    // pieces each) may stay in flight (uniform per wave)
    const int younger = min(ahead - 1, nkb - 1 - kb);
    if (younger >= 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (ST) {
      if (kb == 0) st[1] = __builtin_amdgcn_s_memtime();
    }
    // block kb + ahead into its ring's buffer of block kb - 1 (every wave is past it)
    if (dma_wave && kb + ahead < nkb) dma(kb + ahead);
    if (live) {
      const u4* bufa = ldsA + (kb % NA) * BUFA;
      const u4* bufb = ldsB + (kb % NBR) * BUFB;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = (2 * ks + hl) ^ sw, cl = (4 + 2 * ks + hl) ^ sw;
        const h8 ah = __builtin_bit_cast(h8, bufa[ra + ch]);
        const h8 al = __builtin_bit_cast(h8, bufa[ra + cl]);
        const h8 bh0 = __builtin_bit_cast(h8, bufb[rb0 + ch]);
        const h8 bl0 = __builtin_bit_cast(h8, bufb[rb0 + cl]);
        const h8 bh1 = __builtin_bit_cast(h8, bufb[rb1 + ch]);
        const h8 bl1 = __builtin_bit_cast(h8, bufb[rb1 + cl]);
        H[0] = mfma32_f16(ah, bh0, H[0]);
        H[1] = mfma32_f16(ah, bh1, H[1]);
        P[0] = mfma32_f16(ah, bl0, P[0]);
        P[1] = mfma32_f16(ah, bl1, P[1]);
        Q[0] = mfma32_f16(al, bh0, Q[0]);
        Q[1] = mfma32_f16(al, bh1, Q[1]);
      }
    }
  }
  if (!live) return;
  if constexpr (ST) st[2] = __builtin_amdgcn_s_memtime();

  // ---- epilogue (the ROWS kernel's): K = exp(-g max(|a|^2 + |b|^2 - 2 dot, 0)) ----
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cb = wn * 64 + 32 * j + (lane & 31);
    const float bsq = s_bsq[cb];
    const int bsh = s_bsh[cb];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
      const float dot = ldexpf(H[j][r] + (P[j][r] + Q[j][r]), -(s_ash[lr] + bsh));
      H[j][r] = rbf_split_value(s_asq[lr], bsq, dot, gamma);
    }
  }
  const bool interior = n0 + TN <= N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int32_t orow = s_orow[wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
      if (orow >= 0 && (interior || col < N)) out[(int64_t)orow * ldo + col] = H[j][r];
    }
  }
  if constexpr (ST) {
    st[3] = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st[4] = __builtin_amdgcn_s_memtime();
    const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      uint64_t* o = stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;
#pragma unroll
      for (int i = 0; i < 5; ++i) o[i] = st[i];
      o[5] = rt0;
      o[6] = rt1;
      o[7] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// Persistent LDS-DMA ROWS GEMM (the default for one tile row, M <= 192, and
// nkb >= 3: a one-block ws-cache round's misses against all of this rank's B
// rows — synthetic-2m's round).  The tile-per-workgroup kernel above spends
// ~8% of a tile in its prologue (the miss rows' data and DMA sources, the
// first blocks' latency) and the device runs ~239 of 256 workgroups at a time
// (stamps, profiles/r6_rows_kernel.txt).  Here one workgroup per CU walks
// column tiles ty = b, b + G, ...: the A side (the misses' |x|^2, shifts,
// output lines and DMA sources) is set up once, and the DMA rings run on
// across tiles — during a tile's last two k blocks the prefetch slots load
// blocks 0 and 1 of the next (A's are the same blocks, B's the next tile's
// rows), the next tile's B row data is loaded into registers during the k
// loop and stored into the other parity of a row-data area after it.  Every
// DMA wave issues 4 pieces every k block (the last tile re-loads its own
// blocks 0 / 1 into dead buffers), so one uniform vmcnt(4) retires a block;
// each epilogue ends with vmcnt(0).  Same MFMA sequence and epilogue per tile:
// bit-identical to the kernel above.
// ---------------------------------------------------------------------------
template <int BAUX>
__global__ __launch_bounds__(kRowsGldsThreads, 1) void rbf_rows_split_glds_persist_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq,
    const int32_t* __restrict__ a_rows, const int32_t* __restrict__ m_dev, const u4* __restrict__ B,
    const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int64_t N, int nkb, float gamma,
    float* __restrict__ out, int64_t ldo, const int32_t* __restrict__ out_rows, int ntiles) {
  constexpr int WN = 2, TM = 192, TN = 128, CPR = 8, NBUF = 3;
  constexpr int BUFA = TM * CPR, BUFB = TN * CPR;
  constexpr int DMA_WAVES = (TM + TN) / 32;  // 10: waves 0-5 stage A rows, 6-9 B rows (4 pieces of 8 rows each)
  __shared__ u4 lds[NBUF * BUFA + NBUF * BUFB + (3 * TM + 4 * TN) / 4];
  u4* const ldsA = lds;
  u4* const ldsB = lds + NBUF * BUFA;
  float* const s_asq = (float*)(lds + NBUF * (BUFA + BUFB));
  int32_t* const s_ash = (int32_t*)(s_asq + TM);
  int32_t* const s_orow = s_ash + TM;
  float* const s_bsq = (float*)(s_orow + TM);    // [2][TN] by parity
  int32_t* const s_bsh = (int32_t*)(s_bsq + 2 * TN);  // [2][TN]
  const int M = *m_dev;
  const int G = gridDim.x;
  int ty = blockIdx.x;
  if (ty >= ntiles || M <= 0) return;  // uniform
  // (the wave index in an SGPR: the epilogue's row addresses stay scalar
  // instead of 16 VGPRs hoisted across the tile loop)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const int64_t rstride = (int64_t)nkb * 8;  // u4 per split row
  if (tid < TM) {
    const int64_t ar = a_rows[min(tid, M - 1)];
    s_asq[tid] = Asq[ar];
    s_ash[tid] = Ash[ar];
    s_orow[tid] = tid < M ? out_rows[tid] : -1;
  } else if (tid < TM + TN) {
    const int64_t cc = min((int64_t)ty * TN + (tid - TM), N - 1);
    s_bsq[tid - TM] = Bsq[cc];
    s_bsh[tid - TM] = Bsh[cc];
  }
  // DMA sources: the kernel above's geometry; A's fixed for the launch, B's as
  // a per-lane offset from the tile's first row (a uniform base per tile)
  const bool dma_wave = wave < DMA_WAVES;
  const bool b_wave = 32 * wave >= TM;
  // (32-bit u4 offsets: launcher, (N + 512) x nkb x 8 < 2^32; registers are
  // what the 96 accumulators leave at three waves per SIMD)
  uint32_t off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = min(32 * wave + 8 * i + (lane >> 3), TM + TN - 1);
    const uint32_t c = (uint32_t)((lane & 7) ^ ((r >> 1) & 7));
    off[i] = r < TM ? (uint32_t)a_rows[min(r, M - 1)] * (uint32_t)rstride + c : (uint32_t)(r - TM) * (uint32_t)rstride + c;
  }
  // piece set of global block g (kb of tile tt): into ring buffer g % 3
  auto dma = [&](uint32_t g, int kb, int tt) {
    const u4* base = b_wave ? B + (int64_t)tt * TN * rstride + (int64_t)kb * 8 : A + (int64_t)kb * 8;  // uniform
    u4* dst = b_wave ? ldsB + (g % NBUF) * BUFB + (32 * wave - TM) * CPR : ldsA + (g % NBUF) * BUFA + 32 * wave * CPR;
    if (b_wave) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(base + off[i]),
                                         (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, BAUX);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(base + off[i]),
                                         (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, 0);
    }
  };
  __syncthreads();  // row data written (no DMA in flight yet)
  uint32_t g = 0;   // k blocks started over all of this workgroup's tiles
  if (dma_wave) {
    dma(0, 0, ty);
    dma(1, 1, ty);  // (launcher: nkb >= 3)
  }
  const int sw = ((lane & 31) >> 1) & 7;
  const int ra = (wm * 32 + (lane & 31)) * CPR;
  const int rb0 = (wn * 64 + (lane & 31)) * CPR, rb1 = rb0 + 32 * CPR;
  const bool live = wm * 32 < M;  // a wave whose rows all lie past M only stages
  int par = 0;
  while (true) {
    const int tn_next = ty + G;
    const bool has_next = tn_next < ntiles;  // uniform
    const int tp = has_next ? tn_next : ty;  // the last tile prefetches itself into dead buffers
    // the next tile's B row data, in flight across the k loop
    float nbsq = 0.f;
    int32_t nbsh = 0;
    if (has_next && tid >= TM && tid < TM + TN) {
      const int64_t cc = min((int64_t)tn_next * TN + (tid - TM), N - 1);
      nbsq = Bsq[cc];
      nbsh = Bsh[cc];
    }
    f16v H[2], P[2], Q[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) H[j][r] = P[j][r] = Q[j][r] = 0.f;
    for (int kb = 0; kb < nkb; ++kb) {
      // block kb landed: only block kb + 1's 4 pieces may stay in flight
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // block kb + 2 of this tile, or block kb + 2 - nkb of the next, into the
      // buffer of block g - 1 (every wave is past it)
      if (dma_wave) {
        const bool own = kb + 2 < nkb;
        dma(g + 2, own ? kb + 2 : kb + 2 - nkb, own ? ty : tp);
      }
      if (live) {
        const u4* bufa = ldsA + (g % NBUF) * BUFA;
        const u4* bufb = ldsB + (g % NBUF) * BUFB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int ch = (2 * ks + hl) ^ sw, cl = (4 + 2 * ks + hl) ^ sw;
          const h8 ah = __builtin_bit_cast(h8, bufa[ra + ch]);
          const h8 al = __builtin_bit_cast(h8, bufa[ra + cl]);
          const h8 bh0 = __builtin_bit_cast(h8, bufb[rb0 + ch]);
          const h8 bl0 = __builtin_bit_cast(h8, bufb[rb0 + cl]);
          const h8 bh1 = __builtin_bit_cast(h8, bufb[rb1 + ch]);
          const h8 bl1 = __builtin_bit_cast(h8, bufb[rb1 + cl]);
          H[0] = mfma32_f16(ah, bh0, H[0]);
          H[1] = mfma32_f16(ah, bh1, H[1]);
          P[0] = mfma32_f16(ah, bl0, P[0]);
          P[1] = mfma32_f16(ah, bl1, P[1]);
          Q[0] = mfma32_f16(al, bh0, Q[0]);
          Q[1] = mfma32_f16(al, bh1, Q[1]);
        }
      }
      ++g;
    }
    // the next tile's B row data into the other parity (last read by the
    // previous tile's epilogue, before this tile's first barrier)
    if (has_next && tid >= TM && tid < TM + TN) {
      s_bsq[(par ^ 1) * TN + (tid - TM)] = nbsq;
      s_bsh[(par ^ 1) * TN + (tid - TM)] = nbsh;
    }
    if (live) {
      // ---- epilogue (the kernel above's) ----
      // (per-lane addresses from a laundered lane id: hoisted out of the tile
      // loop they would hold registers across the k loop and spill)
      int el = lane;
      asm volatile("" : "+v"(el));
      const int ehl = el >> 5;
      const int64_t n0 = (int64_t)ty * TN;
      const float* bq = s_bsq + par * TN;
      const int32_t* bs = s_bsh + par * TN;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cb = wn * 64 + 32 * j + (el & 31);
        const float bsq = bq[cb];
        const int bsh = bs[cb];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * ehl;
          const float dot = ldexpf(H[j][r] + (P[j][r] + Q[j][r]), -(s_ash[lr] + bsh));
          H[j][r] = rbf_split_value(s_asq[lr], bsq, dot, gamma);
        }
      }
      const bool interior = n0 + TN <= N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int32_t orow = s_orow[wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * ehl];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t col = n0 + wn * 64 + 32 * j + (el & 31);
          if (orow >= 0 && (interior || col < N)) out[(int64_t)orow * ldo + col] = H[j][r];
        }
      }
    }
    // the stores and the next tile's blocks 0 / 1 retired: the loop's uniform
    // vmcnt(4) holds at the next tile's first block (and no DMA is in flight
    // when the kernel ends)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!has_next) break;
    ty = tn_next;
    par ^= 1;
  }
}

// ---------------------------------------------------------------------------
// Persistent small-K ROWS GEMM (nkb <= 2 k blocks: d <= 64, covtype's 54
// features).  There a tile is two k blocks of MFMA work against 24-98 KiB of
// operand and store traffic, so a tile-per-workgroup grid is a chain of
// latencies (load, multiply, store) per tile.  Here one 768-thread workgroup
// per CU walks the tiles of its grid stride (64 x 192 up to 192 x 64 by the
// miss count): the A rows of its tile row (<= 48 KiB) are staged into LDS
// once, the B column tiles (and their |x|^2 / shifts) stream through two LDS buffers by LDS-DMA, the next
// tile's DMA issued before this tile's multiply, so its latency hides under
// the multiply, the epilogue and the stores; a wave then waits with vmcnt(16)
// (its 16 stores of the tile before are younger than that DMA), so the stores
// drain under the next tile instead of being waited for (every live lane
// stores exactly 16 values: rows past M and columns past N go to a scratch
// line).  MFMA sequence and epilogue as the ROWS kernels: bit-identical rows.
// ---------------------------------------------------------------------------
constexpr int kRowsPersistThreads = 768;
template <int NKB>
__global__ __launch_bounds__(kRowsPersistThreads, 1) void rbf_rows_split_persist_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq,
    const int32_t* __restrict__ a_rows, const int32_t* __restrict__ m_dev, const u4* __restrict__ B,
    const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int64_t N, float gamma,
    float* __restrict__ out, int64_t ldo, const int32_t* __restrict__ out_rows, float* __restrict__ trash) {
  // 12 waves of 32 x 32 (one MFMA tile, three accumulators each), laid out by
  // the round's miss count M: WM x WN = 2 x 6 (64 x 192 tiles) up to 64
  // misses, 4 x 3 (128 x 96) up to 128, else 6 x 2 (192 x 64) — the fewest,
  // widest tiles that cover the live rows (a tile's cost is mostly latency)
  constexpr int CPR = 8, TMX = 192, TNX = 192;
  constexpr int ABUF = TMX * NKB * CPR, BBUF = TNX * NKB * CPR;  // u4
  const int M = *m_dev;
  const int WM = M <= 64 ? 2 : M <= 128 ? 4 : 6, WN = 12 / WM, TM = 32 * WM, TN = 32 * WN;
  const int tn = (int)((N + TN - 1) / TN), tm = (M + TM - 1) / TM, total = tm * tn;
  int L = blockIdx.x;
  if (L >= total) return;  // uniform
  __shared__ u4 lds[ABUF + 2 * BBUF + (2 * 2 * TNX) / 4 + (3 * TMX) / 4];
  u4* s_a = lds;                                          // [NKB][TM rows][CPR]
  u4* s_b = lds + ABUF;                                   // [2][NKB][TN rows][CPR]
  float* s_bsq = (float*)(lds + ABUF + 2 * BBUF);         // [2][TNX], then s_bsh [2][TNX]
  int32_t* s_bsh = (int32_t*)(s_bsq + 2 * TNX);
  float* s_asq = (float*)(s_bsh + 2 * TNX);
  int32_t* s_ash = (int32_t*)(s_asq + TMX);
  int32_t* s_orow = s_ash + TMX;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  constexpr int64_t rstride = (int64_t)NKB * 8;
  const int nb = TN * NKB / 8, nv = (TN + 63) / 64;  // B-row DMA instructions; |x|^2 (and shift) ones per tile
  // B DMA of column tile ty into buffer b: instruction i (8 k-rows x 128 B) by
  // wave i % 12, then the |x|^2 / shift dwords by the waves after
  auto dma = [&](int ty, int b) {
    const int64_t n0 = (int64_t)ty * TN;
    for (int i = wave; i < nb + 2 * nv; i += 12) {
      if (i < nb) {
        const int q = 8 * i + (lane >> 3), kb = q / TN, r = q % TN;
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        __builtin_amdgcn_global_load_lds((const void*)(B + (n0 + r) * rstride + kb * 8 + c),
                                         (__attribute__((address_space(3))) void*)(s_b + b * BBUF + 8 * i * CPR),
                                         16, 0, 0);
      } else {
        const int v = i - nb, part = v % nv;
        const int64_t cc = min(n0 + 64 * part + lane, N - 1);
        if (v < nv)
          __builtin_amdgcn_global_load_lds((const void*)(Bsq + cc),
                                           (__attribute__((address_space(3))) void*)(s_bsq + b * TNX + 64 * part), 4,
                                           0, 0);
        else
          __builtin_amdgcn_global_load_lds((const void*)(Bsh + cc),
                                           (__attribute__((address_space(3))) void*)(s_bsh + b * TNX + 64 * part), 4,
                                           0, 0);
      }
    }
  };
  dma(L % tn, 0);
  int ltx = -1, buf = 0;
  bool stored = false;  // this wave's 16 stores of the previous tile are younger than the pending DMA
  const int sw = ((lane & 31) >> 1) & 7;
  for (; L < total; L += gridDim.x) {
    const int tx = L / tn, ty = L % tn;
    const int64_t m0 = (int64_t)tx * TM, n0 = (int64_t)ty * TN;
    if (tx != ltx) {
      // the A rows of this tile row (plain loads: the first tile, or a new tile
      // row of a multi-block round's misses); every wave is past the old rows
      __syncthreads();
      for (int id = tid; id < TM * NKB * CPR; id += kRowsPersistThreads) {
        const int kb = id / (TM * CPR), r = (id / CPR) % TM, c = id % CPR;
        const int64_t ar = a_rows[min(m0 + r, (int64_t)M - 1)];
        s_a[(kb * TM + r) * CPR + (c ^ ((r >> 1) & 7))] = A[ar * rstride + kb * 8 + c];
      }
      if (tid < TM) {
        const int64_t row = m0 + tid;
        const int64_t ar = a_rows[min(row, (int64_t)M - 1)];
        s_asq[tid] = Asq[ar];
        s_ash[tid] = Ash[ar];
        s_orow[tid] = row < M ? out_rows[row] : -1;
      }
      ltx = tx;
      stored = false;  // those loads were waited for: nothing older is outstanding
    }
    const bool live = m0 + wm * 32 < M;
    // this tile's DMA has landed; the previous tile's stores may still drain
    if (stored) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (L + (int)gridDim.x < total) dma((L + gridDim.x) % tn, buf ^ 1);  // every wave is past buffer buf ^ 1
    if (live) {
      f16v H, P, Q;
#pragma unroll
      for (int r = 0; r < 16; ++r) H[r] = P[r] = Q[r] = 0.f;
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        const int ra = ((kb * TM) + wm * 32 + (lane & 31)) * CPR;
        const int rb = (buf * BBUF) + (kb * TN + wn * 32 + (lane & 31)) * CPR;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int ch = (2 * ks + hl) ^ sw, cl = (4 + 2 * ks + hl) ^ sw;
          const h8 ah = __builtin_bit_cast(h8, s_a[ra + ch]);
          const h8 al = __builtin_bit_cast(h8, s_a[ra + cl]);
          const h8 bh = __builtin_bit_cast(h8, s_b[rb + ch]);
          const h8 bl = __builtin_bit_cast(h8, s_b[rb + cl]);
          H = mfma32_f16(ah, bh, H);
          P = mfma32_f16(ah, bl, P);
          Q = mfma32_f16(al, bh, Q);
        }
      }
      const int cb = wn * 32 + (lane & 31);
      const float bsq = s_bsq[buf * TNX + cb];
      const int bsh = s_bsh[buf * TNX + cb];
      const int64_t col = n0 + cb;
      const bool ok = col < N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const float dot = ldexpf(H[r] + (P[r] + Q[r]), -(s_ash[lr] + bsh));
        const float v = rbf_split_value(s_asq[lr], bsq, dot, gamma);
        const int32_t orow = s_orow[lr];
        // exactly 16 stores per lane (the vmcnt(16) above): rows past M and
        // columns past N go to the scratch line
        float* dst = (orow >= 0 && ok) ? out + (int64_t)orow * ldo + col : trash + lane;
        *dst = v;
      }
    }
    stored = live;
    buf ^= 1;
  }
}

// The w64 kernels' epilogue (PE, the default): the values two at a time in
// packed f32 (v_pk_add / v_pk_mul; the same IEEE operations per value, so the
// same bits as rbf_split_value), stores through buffer descriptors: a lane
// outside the tile's columns gets an out-of-range offset and rows past M fall
// beyond the descriptor's size, so the hardware drops them — one address add
// per store and no exec-mask branch.  The scalar epilogue was ~20 VALU and ~13
// SALU per value, VALU-issue-bound: 13.4k -> 10.0k cycles a tile
// (profiles/r6_gram_lds_readahead_ab.json).  Host: the last row tile's
// (M - m0) x ldo floats < 2^31 bytes.  lane: the caller's (laundered) lane id.
// AD: the adaptive Gram's hot-tile pass — every element takes the one-product
// value where split_cold allows it (R = log2 |x| from Ar / Br, global loads:
// this pass runs only the few tiles the one-product pass reported).
typedef int i4v_t __attribute__((ext_vector_type(4)));
template <bool AD = false>
__device__ __forceinline__ void w64_epilogue_pe(f16v (&H)[2][2], const f16v (&P)[2][2], const f16v (&Q)[2][2],
                                                const float* s_sq, const int32_t* s_sh, int lane, int wm, int wn,
                                                bool mirror, float* out, int64_t m0, int64_t n0, int64_t M, int64_t N,
                                                int64_t ldo, float gamma, const float* Ar = nullptr,
                                                const float* Br = nullptr, float c0 = 0.f, float c1 = 0.f) {
  constexpr int TM = 256, TN = 128;
  typedef i4v_t i4v;
  const int hl = lane >> 5;
  float* const ob = out + m0 * ldo + n0;  // direct block
  float* const mb = out + n0 * ldo + m0;  // mirrored block (symmetric: M == N)
  const uint32_t ld = (uint32_t)ldo;
  const int rlim = (int)min<int64_t>(M - m0, TM);  // tile rows inside [0, M)
  const int clim = (int)min<int64_t>(N - n0, TN);  // tile columns inside [0, N)
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr uint32_t OOB = 0x80000000u;
  const int64_t ob_bytes = min<int64_t>((M - m0) * ldo * 4 - n0 * 4, (int64_t)OOB);
  const int64_t mb_bytes = min<int64_t>((N - n0) * ldo * 4 - m0 * 4, (int64_t)OOB);
  const __amdgpu_buffer_rsrc_t rs_o = __builtin_amdgcn_make_buffer_rsrc(ob, 0, (int)ob_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_m = __builtin_amdgcn_make_buffer_rsrc(mb, 0, (int)mb_bytes, 0x00020000);
  const float ng = -gamma, l2e = 1.4426950408889634f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = wn * 64 + 32 * j + (lane & 31);
    const bool okc = cl < clim;
    const float bsq = s_sq[TM + cl];
    const int nbsh = -s_sh[TM + cl];
    const float rb = AD ? Br[min<int64_t>(n0 + cl, N - 1)] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr0 = wm * 64 + 32 * i + 4 * hl;  // value r sits on row lr0 + 8 (r >> 2) + (r & 3)
      const uint32_t vo = okc ? ((uint32_t)lr0 * ld + (uint32_t)cl) * 4u : OOB;  // value 0's byte offset
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f4 asq = *(const f4*)(s_sq + lr0 + 8 * g);
        const i4v ash = *(const i4v*)(s_sh + lr0 + 8 * g);
        f4 ar = {0.f, 0.f, 0.f, 0.f};
        if constexpr (AD) {
#pragma unroll
          for (int c = 0; c < 4; ++c) ar[c] = Ar[min<int64_t>(m0 + lr0 + 8 * g + c, M - 1)];
        }
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int r = 4 * g + e;
          f2 h, pp, qq;
          h.x = H[i][j][r];
          h.y = H[i][j][r + 1];
          pp.x = P[i][j][r];
          pp.y = P[i][j][r + 1];
          qq.x = Q[i][j][r];
          qq.y = Q[i][j][r + 1];
          f2 dot, sq, d2, t;
          {
#pragma clang fp contract(off)
            const f2 sum = h + (pp + qq);
            dot.x = ldexpf(sum.x, nbsh - ash[e]);
            dot.y = ldexpf(sum.y, nbsh - ash[e + 1]);
            sq.x = asq[e];
            sq.y = asq[e + 1];
            d2 = (sq + bsq) - (dot + dot);  // |a|^2 + |b|^2 - 2 dot (rbf_split_value)
            d2.x = d2.x > 0.f ? d2.x : 0.f;
            d2.y = d2.y > 0.f ? d2.y : 0.f;
            t = (ng * d2) * l2e;  // __expf(-gamma d2) = exp2((-gamma d2) log2 e)
            if constexpr (AD) {  // the one-product pass's value where it is within tau (split_cold)
              f2 dot1, d21, t1;
              dot1.x = ldexpf(h.x, nbsh - ash[e]);
              dot1.y = ldexpf(h.y, nbsh - ash[e + 1]);
              d21 = (sq + bsq) - (dot1 + dot1);
              d21.x = d21.x > 0.f ? d21.x : 0.f;
              d21.y = d21.y > 0.f ? d21.y : 0.f;
              t1 = (ng * d21) * l2e;
              if (split_cold(t1.x, ar[e] + rb, c0, c1)) t.x = t1.x;
              if (split_cold(t1.y, ar[e + 1] + rb, c0, c1)) t.y = t1.y;
            }
          }
          H[i][j][r] = __builtin_amdgcn_exp2f(t.x);
          H[i][j][r + 1] = __builtin_amdgcn_exp2f(t.y);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          // (a float local first: __builtin_bit_cast of a vector element
          // subscript reads element 0 in this hipcc)
          const float hv = H[i][j][r];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hv), rs_o, (int)(vo + (uint32_t)(8 * g + e) * ld * 4u),
                                                0, 0);
        }
      }
      if (mirror) {
        // transposed: lane (column cl) writes rows lr .. lr + 3 of mirrored row cl
        const uint32_t vm = okc ? ((uint32_t)cl * ld + (uint32_t)lr0) * 4u : OOB;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int lr = lr0 + 8 * q;
          f4 v;
          v.x = H[i][j][4 * q + 0];
          v.y = H[i][j][4 * q + 1];
          v.z = H[i][j][4 * q + 2];
          v.w = H[i][j][4 * q + 3];
          const uint32_t o = lr + 3 < rlim ? vm + 32u * q : OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4v, v), rs_m, (int)o, 0, 0);
          if (rlim < TM) {  // uniform: the last row tile — the values of a partial quad one at a time
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const uint32_t oc = (lr + 3 >= rlim && lr + c < rlim) ? vm + 32u * q + 4u * c : OOB;
              const float vc = v[c];
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vc), rs_m, (int)oc, 0, 0);
            }
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Wide-wave LDS-DMA STORE GEMM (variant 5): 256 x 128 tiles, 8 waves of
// 64 x 64 (2 x 2 MFMA tiles, three accumulators each: 192 accumulator
// registers at two waves per SIMD).  The 32 x 64 waves of the kernels above
// read 6 KiB of LDS operands per 6 MFMAs; with the DMA's 32 KiB of LDS writes
// per k block the LDS port needs ~167 B/clk per CU against 128 (PMC: ~35% MFMA
// busy).  A 64 x 64 wave reads 8 KiB per 12 MFMAs: ~114 B/clk with the DMA, so
// the MFMA pipe, not the LDS port, sets the pace.  Same per-element k order
// (H, P, Q over the k blocks in order): bit-identical to the other kernels.
// Symmetric mode: tile (tx, ty) covers 128-row blocks 2 tx and 2 tx + 1 of
// column block ty; computed when ty >= 2 tx, each block above the diagonal
// also stored transposed (the diagonal-straddling tile's lower block is
// written twice with the same bits).  Three 48 KiB buffers of 32 k, one block
// in flight while one is multiplied.
// ---------------------------------------------------------------------------
constexpr int kW64Threads = 512;
// NT 1: non-temporal Gram stores (measured slower, profiles/r4_gram_nt_store_ab.txt);
// NT 2: diagnostics only — stores skipped unless a value is NaN (the store-free time);
// NT 3: diagnostics only — plain stores plus per-workgroup s_memtime stamps
// (entry, first k block landed, k loop done, stores issued, stores done) and
// s_memrealtime at entry / end into stamps[8 blockIdx.x ..] (bench/gram_stamps.py)
// tiles: nullptr = the whole tm x tn grid in the XCD order; else a compact
// table of the tiles to compute (the symmetric Gram's upper tiles, host-built
// in the XCD order: no workgroup is launched only to exit)
// SP 1: the next-but-one block's six LDS-DMA pieces are issued one after each
// group of four MFMAs instead of all six right after the k-block barrier (all
// eight waves then stall on the load path at once while the MFMA pipe idles)
// SP 2 (default): SP 1 plus the operand fragments read from LDS one MFMA group
// ahead with counted lgkmcnt waits, so only the block's first group waits on
// LDS latency (k loop 63.8k -> 59.1k cycles a tile, bench/gram_stamps.py)


template <int NT, int SP = 0, bool PE = false>
__global__ __launch_bounds__(kW64Threads, 1) void rbf_gemm_split_w64_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq, int64_t M,
    const u4* __restrict__ B, const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int64_t N, int nkb,
    float gamma, float* __restrict__ out, int64_t ldo, int sym, const uint32_t* __restrict__ tiles,
    uint64_t* __restrict__ stamps) {
  constexpr int WN = 2, TM = 256, TN = 128, ROWS = TM + TN, CPR = 8, BUF = ROWS * CPR, NB = 3;
  uint64_t st[5] = {0, 0, 0, 0, 0}, rt0 = 0;
  if constexpr (NT == 3) {
    st[0] = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  int64_t tx, ty;
  if (tiles) {
    const uint32_t t = tiles[blockIdx.x];  // (tx << 16) | ty
    tx = t >> 16;
    ty = t & 0xffffu;
  } else {
    xcd_tile(tx, ty);
  }
  if (sym && ty < 2 * tx) return;  // uniform: both 128-row blocks below the diagonal
  __shared__ u4 lds[NB * BUF + 2 * ROWS / 4];  // 3 operand buffers, then |x|^2 [ROWS] and shifts [ROWS]
  float* s_sq = (float*)(lds + NB * BUF);
  int32_t* s_sh = (int32_t*)(lds + NB * BUF) + ROWS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const int64_t m0 = tx * TM, n0 = ty * TN;
  const int64_t rstride = (int64_t)nkb * 8;  // u4 per split row
  if (tid < ROWS) {
    const int64_t ri = tid < TM ? min(m0 + tid, M - 1) : min(n0 + (tid - TM), N - 1);
    s_sq[tid] = tid < TM ? Asq[ri] : Bsq[ri];
    s_sh[tid] = tid < TM ? Ash[ri] : Bsh[ri];
  }
  // DMA: wave w fills stage rows 48 w + 8 i + (lane >> 3), i = 0..5; lane
  // position p = lane & 7 takes global chunk p ^ ((row >> 1) & 7).  An 8-row
  // group is all A or all B rows: a wave-uniform base (SGPRs) plus a 32-bit
  // lane offset keeps the addressing out of the 256 registers the 192
  // accumulators leave room in
  const u4* base[6];
  uint32_t off[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int g = __builtin_amdgcn_readfirstlane(48 * wave + 8 * i);  // first row of the group (uniform)
    const int r = g + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    base[i] = g < TM ? A + (m0 + g) * rstride : B + (n0 + (g - TM)) * rstride;
    off[i] = (uint32_t)((lane >> 3) * rstride + c);
  }
  auto dma_piece = [&](int kb, int i) {
    u4* dst = lds + (kb % NB) * BUF + 48 * wave * CPR;
    __builtin_amdgcn_global_load_lds((const void*)(base[i] + (int64_t)kb * 8 + off[i]),
                                     (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, 0);
  };
  auto dma = [&](int kb) {
#pragma unroll
    for (int i = 0; i < 6; ++i) dma_piece(kb, i);
  };
  __syncthreads();  // row data written (no DMA in flight yet)
  dma(0);
  if (nkb > 1) dma(1);

  f16v H[2][2], P[2][2], Q[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) H[i][j][r] = P[i][j][r] = Q[i][j][r] = 0.f;
  const int sw = ((lane & 31) >> 1) & 7;
  const int ra0 = (wm * 64 + (lane & 31)) * CPR;
  const int rb0 = (TM + wn * 64 + (lane & 31)) * CPR;
  for (int kb = 0; kb < nkb; ++kb) {
    // retire block kb's DMA (block kb + 1 may stay in flight)
    if (kb + 1 < nkb) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (NT == 3) {
      if (kb == 0) st[1] = __builtin_amdgcn_s_memtime();
    }
    // block kb + 2 goes into the buffer of block kb - 1 (every wave is past it)
    if (SP == 0 && kb + 2 < nkb) dma(kb + 2);
    const bool spread = SP != 0 && kb + 2 < nkb;  // uniform
    auto piece = [&](int i) {
      if (spread) {
        __builtin_amdgcn_sched_barrier(0);
        dma_piece(kb + 2, i);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    const u4* buf = lds + (kb % NB) * BUF;
    if constexpr (SP == 2) {
      // LDS reads issued one MFMA group ahead, in asm with counted waits (the
      // compiler drains lgkmcnt to 0 around the LDS-DMA): a group's fragments
      // land while the previous group's MFMAs run, except the block's first.
      // Eight fragments live at most.  A wait names the fragments it retires
      // ("+v"), so no MFMA can move above it
      const uint32_t abase = lds_addr(buf + ra0), bbase = lds_addr(buf + rb0);
      auto rd2 = [&](uint32_t base, int c, h8& x0, h8& x1) {
        const uint32_t a0 = base + 16u * (uint32_t)c;
        asm volatile("ds_read_b128 %0, %1" : "=v"(x0) : "v"(a0) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(x1) : "v"(a0) : "memory");  // + 32 rows
      };
      const int ch0 = hl ^ sw, cl0 = (4 + hl) ^ sw, ch1 = (2 + hl) ^ sw, cl1 = (6 + hl) ^ sw;
      h8 ah0, ah1, bh0, bh1, bl0, bl1, al0, al1, bh0n, bh1n;
      rd2(abase, ch0, ah0, ah1);
      rd2(bbase, ch0, bh0, bh1);
      rd2(bbase, cl0, bl0, bl1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(ah0), "+v"(ah1), "+v"(bh0), "+v"(bh1));
      H[0][0] = mfma32_f16(ah0, bh0, H[0][0]);
      H[0][1] = mfma32_f16(ah0, bh1, H[0][1]);
      H[1][0] = mfma32_f16(ah1, bh0, H[1][0]);
      H[1][1] = mfma32_f16(ah1, bh1, H[1][1]);
      piece(0);
      rd2(abase, cl0, al0, al1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(bl0), "+v"(bl1));
      P[0][0] = mfma32_f16(ah0, bl0, P[0][0]);
      P[0][1] = mfma32_f16(ah0, bl1, P[0][1]);
      P[1][0] = mfma32_f16(ah1, bl0, P[1][0]);
      P[1][1] = mfma32_f16(ah1, bl1, P[1][1]);
      piece(1);
      rd2(abase, ch1, ah0, ah1);  // k step 1 (A hi of step 0 is dead)
      rd2(bbase, ch1, bh0n, bh1n);
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(al0), "+v"(al1));
      Q[0][0] = mfma32_f16(al0, bh0, Q[0][0]);
      Q[0][1] = mfma32_f16(al0, bh1, Q[0][1]);
      Q[1][0] = mfma32_f16(al1, bh0, Q[1][0]);
      Q[1][1] = mfma32_f16(al1, bh1, Q[1][1]);
      piece(2);
      rd2(bbase, cl1, bl0, bl1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(ah0), "+v"(ah1), "+v"(bh0n), "+v"(bh1n));
      H[0][0] = mfma32_f16(ah0, bh0n, H[0][0]);
      H[0][1] = mfma32_f16(ah0, bh1n, H[0][1]);
      H[1][0] = mfma32_f16(ah1, bh0n, H[1][0]);
      H[1][1] = mfma32_f16(ah1, bh1n, H[1][1]);
      piece(3);
      rd2(abase, cl1, al0, al1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(bl0), "+v"(bl1));
      P[0][0] = mfma32_f16(ah0, bl0, P[0][0]);
      P[0][1] = mfma32_f16(ah0, bl1, P[0][1]);
      P[1][0] = mfma32_f16(ah1, bl0, P[1][0]);
      P[1][1] = mfma32_f16(ah1, bl1, P[1][1]);
      piece(4);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(al0), "+v"(al1));
      Q[0][0] = mfma32_f16(al0, bh0n, Q[0][0]);
      Q[0][1] = mfma32_f16(al0, bh1n, Q[0][1]);
      Q[1][0] = mfma32_f16(al1, bh0n, Q[1][0]);
      Q[1][1] = mfma32_f16(al1, bh1n, Q[1][1]);
      piece(5);
      continue;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = (2 * ks + hl) ^ sw, cl = (4 + 2 * ks + hl) ^ sw;
      // hi x hi, then hi x lo (the A hi fragments die), then lo x hi: at most
      // six operand fragments live
      const h8 ah0 = __builtin_bit_cast(h8, buf[ra0 + ch]);
      const h8 ah1 = __builtin_bit_cast(h8, buf[ra0 + 32 * CPR + ch]);
      const h8 bh0 = __builtin_bit_cast(h8, buf[rb0 + ch]);
      const h8 bh1 = __builtin_bit_cast(h8, buf[rb0 + 32 * CPR + ch]);
      H[0][0] = mfma32_f16(ah0, bh0, H[0][0]);
      H[0][1] = mfma32_f16(ah0, bh1, H[0][1]);
      H[1][0] = mfma32_f16(ah1, bh0, H[1][0]);
      H[1][1] = mfma32_f16(ah1, bh1, H[1][1]);
      piece(3 * ks);
      const h8 bl0 = __builtin_bit_cast(h8, buf[rb0 + cl]);
      const h8 bl1 = __builtin_bit_cast(h8, buf[rb0 + 32 * CPR + cl]);
      P[0][0] = mfma32_f16(ah0, bl0, P[0][0]);
      P[0][1] = mfma32_f16(ah0, bl1, P[0][1]);
      P[1][0] = mfma32_f16(ah1, bl0, P[1][0]);
      P[1][1] = mfma32_f16(ah1, bl1, P[1][1]);
      piece(3 * ks + 1);
      const h8 al0 = __builtin_bit_cast(h8, buf[ra0 + cl]);
      const h8 al1 = __builtin_bit_cast(h8, buf[ra0 + 32 * CPR + cl]);
      Q[0][0] = mfma32_f16(al0, bh0, Q[0][0]);
      Q[0][1] = mfma32_f16(al0, bh1, Q[0][1]);
      Q[1][0] = mfma32_f16(al1, bh0, Q[1][0]);
      Q[1][1] = mfma32_f16(al1, bh1, Q[1][1]);
      piece(3 * ks + 2);
    }
  }

  if constexpr (NT == 3) st[2] = __builtin_amdgcn_s_memtime();
  // ---- epilogue, one 32 x 32 MFMA tile at a time: values, direct stores,
  // transposed stores.  ONE code path for interior and edge tiles: a second,
  // interior-only copy (round 4) made the compiler spill 396 B of the live
  // accumulators to scratch (175 scratch instructions).  |x|^2 and shifts are
  // read as 4-row vectors (one LDS round trip per 4 values), stores go to
  // 32-bit offsets from uniform tile bases (host: ldo < 2^24) under a row /
  // column mask that is all-true on interior tiles ----
  typedef int i4v __attribute__((ext_vector_type(4)));
  const bool mirror = sym && ty > 2 * tx + (wm >> 1);  // this wave's 64 rows lie in 128-row block 2 tx + (wm >> 1)
  float* const ob = out + m0 * ldo + n0;  // direct block
  float* const mb = out + n0 * ldo + m0;  // mirrored block (symmetric: M == N)
  const uint32_t ld = (uint32_t)ldo;
  const int rlim = (int)min<int64_t>(M - m0, TM);  // tile rows inside [0, M)
  const int clim = (int)min<int64_t>(N - n0, TN);  // tile columns inside [0, N)
  if constexpr (PE) w64_epilogue_pe(H, P, Q, s_sq, s_sh, lane, wm, wn, mirror, out, m0, n0, M, N, ldo, gamma);
#pragma unroll
  for (int j = 0; j < (PE ? 0 : 2); ++j) {
    const int cl = wn * 64 + 32 * j + (lane & 31);
    const bool okc = cl < clim;
    const float bsq = s_sq[TM + cl];
    const int bsh = s_sh[TM + cl];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr0 = wm * 64 + 32 * i + 4 * hl;  // value r sits on row lr0 + 8 (r >> 2) + (r & 3)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f4 asq = *(const f4*)(s_sq + lr0 + 8 * g);
        const i4v ash = *(const i4v*)(s_sh + lr0 + 8 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e, lr = lr0 + 8 * g + e;
          const float dot = ldexpf(H[i][j][r] + (P[i][j][r] + Q[i][j][r]), -(ash[e] + bsh));
          H[i][j][r] = rbf_split_value(asq[e], bsq, dot, gamma);
          if (NT == 2 && !(H[i][j][r] != H[i][j][r])) continue;
          if (okc && lr < rlim) {
            float* dst = ob + ((uint32_t)lr * ld + (uint32_t)cl);
            if constexpr (NT == 1) __builtin_nontemporal_store(H[i][j][r], dst);
            else *dst = H[i][j][r];
          }
        }
      }
      if (mirror && NT != 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int lr = lr0 + 8 * q;
          float* dst = mb + ((uint32_t)cl * ld + (uint32_t)lr);
          f4 v;
          v.x = H[i][j][4 * q + 0];
          v.y = H[i][j][4 * q + 1];
          v.z = H[i][j][4 * q + 2];
          v.w = H[i][j][4 * q + 3];
          if (okc && lr + 3 < rlim) {
            if constexpr (NT == 1) __builtin_nontemporal_store(v, (f4*)dst);
            else *(f4*)dst = v;
          } else if (okc) {
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (lr + c < rlim) dst[c] = v[c];
          }
        }
      }
    }
  }
  if constexpr (NT == 3) {
    st[3] = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st[4] = __builtin_amdgcn_s_memtime();
    const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      uint64_t* o = stamps + (size_t)blockIdx.x * 8;
#pragma unroll
      for (int i = 0; i < 5; ++i) o[i] = st[i];
      o[5] = rt0;
      o[6] = rt1;
      o[7] = ((uint64_t)tx << 32) | (uint64_t)ty;
    }
  }
}

// ---------------------------------------------------------------------------
// Persistent wide-wave STORE GEMM (the default; PE: the packed epilogue,
// variant 12; variant 7 without it; DPSVM_GRAM_PERSIST=0 for the tile-per-
// workgroup kernel): the w64 kernel's tile, k loop (with SP 2's read-ahead)
// and epilogue, one workgroup per CU walking tiles L = b, b + G, ... of the
// same table.  The w64 kernel's stamps put ~12% of a tile in its prologue (row
// data, then the first LDS-DMA block's latency) with the MFMA pipe idle, and
// ~7% of the CU time between workgroups (237.5 of 256 in flight).  Here the
// LDS-DMA ring runs on across tiles: during the last two k blocks of tile t
// the prefetch slots load blocks 0 and 1 of tile t + 1 (a block counter g
// over all tiles picks the buffer, g mod 3), and the next tile's |x|^2 and
// shifts arrive by LDS-DMA into the other parity of a row-data area (issued
// after tile t's k loop); every epilogue ends with vmcnt(0), so the loop's one
// uniform wait holds at the next tile's first block.  With the packed
// epilogue: 8.86 vs 9.01 ms symmetric, 2.30 vs 2.47 ms for the P = 8 slab
// against the w64 kernel (profiles/r6_gram_lds_readahead_ab.json).  Same MFMA
// sequence per output: bit-identical to the w64 kernel.
// NT 3: per-tile stamps (first wait, first block landed, k loop done, stores
// issued) and s_memrealtime at the tile's start / end into stamps[8 L ..].
// ---------------------------------------------------------------------------
// LDS-DMA piece of a k block into ring buffer buf.  The persistent kernel
// gives every wave four pieces of A rows (wave w: rows 32 w + 8 i) and two of B
// rows (rows 256 + 16 w + 8 i): six pieces a wave as in the w64 kernel (one
// uniform vmcnt), with two fixed source pointers and row bases, so a piece is
// one scalar add and two vector ops (u: the k block's row offset, uniform).
// Lane position p = lane & 7 takes global chunk p ^ ((row >> 1) & 7), the w64
// kernel's swizzle; for these rows that is p ^ (((lane >> 4) + 4 (i & 1)) & 7):
// two lane offsets for all pieces (off_e / off_o).
// The address is a uniform base plus the lane's byte offset (laundered by the
// caller, so it is not re-derived per piece): the saddr form of the DMA, no
// vector math per piece.
__device__ __forceinline__ void w64p_piece(const u4* __restrict__ src, u4* lds, uint32_t u, uint32_t step,
                                           int dst_row8, uint32_t off_e, uint32_t off_o, int buf, int i) {
  constexpr int BUF = 384 * 8;
  u4* dst = lds + buf * BUF + dst_row8 + i * 64;
  const char* base = (const char*)(src + (u + (uint32_t)i * step));  // uniform
  __builtin_amdgcn_global_load_lds((const void*)(base + ((i & 1) ? off_o : off_e)),
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// a tile's |x|^2 and shifts into row-data parity par: dwords d = 64 (2 wave +
// i) + lane (two 4-B LDS-DMA instructions a wave, every wave: a uniform count
// for the waits; ROWS = 384 and TM = 256 are multiples of 64, so the array an
// instruction reads is wave-uniform); rows past M / N clamp as the w64 kernel's
// loads do
__device__ __forceinline__ void w64p_row_dma(const float* __restrict__ Asq, const float* __restrict__ Bsq,
                                             const int32_t* __restrict__ Ash, const int32_t* __restrict__ Bsh, int M,
                                             int N, uint32_t* s_rows, int wave, int lane, int m0, int n0, int par) {
  constexpr int TM = 256, ROWS = 384, RD = 1024;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int d0 = __builtin_amdgcn_readfirstlane(64 * (2 * wave + i));
    const int r0 = d0 < ROWS ? d0 : d0 - ROWS;    // uniform
    const bool a_rows = r0 < TM, sq = d0 < ROWS;  // uniform
    const uint32_t* arr = sq ? (a_rows ? (const uint32_t*)Asq : (const uint32_t*)Bsq)
                             : (a_rows ? (const uint32_t*)Ash : (const uint32_t*)Bsh);
    const int r = r0 + lane;
    const int ri = a_rows ? min(m0 + r, M - 1) : min(n0 + (r - TM), N - 1);
    const uint32_t* src = d0 >= 2 * ROWS ? arr : arr + ri;  // padding: any valid address
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(s_rows + par * RD + d0),
                                     4, 0, 0);
  }
}

// AD (with PE): the adaptive Gram's hot-tile pass — the tile count is read from
// ntiles_dev (written by the one-product pass) and the epilogue applies
// split_cold with Ar / Br, c0, c1.
template <int NT, bool PE = false, bool AD = false>
__global__ __launch_bounds__(kW64Threads, 1) void rbf_gemm_split_w64p_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq, int M,
    const u4* __restrict__ B, const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int N, int nkb,
    float gamma, float* __restrict__ out, int ldo, int sym, const uint32_t* __restrict__ tiles, int ntiles,
    int tm, int tn, uint64_t* __restrict__ stamps, const float* __restrict__ Ar = nullptr,
    const float* __restrict__ Br = nullptr, float c0 = 0.f, float c1 = 0.f,
    const uint32_t* __restrict__ ntiles_dev = nullptr) {
  // 32-bit indices throughout (launcher: M, N, ldo and (M + 512) x nkb x 8 < 2^31):
  // the loop-carried tile state must fit the scalar registers beside the
  // k loop's, or the 192 accumulators spill
  constexpr int WN = 2, TM = 256, TN = 128, ROWS = TM + TN, CPR = 8, BUF = ROWS * CPR, NB = 3;
  constexpr int RD = 1024;  // row-data dwords per parity: |x|^2 [ROWS], shifts [ROWS], DMA padding
  __shared__ u4 lds[NB * BUF + 2 * RD / 4];  // 3 operand buffers, then row data [2][RD]
  uint32_t* const s_rows = (uint32_t*)(lds + NB * BUF);
  const int G = gridDim.x;
  int L = blockIdx.x;
  if constexpr (AD) ntiles = (int)__builtin_amdgcn_readfirstlane(*ntiles_dev);
  if (L >= ntiles) return;  // uniform: no barrier reached
  uint32_t t = tiles[L];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const uint32_t rs = (uint32_t)nkb * 8;  // u4 per split row
  // every wave: 4 pieces of A rows, 2 of B rows a k block (w64p_piece)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t step = 8 * rs;
  // the lanes' byte offsets within a piece (even / odd pieces)
  uint32_t off_e = 16u * ((uint32_t)(lane >> 3) * rs + (uint32_t)((lane & 7) ^ (lane >> 4)));
  uint32_t off_o = 16u * ((uint32_t)(lane >> 3) * rs + (uint32_t)((lane & 7) ^ ((lane >> 4) + 4)));
  asm volatile("" : "+v"(off_e), "+v"(off_o));
  const int dstA = 32 * wv * 8, dstB = (TM + 16 * wv) * 8;
#define PIECE_A(uA_, buf_, i_) w64p_piece(A, lds, uA_, step, dstA, off_e, off_o, buf_, i_)
#define PIECE_B(uB_, buf_, i_) w64p_piece(B, lds, uB_, step, dstB, off_e, off_o, buf_, i_)
#define ROW_DMA(m0_, n0_, par_) w64p_row_dma(Asq, Bsq, Ash, Bsh, M, N, s_rows, wave, lane, m0_, n0_, par_)
  int Ln = L + G;
  uint32_t tn_next = Ln < ntiles ? tiles[Ln] : 0u;
  int par = 0;
  uint32_t g = 0;  // k blocks started over all of this workgroup's tiles: ring buffer g % NB
  {
    const int m0 = (int)(t >> 16) * TM, n0 = (int)(t & 0xffffu) * TN;
    ROW_DMA(m0, n0, 0);
#pragma unroll
    for (int b = 0; b < 2; ++b) {  // blocks 0 and 1 (launcher: nkb >= 3)
      const uint32_t uA = (uint32_t)(m0 + 32 * wv) * rs + (uint32_t)b * 8;
      const uint32_t uB = (uint32_t)(n0 + 16 * wv) * rs + (uint32_t)b * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) PIECE_A(uA, b, i);
#pragma unroll
      for (int i = 0; i < 2; ++i) PIECE_B(uB, b, i);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the loop's first wait counts 6 younger: tile 0 starts landed
  }
  const int sw = ((lane & 31) >> 1) & 7;
  const int ra0 = (wm * 64 + (lane & 31)) * CPR;
  const int rb0 = (TM + wn * 64 + (lane & 31)) * CPR;
  while (true) {
    uint64_t st[4] = {0, 0, 0, 0}, rt0 = 0;
    if constexpr (NT == 3) {
      st[0] = __builtin_amdgcn_s_memtime();
      rt0 = __builtin_amdgcn_s_memrealtime();
    }
    const bool has_next = Ln < ntiles;  // uniform
    const int tx = (int)(t >> 16), ty = (int)(t & 0xffffu);
    const int m0 = tx * TM, n0 = ty * TN;
    // (the last tile prefetches its own blocks 0 / 1 into dead buffers: no branch in the loop)
    const uint32_t tp = has_next ? tn_next : t;
    const int nm0 = (int)(tp >> 16) * TM, nn0 = (int)(tp & 0xffffu) * TN;
    f16v H[2][2], P[2][2], Q[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) H[i][j][r] = P[i][j][r] = Q[i][j][r] = 0.f;
#pragma clang loop unroll(disable)
    for (int kb = 0; kb < nkb; ++kb) {
      // retire block kb's DMA: block kb + 1 (6 pieces a wave) may stay in flight.
      // Every k block prefetches (the last tile's last two re-load blocks 0 / 1
      // of itself into dead buffers) and every epilogue ends with vmcnt(0): one
      // wait, no branch (a taken branch a piece cost ~10% of the loop)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if constexpr (NT == 3) {
        if (kb == 0) st[1] = __builtin_amdgcn_s_memtime();
      }
      // the prefetch slot: block kb + 2 of this tile, or block kb + 2 - nkb of
      // the next one, into the buffer of block g - 1 (every wave is past it)
      const bool own = kb + 2 < nkb;
      const int pkb = own ? kb + 2 : kb + 2 - nkb;
      const uint32_t uA = (uint32_t)((own ? m0 : nm0) + 32 * wv) * rs + (uint32_t)pkb * 8;
      const uint32_t uB = (uint32_t)((own ? n0 : nn0) + 16 * wv) * rs + (uint32_t)pkb * 8;
      const int pbuf = (int)((g + 2) % NB);
      // after MFMA group j (0..5) of the block: A0, A1, B0, A2, A3, B1
      auto piece = [&](int j) {
        __builtin_amdgcn_sched_barrier(0);
        if (j == 2 || j == 5) PIECE_B(uB, pbuf, j == 2 ? 0 : 1);
        else PIECE_A(uA, pbuf, j < 2 ? j : j - 1);
        __builtin_amdgcn_sched_barrier(0);
      };
      // operand fragments read one MFMA group ahead (the w64 kernel's SP 2)
      const u4* buf = lds + (g % NB) * BUF;
      const uint32_t abase = lds_addr(buf + ra0), bbase = lds_addr(buf + rb0);
      auto rd2 = [&](uint32_t base, int c, h8& x0, h8& x1) {
        const uint32_t a0 = base + 16u * (uint32_t)c;
        asm volatile("ds_read_b128 %0, %1" : "=v"(x0) : "v"(a0) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(x1) : "v"(a0) : "memory");  // + 32 rows
      };
      const int ch0 = hl ^ sw, cl0 = (4 + hl) ^ sw, ch1 = (2 + hl) ^ sw, cl1 = (6 + hl) ^ sw;
      h8 ah0, ah1, bh0, bh1, bl0, bl1, al0, al1, bh0n, bh1n;
      rd2(abase, ch0, ah0, ah1);
      rd2(bbase, ch0, bh0, bh1);
      rd2(bbase, cl0, bl0, bl1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(ah0), "+v"(ah1), "+v"(bh0), "+v"(bh1));
      H[0][0] = mfma32_f16(ah0, bh0, H[0][0]);
      H[0][1] = mfma32_f16(ah0, bh1, H[0][1]);
      H[1][0] = mfma32_f16(ah1, bh0, H[1][0]);
      H[1][1] = mfma32_f16(ah1, bh1, H[1][1]);
      piece(0);
      rd2(abase, cl0, al0, al1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(bl0), "+v"(bl1));
      P[0][0] = mfma32_f16(ah0, bl0, P[0][0]);
      P[0][1] = mfma32_f16(ah0, bl1, P[0][1]);
      P[1][0] = mfma32_f16(ah1, bl0, P[1][0]);
      P[1][1] = mfma32_f16(ah1, bl1, P[1][1]);
      piece(1);
      rd2(abase, ch1, ah0, ah1);
      rd2(bbase, ch1, bh0n, bh1n);
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(al0), "+v"(al1));
      Q[0][0] = mfma32_f16(al0, bh0, Q[0][0]);
      Q[0][1] = mfma32_f16(al0, bh1, Q[0][1]);
      Q[1][0] = mfma32_f16(al1, bh0, Q[1][0]);
      Q[1][1] = mfma32_f16(al1, bh1, Q[1][1]);
      piece(2);
      rd2(bbase, cl1, bl0, bl1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(ah0), "+v"(ah1), "+v"(bh0n), "+v"(bh1n));
      H[0][0] = mfma32_f16(ah0, bh0n, H[0][0]);
      H[0][1] = mfma32_f16(ah0, bh1n, H[0][1]);
      H[1][0] = mfma32_f16(ah1, bh0n, H[1][0]);
      H[1][1] = mfma32_f16(ah1, bh1n, H[1][1]);
      piece(3);
      rd2(abase, cl1, al0, al1);
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(bl0), "+v"(bl1));
      P[0][0] = mfma32_f16(ah0, bl0, P[0][0]);
      P[0][1] = mfma32_f16(ah0, bl1, P[0][1]);
      P[1][0] = mfma32_f16(ah1, bl0, P[1][0]);
      P[1][1] = mfma32_f16(ah1, bl1, P[1][1]);
      piece(4);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(al0), "+v"(al1));
      Q[0][0] = mfma32_f16(al0, bh0n, Q[0][0]);
      Q[0][1] = mfma32_f16(al0, bh1n, Q[0][1]);
      Q[1][0] = mfma32_f16(al1, bh0n, Q[1][0]);
      Q[1][1] = mfma32_f16(al1, bh1n, Q[1][1]);
      piece(5);
      ++g;
    }
    if constexpr (NT == 3) st[2] = __builtin_amdgcn_s_memtime();
    // the next tile's row data into the other parity (last read by the previous
    // tile's epilogue, before this tile's first barrier)
    if (has_next) ROW_DMA(nm0, nn0, par ^ 1);

    // ---- epilogue of the w64 kernel (row data from parity `par`) ----
    if constexpr (PE) {
      int el = lane;
      asm volatile("" : "+v"(el));
      w64_epilogue_pe<AD>(H, P, Q, (const float*)(s_rows + par * RD), (const int32_t*)(s_rows + par * RD + ROWS),
                          el, wm, wn, sym && ty > 2 * tx + (wm >> 1), out, m0, n0, M, N, ldo, gamma, Ar, Br, c0,
                          c1);
    }
    // (the per-lane epilogue addresses are recomputed per tile from a
    // laundered lane id: hoisted out of the tile loop they would hold ~64
    // registers across the k loop)
    int el = lane;
    asm volatile("" : "+v"(el));
    const int ewn = wn, ewm = wm, ehl = el >> 5;
    typedef int i4v __attribute__((ext_vector_type(4)));
    const float* s_sq = (const float*)(s_rows + par * RD);
    const int32_t* s_sh = (const int32_t*)(s_rows + par * RD + ROWS);
    const bool mirror = sym && ty > 2 * tx + (ewm >> 1);
    float* const ob = out + ((uint32_t)m0 * (uint32_t)ldo + (uint32_t)n0);
    float* const mb = out + ((uint32_t)n0 * (uint32_t)ldo + (uint32_t)m0);
    const uint32_t ld = (uint32_t)ldo;
    const int rlim = min(M - m0, TM);
    const int clim = min(N - n0, TN);
#pragma unroll
    for (int j = 0; j < (PE ? 0 : 2); ++j) {
      const int cl = ewn * 64 + 32 * j + (el & 31);
      const bool okc = cl < clim;
      const float bsq = s_sq[TM + cl];
      const int bsh = s_sh[TM + cl];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int lr0 = ewm * 64 + 32 * i + 4 * ehl;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const f4 asq = *(const f4*)(s_sq + lr0 + 8 * q4);
          const i4v ash = *(const i4v*)(s_sh + lr0 + 8 * q4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * q4 + e, lr = lr0 + 8 * q4 + e;
            const float dot = ldexpf(H[i][j][r] + (P[i][j][r] + Q[i][j][r]), -(ash[e] + bsh));
            H[i][j][r] = rbf_split_value(asq[e], bsq, dot, gamma);
            if (okc && lr < rlim) ob[(uint32_t)lr * ld + (uint32_t)cl] = H[i][j][r];
          }
        }
        if (mirror) {
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const int lr = lr0 + 8 * q4;
            float* dst = mb + ((uint32_t)cl * ld + (uint32_t)lr);
            f4 v;
            v.x = H[i][j][4 * q4 + 0];
            v.y = H[i][j][4 * q4 + 1];
            v.z = H[i][j][4 * q4 + 2];
            v.w = H[i][j][4 * q4 + 3];
            if (okc && lr + 3 < rlim) {
              *(f4*)dst = v;
            } else if (okc) {
#pragma unroll
              for (int c = 0; c < 4; ++c)
                if (lr + c < rlim) dst[c] = v[c];
            }
          }
        }
      }
    }
    // the stores, the next tile's blocks 0 / 1 and its row data retired here:
    // the loop's uniform vmcnt(6) then holds at the next tile's first block (and
    // no DMA is in flight when the kernel ends)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (NT == 3) {
      st[3] = __builtin_amdgcn_s_memtime();
      const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
      if (tid == 0) {
        uint64_t* o = stamps + (size_t)L * 8;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = st[i];
        o[4] = st[3];
        o[5] = rt0;
        o[6] = rt1;
        o[7] = t;
      }
    }
    if (!has_next) break;
    L = Ln;
    t = tn_next;
    par ^= 1;
    Ln = L + G;
    if (Ln < ntiles) tn_next = tiles[Ln];
  }
}
#undef PIECE_A
#undef PIECE_B
#undef ROW_DMA

// ---------------------------------------------------------------------------
// Adaptive split Gram, pass 1: the one-product (h_a . h_b) Gram with per-tile
// hot reports (docs/DESIGN.md §13).  Where the kernel is far from the identity
// only near the diagonal (the headline: every off-diagonal K < 3e-6), the two
// correction products change no stored value by more than tau = 2^-22 — 45x
// below the three-product Gram's own error vs float64 — and split_cold proves
// it element by element.  This pass multiplies the h planes only (1/3 of the
// MFMAs, half the operand bytes), stores K1 everywhere and appends every tile
// holding an element split_cold rejects to a list; pass 2 (w64p, AD) recomputes
// those tiles with all three products.  The H accumulator's MFMA sequence is
// the three-product kernels' (same k order), so K1 and the rule's inputs are
// the same bits in both passes.
// Tiles and the persistent LDS-DMA ring are the w64p kernel's; the operands are
// h planes (split_hplane_kernel: a row's h halves back to back, zero-padded to an
// even block count), so a ring stage is 64 k = one whole 128-B line a row; an
// odd block count's last stage multiplies the zero pad (H + 0 is H).  64
// accumulator registers instead of 192.  Measured and dropped on the way
// (profiles/r6_gram_adapt/h1_ablation_kernels.txt): one workgroup whose waves
// both feed the ring and store (each tile then waits on its own stores:
// 6.32 ms), the split rows' h halves as operands (half of every fetched line
// unused: 7.32 ms), deferring a tile's stores into the next tile's ring (spills,
// 10.3 ms), two workgroups per CU of 128 x 64 waves over 32-k stages (8.5 ms),
// staggered workgroup starts (no change).
// tile_hot [ntiles] (zeroed): per-tile report counts; hot[0] (zeroed) the
// list's length, hot[1 ..] the reported tiles' table entries.
// ---------------------------------------------------------------------------
// the one-product epilogue's math: H becomes K1 = exp2(t1) in place; returns
// (wave-uniform) whether any of the wave's elements is hot
__device__ __forceinline__ bool h1_values(f16v (&H)[2][2], const float* s_sq, const int32_t* s_sh, const float* s_r,
                                          int lane, int wm, int wn, float gamma, float c0, float c1) {
  constexpr int TM = 256;
  typedef i4v_t i4v;
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int hl = lane >> 5;
  const float ng = -gamma, l2e = 1.4426950408889634f;
  bool hot = false;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = wn * 64 + 32 * j + (lane & 31);
    const float bsq = s_sq[TM + cl];
    const int nbsh = -s_sh[TM + cl];
    const float rb = s_r[TM + cl];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      // one 32 x 32 block's row data at a time (the scheduler hoisting every
      // block's LDS reads ahead made the specialised kernel spill)
      __builtin_amdgcn_sched_barrier(0);
      const int lr0 = wm * 64 + 32 * i + 4 * hl;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f4 asq = *(const f4*)(s_sq + lr0 + 8 * g);
        const i4v ash = *(const i4v*)(s_sh + lr0 + 8 * g);
        const f4 ar = *(const f4*)(s_r + lr0 + 8 * g);
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int r = 4 * g + e;
          f2 h, dot, sq, d2, t;
          h.x = H[i][j][r];
          h.y = H[i][j][r + 1];
          {
#pragma clang fp contract(off)
            dot.x = ldexpf(h.x, nbsh - ash[e]);
            dot.y = ldexpf(h.y, nbsh - ash[e + 1]);
            sq.x = asq[e];
            sq.y = asq[e + 1];
            d2 = (sq + bsq) - (dot + dot);
            d2.x = d2.x > 0.f ? d2.x : 0.f;
            d2.y = d2.y > 0.f ? d2.y : 0.f;
            t = (ng * d2) * l2e;
            hot |= !split_cold(t.x, ar[e] + rb, c0, c1);
            hot |= !split_cold(t.y, ar[e + 1] + rb, c0, c1);
          }
          H[i][j][r] = __builtin_amdgcn_exp2f(t.x);
          H[i][j][r + 1] = __builtin_amdgcn_exp2f(t.y);
        }
      }
    }
  }
  return __builtin_amdgcn_ballot_w64(hot) != 0;
}

// the stores of one 32 x 32 MFMA block (i, j) of a wave's values v: 16 direct
// 4-B stores per lane, and for a mirroring wave 4 transposed 16-B ones (plus,
// on the last row tile, a partial quad's values one at a time); out-of-range
// offsets where a value has no place (the hardware drops those).  ABL
// (diagnostics): 1 every store dropped, 2 the mirrored ones; 4 (A/B): every
// store with the non-temporal cache policy.
template <int ABL = 0>
__device__ __forceinline__ void h1_store_block(const f16v& v, int i, int j, int lane, int wm, int wn, bool mirror,
                                               bool valid, float* out, int m0, int n0, int M, int N, int ldo) {
  constexpr int TM = 256, TN = 128;
  typedef i4v_t i4v;
  constexpr uint32_t OOB = 0x80000000u;
  const int hl = lane >> 5;
  float* const ob = out + ((int64_t)m0 * ldo + n0);
  float* const mb = out + ((int64_t)n0 * ldo + m0);
  const uint32_t ld = (uint32_t)ldo;
  const int rlim = min(M - m0, TM);
  const int clim = min(N - n0, TN);
  const int64_t ob_bytes = min<int64_t>((int64_t)(M - m0) * ldo * 4 - (int64_t)n0 * 4, (int64_t)OOB);
  const int64_t mb_bytes = min<int64_t>((int64_t)(N - n0) * ldo * 4 - (int64_t)m0 * 4, (int64_t)OOB);
  const __amdgpu_buffer_rsrc_t rs_o = __builtin_amdgcn_make_buffer_rsrc(ob, 0, (int)ob_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_m = __builtin_amdgcn_make_buffer_rsrc(mb, 0, (int)mb_bytes, 0x00020000);
  const int cl = wn * 64 + 32 * j + (lane & 31);
  const bool okc = valid && cl < clim && ABL != 1;
  constexpr int CP = ABL == 4 ? 2 : 0;  // buffer-store cache policy: nt
  const int lr0 = wm * 64 + 32 * i + 4 * hl;
  const uint32_t vo = okc ? ((uint32_t)lr0 * ld + (uint32_t)cl) * 4u : OOB;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float hv = v[r];
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hv), rs_o,
                                          (int)(vo + (uint32_t)(8 * (r >> 2) + (r & 3)) * ld * 4u), 0, CP);
  }
  if (!(mirror && valid) || ABL == 2) return;  // uniform
  const bool okm = okc;
  const uint32_t vm = okm ? ((uint32_t)cl * ld + (uint32_t)lr0) * 4u : OOB;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int lr = lr0 + 8 * q;
    f4 w;
    w.x = v[4 * q + 0];
    w.y = v[4 * q + 1];
    w.z = v[4 * q + 2];
    w.w = v[4 * q + 3];
    const uint32_t o = lr + 3 < rlim && okm ? vm + 32u * q : OOB;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4v, w), rs_m, (int)o, 0, CP);
    if (rlim < TM) {  // uniform: the last row tile — a partial quad's values one at a time
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t oc = (okm && lr + 3 >= rlim && lr + c < rlim) ? vm + 32u * q + 4u * c : OOB;
        const float vc = w[c];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vc), rs_m, (int)oc, 0, CP);
      }
    }
  }
}

// the h1s kernel's DMA waves (a function of its own: its uniform addressing
// does not share the compute waves' scalar registers)
__device__ __noinline__ void h1s_dma(const u4* __restrict__ A, const int32_t* __restrict__ Ash,
                                     const float* __restrict__ Asq, const float* __restrict__ Ar, int M,
                                     const u4* __restrict__ B, const int32_t* __restrict__ Bsh,
                                     const float* __restrict__ Bsq, const float* __restrict__ Br, int N, int nst,
                                     const uint32_t* __restrict__ tiles, int ntiles, int L, int dwave, int lane,
                                     u4* lds, uint32_t* s_rows) {
  constexpr int TM = 256, TN = 128, ROWS = TM + TN, NB = 3, RD = 1536;
  const int G = gridDim.x;
  const uint32_t rs = (uint32_t)nst * 8;
  uint32_t t = tiles[L];
  int Ln = L + G;
  uint32_t tn_next = Ln < ntiles ? tiles[Ln] : 0u;
  uint32_t g = 0;
  const int dw = __builtin_amdgcn_readfirstlane(dwave);
    const int p = lane & 7;
    uint32_t off_e = 16u * ((uint32_t)(lane >> 3) * rs + (uint32_t)(p ^ (lane >> 4)));
    uint32_t off_o = 16u * ((uint32_t)(lane >> 3) * rs + (uint32_t)(p ^ ((lane >> 4) + 4)));
    asm volatile("" : "+v"(off_e), "+v"(off_o));
    auto stage = [&](int m0_, int n0_, int st, int buf) {
      const uint32_t uA = (uint32_t)(m0_ + 64 * dw) * rs + (uint32_t)st * 8;
      const uint32_t uB = (uint32_t)(n0_ + 32 * dw) * rs + (uint32_t)st * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) w64p_piece(A, lds, uA, 8 * rs, 64 * dw * 8, off_e, off_o, buf, i);
#pragma unroll
      for (int i = 0; i < 4; ++i) w64p_piece(B, lds, uB, 8 * rs, (TM + 32 * dw) * 8, off_e, off_o, buf, i);
    };
    // row data: DMA wave dw = 0 / 1 / 2 loads |x|^2 / shifts / log2 |x| of the 384 rows (six chunks of 64:
    // A rows for i < 4); wave 3 loads a valid word into the padding (every stage wait counts 6)
    const uint32_t* const rd_a =
        dw == 0 ? (const uint32_t*)Asq : dw == 1 ? (const uint32_t*)Ash : (const uint32_t*)Ar;
    const uint32_t* const rd_b =
        dw == 0 ? (const uint32_t*)Bsq : dw == 1 ? (const uint32_t*)Bsh : (const uint32_t*)Br;
    auto rowdata = [&](int m0_, int n0_, int par_) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int r = 64 * i + lane;
        const int ri = i < 4 ? min(m0_ + r, M - 1) : min(n0_ + (r - TM), N - 1);
        const uint32_t* src = dw == 3 ? (const uint32_t*)Asq : (i < 4 ? rd_a : rd_b) + ri;
        __builtin_amdgcn_global_load_lds(
            (const void*)src, (__attribute__((address_space(3))) void*)(s_rows + par_ * RD + 64 * (6 * dw + i)),
            4, 0, 0);
      }
    };
    {
      const int m0 = (int)(t >> 16) * TM, n0 = (int)(t & 0xffffu) * TN;
      stage(m0, n0, 0, 0);
      stage(m0, n0, 1, 1);
      rowdata(m0, n0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    int par = 0;
    while (true) {
      const bool has_next = Ln < ntiles;  // uniform
      const int m0 = (int)(t >> 16) * TM, n0 = (int)(t & 0xffffu) * TN;
      const uint32_t tp = has_next ? tn_next : t;
      const int nm0 = (int)(tp >> 16) * TM, nn0 = (int)(tp & 0xffffu) * TN;
#pragma clang loop unroll(disable)
      for (int s = 0; s < nst; ++s) {
        // stage s landed: younger are stage s + 1 (12 pieces) and, at s == 1, the next tile's row data (6)
        if (s == 1) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const bool own = s + 2 < nst;
        stage(own ? m0 : nm0, own ? n0 : nn0, own ? s + 2 : s + 2 - nst, (int)((g + 2) % NB));
        // the next tile's row data (the last tile reloads its own into the unused parity: the count stays 6)
        if (s == 0) rowdata(nm0, nn0, par ^ 1);
        ++g;
      }
      if (!has_next) break;
      L = Ln;
      t = tn_next;
      par ^= 1;
      Ln = L + G;
      if (Ln < ntiles) tn_next = tiles[Ln];
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

constexpr int kH1sThreads = 768;  // 8 compute waves + 4 DMA waves
template <int ABL = 0>
__global__ __launch_bounds__(kH1sThreads, 1) void rbf_gemm_split_h1s_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq,
    const float* __restrict__ Ar, int M, const u4* __restrict__ B, const int32_t* __restrict__ Bsh,
    const float* __restrict__ Bsq, const float* __restrict__ Br, int N, int nkb, float gamma, float c0, float c1,
    float* __restrict__ out, int ldo, int sym, const uint32_t* __restrict__ tiles, int ntiles,
    uint32_t* __restrict__ tile_hot, uint32_t* __restrict__ hot) {
  constexpr int WN = 2, TM = 256, TN = 128, ROWS = TM + TN, CPR = 8, BUF = ROWS * CPR, NB = 3, RD = 1536;
  __shared__ u4 lds[NB * BUF + 2 * RD / 4];  // 3 operand buffers, then row data [2][RD]
  uint32_t* const s_rows = (uint32_t*)(lds + NB * BUF);
  const int G = gridDim.x;
  int L = blockIdx.x;
  if (L >= ntiles) return;  // uniform
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nst = (nkb + 1) >> 1;  // ring stages a tile (launcher: nkb >= 5)
  if (__builtin_amdgcn_readfirstlane(wave) >= 8) {
    h1s_dma(A, Ash, Asq, Ar, M, B, Bsh, Bsq, Br, N, nst, tiles, ntiles, L, wave - 8, lane, lds, s_rows);
    return;
  }
  // ---- compute waves: the h1 kernel's 64 x 64 waves; never a load, so their stores drain unwaited ----
  uint32_t t = tiles[L];
  int Ln = L + G;
  uint32_t tn_next = Ln < ntiles ? tiles[Ln] : 0u;
  uint32_t g = 0;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const int sw = ((lane & 31) >> 1) & 7;
  const int ra0 = (wm * 64 + (lane & 31)) * CPR;
  const int rb0 = (TM + wn * 64 + (lane & 31)) * CPR;
  int par = 0;
  while (true) {
    const bool has_next = Ln < ntiles;  // uniform
    const int tx = (int)(t >> 16), ty = (int)(t & 0xffffu);
    const int m0 = tx * TM, n0 = ty * TN;
    f16v H[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) H[i][j][r] = 0.f;
#pragma clang loop unroll(disable)
    for (int s = 0; s < nst; ++s) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const u4* buf = lds + (g % NB) * BUF;
      const uint32_t abase = lds_addr(buf + ra0), bbase = lds_addr(buf + rb0);
      auto rd = [&](int q, h8& a0, h8& a1, h8& b0, h8& b1) {
        const uint32_t c = 16u * (uint32_t)((2 * q + hl) ^ sw);
        const uint32_t pa = abase + c, pb = bbase + c;
        asm volatile("ds_read_b128 %0, %1" : "=v"(a0) : "v"(pa) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(a1) : "v"(pa) : "memory");
        asm volatile("ds_read_b128 %0, %1" : "=v"(b0) : "v"(pb) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(b1) : "v"(pb) : "memory");
      };
      auto mma = [&](const h8& a0, const h8& a1, const h8& b0, const h8& b1) {
        if (ABL == 3) return;
        H[0][0] = mfma32_f16(a0, b0, H[0][0]);
        H[0][1] = mfma32_f16(a0, b1, H[0][1]);
        H[1][0] = mfma32_f16(a1, b0, H[1][0]);
        H[1][1] = mfma32_f16(a1, b1, H[1][1]);
      };
      // (an odd block count's last stage multiplies the h plane's zero pad: H + 0 is H, bit for bit)
      h8 x0, x1, x2, x3, y0, y1, y2, y3;
      rd(0, x0, x1, x2, x3);
      rd(1, y0, y1, y2, y3);
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
      mma(x0, x1, x2, x3);
      rd(2, x0, x1, x2, x3);
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
      mma(y0, y1, y2, y3);
      rd(3, y0, y1, y2, y3);
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
      mma(x0, x1, x2, x3);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
      mma(y0, y1, y2, y3);
      ++g;
    }
    int el = lane;
    asm volatile("" : "+v"(el));
    const float* rows = (const float*)(s_rows + par * RD);
    const bool hotw = h1_values(H, rows, (const int32_t*)(rows + ROWS), rows + 2 * ROWS, el, wm, wn, gamma, c0, c1);
    const bool mirror = sym && ty > 2 * tx + (wm >> 1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        __builtin_amdgcn_sched_barrier(0);
        h1_store_block<ABL>(H[i][j], i, j, el, wm, wn, mirror, true, out, m0, n0, M, N, ldo);
      }
    if (hotw && lane == 0) {  // the tile's first report appends it to the list
      if (atomicAdd(tile_hot + L, 1u) == 0u) {
        const uint32_t k = atomicAdd(hot, 1u);
        hot[1 + k] = t;
      }
    }
    if (!has_next) break;
    L = Ln;
    t = tn_next;
    par ^= 1;
    Ln = L + G;
    if (Ln < ntiles) tn_next = tiles[Ln];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// h planes of split rows (the one-product pass's operands): row r holds the h
// halves of its nkb split blocks back to back, then zeros to an even count
__global__ __launch_bounds__(256) void split_hplane_kernel(const u4* __restrict__ src, int64_t rows, int nkb,
                                                          u4* __restrict__ dst) {
  const int nq = ((nkb + 1) >> 1) * 8;  // u4 per plane row
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * nq) return;
  const int64_t r = e / nq;
  const int q = (int)(e - r * nq), b = q >> 2, c = q & 3;
  dst[e] = b < nkb ? src[r * nkb * 8 + b * 8 + c] : u4{0u, 0u, 0u, 0u};
}

// R = log2 |x| = split_log2norm(|x|^2) of n rows (the adaptive Gram's rule input)
__global__ __launch_bounds__(256) void split_log2norm_kernel(const float* __restrict__ sq, int n,
                                                             float* __restrict__ r) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) r[i] = split_log2norm(sq[i]);
}

// ---------------------------------------------------------------------------
// Persistent LDS-DMA STORE GEMM: the LDS-DMA kernel's k loop, one 512-thread
// workgroup per CU walking tiles as the persistent kernel does, so that a
// tile's Gram stores (128 KiB per tile with the mirror: 4.2 of the tile
// kernel's 13.6 ms, profiles/r3_split_gemm_headline_ab.txt) drain while the
// next tile multiplies.  Order at a tile boundary: the next tile's row data
// (plain loads, issued while no DMA is in flight), the epilogue math, a
// barrier, the next tile's first three DMAs, THEN this tile's stores — so the
// next tile's first three waits count the stores as younger than their DMA:
// vmcnt(8 + S) with S the store instructions each lane issued (interior tiles:
// exactly 32 direct + 8 mirrored, unpredicated; edge tiles store predicated and
// drain with vmcnt(0)).  From block 3 on the stores are older than the block's
// DMA and vmcnt(8) retires them too.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kGldsThreads, 1) void rbf_gemm_split_glds_persist_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq, int64_t M,
    const u4* __restrict__ B, const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int64_t N, int nkb,
    float gamma, float* __restrict__ out, int64_t ldo, int sym, int tm, int tn) {
  constexpr int WN = 2, TM = 128, TN = 128, ROWS = TM + TN, CPR = 8, BUF = ROWS * CPR, NB = 4;
  __shared__ u4 lds[NB * BUF + 4 * ROWS / 4];  // 4 operand buffers, then per tile parity |x|^2 [ROWS], shifts [ROWS]
  float* s_sq0 = (float*)(lds + NB * BUF);
  int32_t* s_sh0 = (int32_t*)(lds + NB * BUF) + 2 * ROWS;

  const int total = tm * tn, G = gridDim.x;
  auto valid = [&](int L, int& x, int& y) {
    xcd_tile_of32(L, tm, tn, x, y);
    return !(sym && y < x);
  };
  int tx = 0, ty = 0, L = blockIdx.x;
  while (L < total && !valid(L, tx, ty)) L += G;
  if (L >= total) return;  // uniform: no barrier reached

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const int64_t rstride = (int64_t)nkb * 8;
  int64_t m0 = (int64_t)tx * TM, n0 = (int64_t)ty * TN;

  // DMA geometry (as rbf_gemm_split_glds_kernel): row 32 w + 8 i + (lane >> 3)
  int srow[4], schunk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    srow[i] = 32 * wave + 8 * i + (lane >> 3);
    schunk[i] = (lane & 7) ^ ((srow[i] >> 1) & 7);
  }
  const u4* src[4];
  auto set_src = [&](int64_t a0, int64_t b0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      src[i] = srow[i] < TM ? A + (a0 + srow[i]) * rstride + schunk[i] : B + (b0 + (srow[i] - TM)) * rstride + schunk[i];
  };
  auto dma = [&](int kb) {
    u4* dst = lds + (kb & (NB - 1)) * BUF + 32 * wave * CPR;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + (int64_t)kb * 8),
                                       (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, 0);
  };
  auto row_data = [&](int64_t a0, int64_t b0, float& q, int32_t& h) {
    if (tid < ROWS) {
      const int64_t ri = tid < TM ? min(a0 + tid, M - 1) : min(b0 + (tid - TM), N - 1);
      q = tid < TM ? Asq[ri] : Bsq[ri];
      h = tid < TM ? Ash[ri] : Bsh[ri];
    }
  };
  {
    float q = 0.f;
    int32_t h = 0;
    row_data(m0, n0, q, h);
    if (tid < ROWS) {
      s_sq0[tid] = q;
      s_sh0[tid] = h;
    }
  }
  __syncthreads();  // row data of tile 0 (no DMA in flight yet)
  set_src(m0, n0);
  dma(0);
  if (nkb > 1) dma(1);
  if (nkb > 2) dma(2);

  const int sw = ((lane & 31) >> 1) & 7;
  const int ra = (wm * 32 + (lane & 31)) * CPR;
  const int rb0 = (TM + wn * 64 + (lane & 31)) * CPR, rb1 = rb0 + 32 * CPR;
  int par = 0;
  int pend = 0;  // store instructions each lane issued after the current tile's first DMAs (0, 32 or 40)
  f16v H[2], P[2], Q[2];
  while (true) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) H[j][r] = P[j][r] = Q[j][r] = 0.f;
    for (int kb = 0; kb < nkb; ++kb) {
      const int ahead = min(2, nkb - 1 - kb);
      // the previous tile's stores sit between the DMAs of blocks 2 and 3
      const int st = kb < 3 ? pend : 0;
      if (ahead == 2) {
        if (st == 40) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
        else if (st == 32) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else if (ahead == 1) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // never with pending stores: nkb >= 5 (launcher)
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kb + 3 < nkb) dma(kb + 3);
      const u4* buf = lds + (kb & (NB - 1)) * BUF;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = (2 * ks + hl) ^ sw, cl = (4 + 2 * ks + hl) ^ sw;
        const h8 ah = __builtin_bit_cast(h8, buf[ra + ch]);
        const h8 al = __builtin_bit_cast(h8, buf[ra + cl]);
        const h8 bh0 = __builtin_bit_cast(h8, buf[rb0 + ch]);
        const h8 bl0 = __builtin_bit_cast(h8, buf[rb0 + cl]);
        const h8 bh1 = __builtin_bit_cast(h8, buf[rb1 + ch]);
        const h8 bl1 = __builtin_bit_cast(h8, buf[rb1 + cl]);
        H[0] = mfma32_f16(ah, bh0, H[0]);
        H[1] = mfma32_f16(ah, bh1, H[1]);
        P[0] = mfma32_f16(ah, bl0, P[0]);
        P[1] = mfma32_f16(ah, bl1, P[1]);
        Q[0] = mfma32_f16(al, bh0, Q[0]);
        Q[1] = mfma32_f16(al, bh1, Q[1]);
      }
    }
    // ---- tile boundary (no DMA in flight: the last block waited vmcnt(0)) ----
    int nL = L + G, ntx = tx, nty = ty;
    while (nL < total && !valid(nL, ntx, nty)) nL += G;
    const bool has_next = nL < total;
    const int64_t nm0 = (int64_t)ntx * TM, nn0 = (int64_t)nty * TN;
    float nq = 0.f;
    int32_t nh = 0;
    if (has_next) row_data(nm0, nn0, nq, nh);
    const float* s_sq = s_sq0 + par * ROWS;
    const int32_t* s_sh = s_sh0 + par * ROWS;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cb = TM + wn * 64 + 32 * j + (lane & 31);
      const float bsq = s_sq[cb];
      const int bsh = s_sh[cb];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const float dot = ldexpf(H[j][r] + (P[j][r] + Q[j][r]), -(s_sh[lr] + bsh));
        H[j][r] = rbf_split_value(s_sq[lr], bsq, dot, gamma);
      }
    }
    if (has_next && tid < ROWS) {
      s_sq0[(par ^ 1) * ROWS + tid] = nq;
      s_sh0[(par ^ 1) * ROWS + tid] = nh;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done with the operand buffers of this tile
    asm volatile("" ::: "memory");
    if (has_next) {
      set_src(nm0, nn0);
      dma(0);
      dma(1);
      dma(2);
    }
    asm volatile("" ::: "memory");  // the stores stay behind the DMAs
    const bool interior = m0 + TM <= M && n0 + TN <= N;
    const bool mirror = sym && ty != tx;
    if (interior) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
        for (int j = 0; j < 2; ++j) out[row * ldo + n0 + wn * 64 + 32 * j + (lane & 31)] = H[j][r];
      }
      if (mirror) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f4 v;
            v.x = H[j][4 * q + 0];
            v.y = H[j][4 * q + 1];
            v.z = H[j][4 * q + 2];
            v.w = H[j][4 * q + 3];
            *(f4*)(out + col * ldo + m0 + wm * 32 + 8 * q + 4 * hl) = v;
          }
        }
      }
      pend = mirror ? 40 : 32;
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
          if (row < M && col < N) out[row * ldo + col] = H[j][r];
        }
      }
      if (mirror) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int64_t row = m0 + wm * 32 + 8 * q + 4 * hl;
            float* dst = out + col * ldo + row;
            if (col < M) {
#pragma unroll
              for (int c = 0; c < 4; ++c)
                if (row + c < N) dst[c] = H[j][4 * q + c];
            }
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // predicated stores: drained here
      pend = 0;
    }
    if (!has_next) break;
    L = nL;
    tx = ntx;
    ty = nty;
    m0 = nm0;
    n0 = nn0;
    par ^= 1;
  }
}

// ---------------------------------------------------------------------------
// Decision GEMM on split operands (predict: training accuracy, GpuPredictor,
// svmTest, the shrinking phases' gradient update): dec_i = sum_j coef_j K(A_i,
// B_j) with A = query rows, B = support vectors.  A workgroup owns 128 query
// rows and a range of SV tiles; the (SV tile, k block) sequence is ONE LDS-DMA
// pipeline (the LDS-DMA STORE kernel's staging: four 32-k buffers, three blocks
// in flight across tile boundaries — the query panel is the same for every SV
// tile), and each SV tile's 128 x 128 kernel block is folded into per-row sums
// in registers (no store).  Partial sums per SV split: partial[split][row].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kGldsThreads, 1) void rbf_predict_split_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq, int64_t M,
    const u4* __restrict__ B, const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq,
    const float* __restrict__ coef, int64_t N, int nkb, float gamma, float* __restrict__ partial, int64_t ldp,
    int per) {
  constexpr int WN = 2, TM = 128, TN = 128, ROWS = TM + TN, CPR = 8, BUF = ROWS * CPR, NB = 4;
  __shared__ u4 lds[NB * BUF + 2 * TM / 4];
  float* s_asq = (float*)(lds + NB * BUF);
  int32_t* s_ash = (int32_t*)(lds + NB * BUF) + TM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN, hl = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * TM;
  const int64_t tn_all = (N + TN - 1) / TN;
  const int64_t t0 = (int64_t)blockIdx.y * per, t1 = min(t0 + per, tn_all);
  float* out = partial + (int64_t)blockIdx.y * ldp + m0;
  if (t0 >= t1) {  // uniform: an empty split contributes zeros
    if (tid < TM) out[tid] = 0.f;
    return;
  }
  const int64_t rstride = (int64_t)nkb * 8;
  if (tid < TM) {
    const int64_t ri = min(m0 + tid, M - 1);
    s_asq[tid] = Asq[ri];
    s_ash[tid] = Ash[ri];
  }
  const u4* src[4];
  bool isb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 32 * wave + 8 * i + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    isb[i] = r >= TM;
    src[i] = r < TM ? A + (m0 + r) * rstride + c : B + (t0 * TN + (r - TM)) * rstride + c;
  }
  const int64_t nblk = (t1 - t0) * nkb;
  auto dma = [&](int64_t g) {
    const int64_t t = g / nkb, kb = g - t * nkb;
    u4* dst = lds + (g & (NB - 1)) * BUF + 32 * wave * CPR;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void*)(src[i] + (isb[i] ? t * TN * rstride : 0) + kb * 8),
          (__attribute__((address_space(3))) void*)(dst + 8 * i * CPR), 16, 0, 0);
  };
  __syncthreads();
  dma(0);
  if (nblk > 1) dma(1);
  if (nblk > 2) dma(2);

  f16v H[2], P[2], Q[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) H[j][r] = P[j][r] = Q[j][r] = 0.f;
  float acc[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int sw = ((lane & 31) >> 1) & 7;
  const int ra = (wm * 32 + (lane & 31)) * CPR;
  const int rb0 = (TM + wn * 64 + (lane & 31)) * CPR, rb1 = rb0 + 32 * CPR;
  int kb = 0;
  int64_t t = t0;
  for (int64_t g = 0; g < nblk; ++g) {
    const int64_t ahead = min((int64_t)2, nblk - 1 - g);
    if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (g + 3 < nblk) dma(g + 3);
    const u4* buf = lds + (g & (NB - 1)) * BUF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = (2 * ks + hl) ^ sw, cl = (4 + 2 * ks + hl) ^ sw;
      const h8 ah = __builtin_bit_cast(h8, buf[ra + ch]);
      const h8 al = __builtin_bit_cast(h8, buf[ra + cl]);
      const h8 bh0 = __builtin_bit_cast(h8, buf[rb0 + ch]);
      const h8 bl0 = __builtin_bit_cast(h8, buf[rb0 + cl]);
      const h8 bh1 = __builtin_bit_cast(h8, buf[rb1 + ch]);
      const h8 bl1 = __builtin_bit_cast(h8, buf[rb1 + cl]);
      H[0] = mfma32_f16(ah, bh0, H[0]);
      H[1] = mfma32_f16(ah, bh1, H[1]);
      P[0] = mfma32_f16(ah, bl0, P[0]);
      P[1] = mfma32_f16(ah, bl1, P[1]);
      Q[0] = mfma32_f16(al, bh0, Q[0]);
      Q[1] = mfma32_f16(al, bh1, Q[1]);
    }
    if (++kb == nkb) {  // the SV tile is complete: fold its kernel block into the row sums
      const int64_t n0 = t * TN;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t col = n0 + wn * 64 + 32 * j + (lane & 31);
        const int64_t cc = col < N ? col : N - 1;
        const float cf = col < N ? coef[cc] : 0.f;
        const float bsq = Bsq[cc];
        const int bsh = Bsh[cc];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          const float dot = ldexpf(H[j][r] + (P[j][r] + Q[j][r]), -(s_ash[lr] + bsh));
          acc[r] += cf * rbf_split_value(s_asq[lr], bsq, dot, gamma);
          H[j][r] = P[j][r] = Q[j][r] = 0.f;
        }
      }
      kb = 0;
      ++t;
    }
  }
  // the 32 columns of a lane group, then the two column waves through LDS
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = acc[r];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    acc[r] = v;
  }
  __syncthreads();  // every wave is past its last operand read (no DMA in flight)
  float* red = (float*)lds;  // [WN][TM]
  if ((lane & 31) == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wn * TM + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl] = acc[r];
  }
  __syncthreads();
  if (tid < TM) out[tid] = red[tid] + red[TM + tid];
}

}  // namespace dev

namespace launch {

namespace {
int g_split_variant = -1;
}

int split_gemm_variant() {
  if (g_split_variant < 0) {
    const char* e = std::getenv("DPSVM_SPLIT_GEMM");  // A/B: 1 tile kernel, 3 LDS-DMA, 4 persistent LDS-DMA, 5 wide-wave
    g_split_variant = e ? atoi(e) : 0;
  }
  return g_split_variant;
}

void set_split_gemm_variant(int v) { g_split_variant = v; }

// diagnostics: non-null = the wide-wave Gram kernel writes per-workgroup stamps here
uint64_t* g_gram_stamps = nullptr;
// diagnostics: non-null = the LDS-DMA rows kernel writes per-workgroup stamps here
uint64_t* g_rows_stamps = nullptr;
void set_rows_stamps(uint64_t* p) { g_rows_stamps = p; }

void set_gram_stamps(uint64_t* p) { g_gram_stamps = p; }

int64_t split_row_u4(int dp) { return (int64_t)((dp + 31) / 32) * 8; }

void rbf_predict_split(const float* A, const float* Asq, int64_t M, int lda, const float* B, const float* Bsq,
                       const float* coef, int64_t N, int ldb, int dp, float gamma, float* partial, int64_t ldp,
                       int max_splits, hipStream_t s) {
  // both operands split into stream-ordered scratch (rows padded: the kernel reads whole 128-row tiles)
  const int nkb = (dp + 31) / 32;
  const int64_t pa = split_pad_rows(M), pb = split_pad_rows(N), ru = split_row_u4(dp) * 16;
  void *a_pl = nullptr, *b_pl = nullptr;
  int32_t *a_sh = nullptr, *b_sh = nullptr;
  HIP_CHECK(hipMallocAsync(&a_pl, (size_t)(pa * ru), s));
  HIP_CHECK(hipMallocAsync(&b_pl, (size_t)(pb * ru), s));
  HIP_CHECK(hipMallocAsync((void**)&a_sh, (size_t)pa * 4, s));
  HIP_CHECK(hipMallocAsync((void**)&b_sh, (size_t)pb * 4, s));
  HIP_CHECK(hipMemsetAsync(a_pl, 0, (size_t)(pa * ru), s));
  HIP_CHECK(hipMemsetAsync(b_pl, 0, (size_t)(pb * ru), s));
  HIP_CHECK(hipMemsetAsync(a_sh, 0, (size_t)pa * 4, s));
  HIP_CHECK(hipMemsetAsync(b_sh, 0, (size_t)pb * 4, s));
  split_rows_f16(A, M, dp, lda, a_pl, a_sh, s);
  split_rows_f16(B, N, dp, ldb, b_pl, b_sh, s);
  const int64_t tm = (M + 127) / 128, tn = (N + 127) / 128;
  // ~2 workgroups per CU of a 256-CU device, at most the scratch's splits
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>({(int64_t)max_splits, tn, (512 + tm - 1) / tm}));
  const int per = (int)((tn + splits - 1) / splits);
  splits = (tn + per - 1) / per;
  dev::rbf_predict_split_kernel<<<dim3((unsigned)tm, (unsigned)splits), dev::kGldsThreads, 0, s>>>(
      (const dev::u4*)a_pl, a_sh, Asq, M, (const dev::u4*)b_pl, b_sh, Bsq, coef, N, nkb, gamma, partial, ldp, per);
  post_launch("rbf_predict_split", s);
  // zero the splits the reduce reads beyond the launched ones
  if (splits < max_splits)
    HIP_CHECK(hipMemsetAsync(partial + splits * ldp, 0, (size_t)(max_splits - splits) * ldp * 4, s));
  HIP_CHECK(hipFreeAsync(a_pl, s));
  HIP_CHECK(hipFreeAsync(b_pl, s));
  HIP_CHECK(hipFreeAsync(a_sh, s));
  HIP_CHECK(hipFreeAsync(b_sh, s));
}

int64_t split_pad_rows(int64_t rows) { return (rows + 255) / 256 * 256 + 256; }

void split_rows_f16(const float* x, int64_t rows, int dp, int ldx, void* out, int32_t* shift, hipStream_t s) {
  if (rows <= 0) return;
  const int nkb = (dp + 31) / 32;
  dev::split_rows_kernel<<<dim3((unsigned)((rows + 3) / 4)), 256, 0, s>>>(x, rows, dp, ldx, (dev::u4*)out, shift,
                                                                          nkb);
  post_launch("split_rows_f16", s);
}

namespace {
// The symmetric Gram's upper tiles of the 256 x 128 wide-wave kernel (tile
// (tx, ty) is needed when ty >= 2 tx) as a compact table in an XCD order
// (chunks of CH tiles of GM tile rows dealt round-robin to the 8 XCDs, as
// xcd_tile_of does with 64 / 8): built once per shape on the host, kept on the device.  The full grid
// launched tm x tn workgroups of which half exited at once (55k of 110k on
// the headline).
struct TileTable {
  uint32_t* dev = nullptr;
  int64_t count = 0;
};
// Keyed by (device, tm, tn): the table lives in the memory of the device that
// launches the GEMM (svmTrain -p N: one rank per device, threads of one process).
// gm / ch > 0: that grouping instead of the default (the one-product pass: 8 / 64,
// 6.73-6.93 vs 7.03-7.10 ms for 4 / 32, profiles/r6_gram_adapt/h1_tile_order_sweep.txt)
const TileTable& sym_tile_table(int64_t tm, int64_t tn, hipStream_t s, bool sym = true, int gm = 0, int ch = 0) {
  static std::mutex mu;
  static std::map<std::tuple<int, int64_t, int64_t, bool, int, int>, TileTable> cache;
  const int device = current_device();
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({device, tm, tn, sym, gm, ch});
  if (it != cache.end()) return it->second;
  // the needed tiles in groups of GM tile rows, column by column, rows inside a
  // column; chunks of CH consecutive tiles dealt round-robin to the 8 XCDs.
  // GM 4 / CH 32 (an XCD's chunk: 4 A panels x 8 B panels) 9.34-9.45 ms vs
  // 9.47-9.50 for GM 8 / CH 64 (profiles/r5_gram_tile_order_ab.txt; bit-identical
  // output).  A/B: DPSVM_GRAM_GM / DPSVM_GRAM_CH
  std::vector<uint32_t> order;
  static const int64_t GM_env = [] {
    const char* e = std::getenv("DPSVM_GRAM_GM");
    const int v = e ? atoi(e) : 4;
    return (int64_t)(v >= 1 && v <= 64 ? v : 4);
  }();
  static const int64_t CH_env = [] {
    const char* e = std::getenv("DPSVM_GRAM_CH");
    const int v = e ? atoi(e) : 32;
    return (int64_t)(v >= 8 && v <= 1024 ? v : 32);
  }();
  const int64_t GM = gm > 0 ? gm : GM_env, CH = ch > 0 ? ch : CH_env;
  for (int64_t g0 = 0; g0 < tm; g0 += GM) {
    const int64_t gm = std::min(GM, tm - g0);
    for (int64_t ty = 0; ty < tn; ++ty)
      for (int64_t tx = g0; tx < g0 + gm; ++tx)
        if (!sym || ty >= 2 * tx) order.push_back((uint32_t)((tx << 16) | ty));
  }
  const int64_t total = (int64_t)order.size(), full = total / (8 * CH) * (8 * CH);
  std::vector<uint32_t> tab((size_t)total);
  for (int64_t L = 0; L < total; ++L) {  // workgroup L runs on XCD L % 8: XCD x takes chunks x, x + 8, ...
    int64_t T = L;
    if (L < full) {
      const int64_t xcd = L % 8, local = L / 8;
      T = ((local / CH) * 8 + xcd) * CH + local % CH;
    }
    tab[(size_t)L] = order[(size_t)T];
  }
  TileTable t;
  t.count = total;
  HIP_CHECK(hipMalloc((void**)&t.dev, (size_t)total * sizeof(uint32_t)));
  HIP_CHECK(hipMemcpyAsync(t.dev, tab.data(), (size_t)total * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return cache.emplace(std::make_tuple(device, tm, tn, sym, gm, ch), t).first->second;
}
}  // namespace

// split_cold's constants: E = e |a| |b| with e = 4.5 2^-11 gamma bounds gamma times the one- vs
// three-product d^2 difference; cold iff R_i + R_j <= c1 (E <= 1) and t1 <= c0 - (R_i + R_j)
// (1.72 K1 E <= tau, e^E - 1 <= 1.72 E for E <= 1), c0 with a 0.01 (0.7%) margin in log2
void split_cold_consts(float gamma, float tau, float* c0, float* c1) {
  const double e = 4.5 * std::ldexp(1.0, -11) * (double)gamma;
  *c1 = (float)(-std::log2(e));
  *c0 = (float)(std::log2((double)tau) - std::log2(1.72 * e) - 0.01);
}

namespace {
// the calling thread's last adaptive Gram (svmTrain -p N: one rank per thread)
thread_local int64_t t_adapt_tiles = -1;
thread_local uint32_t* t_adapt_hot = nullptr;  // pinned: the hot-tile count, copied after pass 1
}  // namespace

void gram_adapt_last(int64_t* tiles, int64_t* hot) {
  *tiles = t_adapt_tiles;
  *hot = t_adapt_tiles >= 0 && t_adapt_hot ? (int64_t)*(volatile uint32_t*)t_adapt_hot : -1;
}

void rbf_gemm_store_split(const void* A, const int32_t* Ash, const float* Asq, int64_t M, const void* B,
                          const int32_t* Bsh, const float* Bsq, int64_t N, int dp, float gamma, float* out,
                          int64_t ldo, hipStream_t s, bool symmetric, float cold_tau) {
  t_adapt_tiles = -1;
  if (M <= 0 || N <= 0) return;
  DPSVM_CHECK(!symmetric || (A == B && Asq == Bsq && Ash == Bsh && M == N && ldo % 4 == 0),
              "rbf_gemm_store_split: symmetric mode needs B == A, N == M");
  const int64_t tm = (M + 127) / 128, tn = (N + 127) / 128;
  DPSVM_CHECK(tn < 65536, "rbf_gemm_store_split: N too large for grid.y");
  static const int ablate = [] {
    const char* e = std::getenv("DPSVM_SPLIT_ABLATE");  // diagnostics (bench/gram_ab.py)
    return e ? atoi(e) : 0;
  }();
  static const int kb = [] {
    const char* e = std::getenv("DPSVM_SPLIT_KB");  // diagnostics: k blocks per stage (A/B)
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  const int variant = split_gemm_variant();
  // default from 5 k blocks: the wide-wave LDS-DMA kernel (60000^2 x 784
  // symmetric: 10.1-10.8 ms vs 10.9-11.1 for the persistent LDS-DMA kernel,
  // bit-identical; profiles/r4_w64_gram_ab.txt)
  // (32-bit store offsets inside a 256 x 128 tile: ldo < 2^24)
  if ((variant == 5 || variant == 6 || variant == 7 || variant == 8 || variant == 11 || variant == 12 || (variant == 0 && (dp + 31) / 32 >= 5)) && ablate == 0 &&
      ldo < (1ll << 24)) {
    static const int nt = [] {
      const char* e = std::getenv("DPSVM_GRAM_NT");  // A/B: 0 plain Gram stores, 1 non-temporal, 2 none (diagnostics)
      return e ? atoi(e) : 0;
    }();
    const int64_t tm2 = (M + 255) / 256;
    // Defaults, each bit-identical to the others (profiles/r6_gram_lds_readahead_ab.json):
    //  - the LDS-DMA issue spread over the MFMA groups (9.41 -> 9.27 ms symmetric)
    //    with the operand reads one MFMA group ahead (-> 8.81-8.93 ms);
    //  - the packed-f32 / buffer-store epilogue (13.4k -> 10.0k cycles a tile);
    //  - persistent over the tiles (below): 9.01 -> 8.86 ms symmetric, 2.47 -> 2.30 ms
    //    for the P = 8 slab against the tile-per-workgroup kernel of the same tree.
    // A/B: variants 5 (no spread), 6 (spread), 8 (spread + read-ahead), 11 (+ PE),
    // 7 / 12 persistent without / with PE; DPSVM_GRAM_SPREAD=0, DPSVM_GRAM_PERSIST=0
    static const int spread = [] {
      const char* e = std::getenv("DPSVM_GRAM_SPREAD");
      return e ? atoi(e) : 1;
    }();
    const int sp = variant == 5 ? 0 : variant == 6 ? 1 : variant == 8 || variant == 11 ? 2 : spread ? 2 : 0;
    const bool pe = variant == 11 || variant == 12 || (variant == 0 && spread);
    auto kern = g_gram_stamps ? (pe        ? dev::rbf_gemm_split_w64_kernel<3, 2, true>
                                 : sp == 2 ? dev::rbf_gemm_split_w64_kernel<3, 2>
                                           : dev::rbf_gemm_split_w64_kernel<3, 1>)
                : nt == 2 ? dev::rbf_gemm_split_w64_kernel<2>
                : nt      ? dev::rbf_gemm_split_w64_kernel<1>
                : pe      ? dev::rbf_gemm_split_w64_kernel<0, 2, true>
                : sp == 2 ? dev::rbf_gemm_split_w64_kernel<0, 2>
                : sp == 1 ? dev::rbf_gemm_split_w64_kernel<0, 1>
                          : dev::rbf_gemm_split_w64_kernel<0>;
    static const bool compact = [] {  // A/B: DPSVM_GRAM_COMPACT=0 launches the full grid (half exit at once)
      const char* e = std::getenv("DPSVM_GRAM_COMPACT");
      return !(e && e[0] == '0');
    }();
    // persistent over the tiles (the default; variants 7 / 12; A/B:
    // DPSVM_GRAM_PERSIST=0): one workgroup per CU, the LDS-DMA ring running on
    // across tiles
    static const int persist_env = [] {
      const char* e = std::getenv("DPSVM_GRAM_PERSIST");
      return e ? atoi(e) : 1;
    }();
    const int nkb = (dp + 31) / 32;
    // (32-bit indices: the split operand buffers hold (rows + 512) x nkb x 8 u4, the output M x ldo floats)
    const bool idx32 = (M + 512) * (int64_t)nkb * 8 < (1ll << 31) && (N + 512) * (int64_t)nkb * 8 < (1ll << 31) &&
                       M * ldo < (1ll << 32) && N * ldo < (1ll << 32);
    const bool persist = (variant == 7 || variant == 12 || (variant == 0 && persist_env == 1 && spread)) && nkb >= 3 && nt == 0 && idx32 &&
                         tm2 < 65536 && tn < 65536 && (!symmetric || compact);
    // the adaptive Gram's kernels (h1s, w64p with the packed epilogue) index a tile's stores from
    // 64-bit tile bases with 32-bit offsets (256 rows x ldo x 4 B < 2^32) and the operand rows in
    // 32 bits: they also take Grams of more than 2^32 elements (200k rows: 160 GB)
    const bool idx_adapt = (M + 512) * (int64_t)nkb * 8 < (1ll << 31) && (N + 512) * (int64_t)nkb * 8 < (1ll << 31) &&
                           ldo < (1ll << 22);
    const bool adapt = pe && cold_tau > 0.f && gamma > 0.f && nkb >= 5 && !g_gram_stamps && nt == 0 && idx_adapt &&
                       tm2 < 65536 && tn < 65536 && (!symmetric || compact) &&
                       (variant == 0 || variant == 7 || variant == 12);
    if (persist || adapt) {
      const int cus = [] {
        int n = 0;
        HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, current_device()));
        return std::max(8, n);
      }();
      const auto& t = sym_tile_table(tm2, tn, s, symmetric);  // non-symmetric: every tile, same XCD order
      const uint32_t* tab = t.dev;
      const int64_t ntiles = t.count;
      const int64_t grid = std::min<int64_t>(ntiles, cus);
      if (adapt) {
        static const bool h1_order = [] {  // A/B: DPSVM_H1_ORDER=0 keeps the three-product kernel's grouping
          const char* e = std::getenv("DPSVM_H1_ORDER");
          return !(e && e[0] == '0') && !std::getenv("DPSVM_GRAM_GM") && !std::getenv("DPSVM_GRAM_CH");
        }();
        const auto& t1 = h1_order ? sym_tile_table(tm2, tn, s, symmetric, 8, 64) : t;
        // adaptive: pass 1 one-product over every tile, pass 2 three products over the reported ones
        float c0 = 0.f, c1 = 0.f;
        split_cold_consts(gamma, cold_tau, &c0, &c1);
        const int64_t nr = symmetric ? M : M + N;
        float* r = nullptr;
        uint32_t* hb = nullptr;  // [ntiles] per-tile reports, then the list's length and entries
        HIP_CHECK(hipMallocAsync((void**)&r, (size_t)nr * 4, s));
        HIP_CHECK(hipMallocAsync((void**)&hb, (size_t)(2 * ntiles + 1) * 4, s));
        HIP_CHECK(hipMemsetAsync(hb, 0, (size_t)(ntiles + 1) * 4, s));
        dev::split_log2norm_kernel<<<dim3((unsigned)((M + 255) / 256)), 256, 0, s>>>(Asq, (int)M, r);
        float* br = r;
        if (!symmetric) {
          br = r + M;
          dev::split_log2norm_kernel<<<dim3((unsigned)((N + 255) / 256)), 256, 0, s>>>(Bsq, (int)N, br);
        }
        post_launch("split_log2norm", s);
        static const int h1_abl = [] {  // diagnostics (bench/gram_adapt_probe.py): h1 pass ablations
          const char* e = std::getenv("DPSVM_H1_ABLATE");
          return e ? atoi(e) : 0;
        }();
        const void *hA = A, *hB = B;
        dev::u4* planes = nullptr;
        {  // the h planes of the rows the tiles read (whole 256 / 128-row tiles)
          const int64_t nq = (int64_t)((nkb + 1) / 2) * 8, ra = tm2 * 256, rb = symmetric ? 0 : tn * 128;
          HIP_CHECK(hipMallocAsync((void**)&planes, (size_t)(ra + rb) * nq * 16, s));
          dev::split_hplane_kernel<<<dim3((unsigned)((ra * nq + 255) / 256)), 256, 0, s>>>((const dev::u4*)A, ra,
                                                                                            nkb, planes);
          hA = hB = planes;
          if (!symmetric) {
            dev::split_hplane_kernel<<<dim3((unsigned)((rb * nq + 255) / 256)), 256, 0, s>>>((const dev::u4*)B, rb,
                                                                                              nkb, planes + ra * nq);
            hB = planes + ra * nq;
          }
          post_launch("split_hplane", s);
        }
        auto h1k = h1_abl == 1   ? dev::rbf_gemm_split_h1s_kernel<1>
                   : h1_abl == 2 ? dev::rbf_gemm_split_h1s_kernel<2>
                   : h1_abl == 3 ? dev::rbf_gemm_split_h1s_kernel<3>
                   : h1_abl == 4 ? dev::rbf_gemm_split_h1s_kernel<4>
                                 : dev::rbf_gemm_split_h1s_kernel<0>;
        h1k<<<dim3((unsigned)grid), dev::kH1sThreads, 0, s>>>(
            (const dev::u4*)hA, Ash, Asq, r, (int)M, (const dev::u4*)hB, Bsh, Bsq, br, (int)N, nkb, gamma, c0, c1, out,
            (int)ldo, symmetric ? 1 : 0, t1.dev, (int)ntiles, hb, hb + ntiles);
        if (planes) HIP_CHECK(hipFreeAsync(planes, s));
        post_launch("rbf_gemm_split_h1", s);
        dev::rbf_gemm_split_w64p_kernel<0, true, true><<<dim3((unsigned)grid), dev::kW64Threads, 0, s>>>(
            (const dev::u4*)A, Ash, Asq, (int)M, (const dev::u4*)B, Bsh, Bsq, (int)N, nkb, gamma, out, (int)ldo,
            symmetric ? 1 : 0, hb + ntiles + 1, 0, (int)tm2, (int)tn, nullptr, r, br, c0, c1, hb + ntiles);
        post_launch("rbf_gemm_split_w64p_hot", s);
        if (!t_adapt_hot) HIP_CHECK(hipHostMalloc((void**)&t_adapt_hot, 4, hipHostMallocDefault));
        HIP_CHECK(hipMemcpyAsync(t_adapt_hot, hb + ntiles, 4, hipMemcpyDeviceToHost, s));
        t_adapt_tiles = ntiles;
        HIP_CHECK(hipFreeAsync(r, s));
        HIP_CHECK(hipFreeAsync(hb, s));
        return;
      }
      auto pk = g_gram_stamps ? (pe ? dev::rbf_gemm_split_w64p_kernel<3, true> : dev::rbf_gemm_split_w64p_kernel<3>)
                : pe ? dev::rbf_gemm_split_w64p_kernel<0, true> : dev::rbf_gemm_split_w64p_kernel<0>;
      pk<<<dim3((unsigned)grid), dev::kW64Threads, 0, s>>>((const dev::u4*)A, Ash, Asq, (int)M, (const dev::u4*)B,
                                                          Bsh, Bsq, (int)N, nkb, gamma, out, (int)ldo,
                                                          symmetric ? 1 : 0, tab, (int)ntiles, (int)tm2, (int)tn,
                                                          g_gram_stamps, nullptr, nullptr, 0.f, 0.f, nullptr);
      post_launch("rbf_gemm_split_w64p", s);
      return;
    }
    if (symmetric && compact && tm2 < 65536 && tn < 65536) {
      const auto& tab = sym_tile_table(tm2, tn, s);
      kern<<<dim3((unsigned)tab.count), dev::kW64Threads, 0, s>>>(
          (const dev::u4*)A, Ash, Asq, M, (const dev::u4*)B, Bsh, Bsq, N, (dp + 31) / 32, gamma, out, ldo, 1, tab.dev,
          g_gram_stamps);
    } else {
      kern<<<dim3((unsigned)tm2, (unsigned)tn), dev::kW64Threads, 0, s>>>(
          (const dev::u4*)A, Ash, Asq, M, (const dev::u4*)B, Bsh, Bsq, N, (dp + 31) / 32, gamma, out, ldo,
          symmetric ? 1 : 0, nullptr, g_gram_stamps);
    }
    post_launch("rbf_gemm_split_w64", s);
    return;
  }
  if ((variant == 0 || variant == 4) && ablate == 0 && (dp + 31) / 32 >= 5 && tm * tn < (1ll << 31)) {
    // default: persistent LDS-DMA, one workgroup per CU (a multiple of 8)
    static const int cus4 = [] {
      int dev = 0, n = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return std::max(8, n / 8 * 8);
    }();
    const int64_t tiles = symmetric ? tm * (tm + 1) / 2 : tm * tn;
    const int grid = (int)std::min<int64_t>(cus4, (tiles + 7) / 8 * 8);
    dev::rbf_gemm_split_glds_persist_kernel<<<dim3((unsigned)grid), dev::kGldsThreads, 0, s>>>(
        (const dev::u4*)A, Ash, Asq, M, (const dev::u4*)B, Bsh, Bsq, N, (dp + 31) / 32, gamma, out, ldo,
        symmetric ? 1 : 0, (int)tm, (int)tn);
    post_launch("rbf_gemm_split_glds_persist", s);
    return;
  }
  if ((variant == 0 || variant == 3) && ablate == 0 && kb == 2) {  // LDS-DMA, three k blocks in flight (dp <= 128 by default)
    dev::rbf_gemm_split_glds_kernel<<<dim3((unsigned)tm, (unsigned)tn), dev::kGldsThreads, 0, s>>>(
        (const dev::u4*)A, Ash, Asq, M, (const dev::u4*)B, Bsh, Bsq, N, (dp + 31) / 32, gamma, out, ldo,
        symmetric ? 1 : 0);
    post_launch("rbf_gemm_split_glds", s);
    return;
  }
  auto kern = kb == 1 ? dev::rbf_gemm_split_kernel<dev::SPLIT_STORE, 4, 1, 0>
              : ablate == 1 ? dev::rbf_gemm_split_kernel<dev::SPLIT_STORE, 4, 2, 1>
              : ablate == 2 ? dev::rbf_gemm_split_kernel<dev::SPLIT_STORE, 4, 2, 2>
                            : dev::rbf_gemm_split_kernel<dev::SPLIT_STORE, 4, 2, 0>;
  kern<<<dim3((unsigned)tm, (unsigned)tn), dev::kSplitThreads, 0, s>>>(
      (const dev::u4*)A, Ash, Asq, M, (const dev::u4*)B, Bsh, Bsq, N, (dp + 31) / 32, gamma, out, ldo,
      symmetric ? 1 : 0, nullptr, nullptr, nullptr);
  post_launch("rbf_gemm_store_split", s);
}

void rbf_rows_indexed_split(const void* X, const int32_t* Xsh, const float* Xsq, const int32_t* a_rows,
                            const int32_t* m_dev, int64_t M_max, const void* B, const int32_t* Bsh, const float* Bsq,
                            int64_t N, int dp, float gamma, float* lines, const int32_t* out_rows, int64_t ldl,
                            hipStream_t s) {
  if (M_max <= 0 || N <= 0) return;
  // 192 x 128 tiles (12 waves): a one-block round's misses (<= 192 rows) are
  // one tile row, so every column panel of B — all of this rank's rows, the
  // bytes that bound this GEMM — is read from HBM once per round (64-row
  // tiles read it once per 64 misses)
  const int64_t tm = (M_max + 191) / 192, tn = (N + 127) / 128;
  DPSVM_CHECK(tn < 65536, "rbf_rows_indexed_split: N too large for grid.y");
  static const bool reg_staged = [] {  // A/B: DPSVM_ROWS_KERNEL=reg, the register-staged ROWS kernel
    const char* e = std::getenv("DPSVM_ROWS_KERNEL");
    return e && std::string(e) == "reg";
  }();
  const int nkb = (dp + 31) / 32;
  static const bool no_persist = [] {  // A/B: DPSVM_ROWS_KERNEL=glds, the tile-per-workgroup LDS-DMA kernel
    const char* e = std::getenv("DPSVM_ROWS_KERNEL");
    return e && std::string(e) == "glds";
  }();
  if (!reg_staged && !no_persist && nkb <= 2) {
    static const int cus = [] {
      int dev = 0, n = 0;
      HIP_CHECK(hipGetDevice(&dev));
      HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
      return std::max(1, n);
    }();
    // the scratch line of the fixed-count stores (64 floats, never read), one per device
    static std::mutex trash_mu;
    static float* trash_of[kMaxDevices] = {};
    float* trash = nullptr;
    {
      const int device = current_device();
      std::lock_guard<std::mutex> lk(trash_mu);
      if (!trash_of[device]) HIP_CHECK(hipMalloc((void**)&trash_of[device], 64 * sizeof(float)));
      trash = trash_of[device];
    }
    const int64_t grid = std::min<int64_t>(tm * tn, cus);
    if (nkb == 1)
      dev::rbf_rows_split_persist_kernel<1><<<dim3((unsigned)grid), dev::kRowsPersistThreads, 0, s>>>(
          (const dev::u4*)X, Xsh, Xsq, a_rows, m_dev, (const dev::u4*)B, Bsh, Bsq, N, gamma, lines, ldl, out_rows,
          trash);
    else
      dev::rbf_rows_split_persist_kernel<2><<<dim3((unsigned)grid), dev::kRowsPersistThreads, 0, s>>>(
          (const dev::u4*)X, Xsh, Xsq, a_rows, m_dev, (const dev::u4*)B, Bsh, Bsq, N, gamma, lines, ldl, out_rows,
          trash);
  } else if (reg_staged) {
    dev::rbf_gemm_split_kernel<dev::SPLIT_ROWS, 6, 1, 0, 2><<<dim3((unsigned)tm, (unsigned)tn), 768, 0, s>>>(
        (const dev::u4*)X, Xsh, Xsq, M_max, (const dev::u4*)B, Bsh, Bsq, N, (dp + 31) / 32, gamma, lines, ldl, 0,
        a_rows, out_rows, m_dev);
  } else {
    static const bool b_cached = [] {  // A/B: DPSVM_ROWS_BNT=0 streams B with the default cache policy
      const char* e = std::getenv("DPSVM_ROWS_BNT");
      return e && std::string(e) == "0";
    }();
    // B ring depth: 3 (A/B: DPSVM_ROWS_BRING=5 — 3.42 vs 3.26-3.28 ms at the
    // synthetic-2m round shape: the kernel is not bound by the B stream's
    // latency; profiles/r6_rows_kernel.txt)
    static const int bring = [] {
      const char* e = std::getenv("DPSVM_ROWS_BRING");
      return e && atoi(e) == 5 ? 5 : 3;
    }();
    auto k = g_rows_stamps ? dev::rbf_rows_split_glds_kernel<2, 3, true>
             : b_cached ? (bring == 5 ? dev::rbf_rows_split_glds_kernel<0, 5> : dev::rbf_rows_split_glds_kernel<0, 3>)
                        : (bring == 5 ? dev::rbf_rows_split_glds_kernel<2, 5> : dev::rbf_rows_split_glds_kernel<2, 3>);
    // persistent over the column tiles (one tile row, nkb >= 3; A/B:
    // DPSVM_ROWS_PERSIST=0)
    static const bool persist = [] {
      const char* e = std::getenv("DPSVM_ROWS_PERSIST");
      return !(e && e[0] == '0');
    }();
    if (persist && tm == 1 && nkb >= 3 && !g_rows_stamps && bring == 3 && (N + 512) * (int64_t)nkb * 8 < (1ll << 32)) {
      static const int cus = [] {
        int n = 0;
        HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, current_device()));
        return std::max(8, n);
      }();
      const int64_t grid = std::min<int64_t>(tn, cus);
      auto kp = b_cached ? dev::rbf_rows_split_glds_persist_kernel<0> : dev::rbf_rows_split_glds_persist_kernel<2>;
      kp<<<dim3((unsigned)grid), dev::kRowsGldsThreads, 0, s>>>((const dev::u4*)X, Xsh, Xsq, a_rows, m_dev,
                                                                (const dev::u4*)B, Bsh, Bsq, N, nkb, gamma, lines, ldl,
                                                                out_rows, (int)tn);
    } else {
      k<<<dim3((unsigned)tm, (unsigned)tn), dev::kRowsGldsThreads, 0, s>>>(
          (const dev::u4*)X, Xsh, Xsq, a_rows, m_dev, (const dev::u4*)B, Bsh, Bsq, N, (dp + 31) / 32, gamma, lines,
          ldl, out_rows, g_rows_stamps);
    }
  }
  post_launch("rbf_rows_indexed_split", s);
}

}  // namespace launch
}  // namespace dpsvm
