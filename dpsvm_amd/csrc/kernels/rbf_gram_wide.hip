// Wide-tile persistent Gram GEMM on split fp16 operands: 256 x 128 tiles.
//
// Why (profiles/r3_pmc_glds_persist/SUMMARY.txt): the 128 x 128 persistent
// LDS-DMA kernel (rbf_gemm_split.hip) ran at ~35% MFMA busy with 41% of wave
// cycles issue-stalled.  Per 32-k block a 128 x 128 tile moves 32 KiB of
// operands through 32 LDS-DMA pieces (1 KiB wave instructions, ~60-185 issue
// cycles each on the wave that issues them) for 96 MFMAs: the DMA issue cost
// is the same order as the MFMA work it feeds.  A 256 x 128 tile moves 48 KiB
// (48 pieces) for 192 MFMAs — half the DMA issue and half the L2 operand
// traffic per MFMA.  Each of the 8 waves owns 64 x 64 outputs (2 x 2 MFMA
// 32x32 tiles, two accumulators each: 128 accumulator registers, two waves per
// SIMD).
//
// Numerics: H = sum h_a h_b as in every split kernel; the cross terms go to ONE
// accumulator PQ, one MFMA per 8-wide k chunk with A' = [h_a | l_a] and
// B' = [l_b | h_b] in the two K halves (h_a l_b + l_a h_b in one fp32 sum).
// Swapping the operands swaps the two K halves of every such MFMA; the Gram's
// bit symmetry K(i, j) == K(j, i) then rests on the MFMA's sum being invariant
// under that swap, which bench/mfma_swap_probe.hip checks on the hardware.
// The values differ from the three-accumulator kernels' by rounding only
// (same products, fp32 sums).
//
// Symmetric mode on 256-row tiles: tile (tx, ty) covers the 128-row blocks
// 2tx and 2tx + 1 of the rows and column block ty; it runs when ty >= 2tx.  A
// wave stores its 128-block (rb, ty) directly when ty >= rb and mirrored when
// ty > rb; the one block below the diagonal a tile can hold (rb = 2tx + 1,
// ty = 2tx) is skipped — its mirror comes from tile (tx, 2tx + 1).
//
// Pipeline: three 48-KiB LDS buffers, two k blocks in flight ahead of the one
// being multiplied (per block: counted vmcnt for the block's own DMA, one raw
// barrier, the DMA of block kb + 2, 2 x 12 MFMAs per wave).  At a tile
// boundary the next tile's first two DMAs are issued BEFORE this tile's
// stores, so they drain under the next tile's MFMAs; the stores are 16-B wide
// (the direct half transposed 4 x 4 across lane quads by DPP): 32 store
// instructions per lane, so the first two waits of the next tile count
// vmcnt(6 + 32) (vmcnt holds 63).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dpsvm/common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "split_util.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

constexpr int kWideThreads = 512;

// x[s] <- x[(s - r) & 3] for the lane's r = 0..3 (two conditional stages)
__device__ __forceinline__ void rot_right4(float (&x)[4], int r) {
  float y[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) y[s] = (r & 1) ? x[(s + 3) & 3] : x[s];
#pragma unroll
  for (int s = 0; s < 4; ++s) x[s] = (r & 2) ? y[(s + 2) & 3] : y[s];
}

template <int CTRL>
__device__ __forceinline__ float quad_perm(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// 4 x 4 transpose across the lanes of a quad: lane i holds v[j] = M(j, i) on
// entry and M(i, j) on exit (lane i of the quad = lane & 3).  Step s sends
// v[(i - s) & 3] and reads lane (i + s) & 3 (one uniform quad_perm per step).
__device__ __forceinline__ void quad_transpose4(float (&v)[4], int i) {
  float r[4] = {v[0], v[3], v[2], v[1]};  // r[s] = v[(-s) & 3]
  rot_right4(r, i);                       // r[s] = v[(i - s) & 3]
  float w[4];
  w[0] = r[0];
  w[1] = quad_perm<0x39>(r[1]);  // lanes read (i + 1) & 3
  w[2] = quad_perm<0x4E>(r[2]);  // (i + 2) & 3
  w[3] = quad_perm<0x93>(r[3]);  // (i + 3) & 3
  rot_right4(w, i);              // column j came at step (j - i) & 3
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = w[j];
}

__global__ __launch_bounds__(kWideThreads, 1) void rbf_gram_wide_kernel(
    const u4* __restrict__ A, const int32_t* __restrict__ Ash, const float* __restrict__ Asq, int M,
    const u4* __restrict__ B, const int32_t* __restrict__ Bsh, const float* __restrict__ Bsq, int N, int nkb,
    float gamma, float* __restrict__ out, int ldo, int sym, int tm, int tn) {
  constexpr int TM = 256, TN = 128, ROWS = TM + TN, CPR = 8, BUF = ROWS * CPR, NB = 3;
  __shared__ u4 lds[NB * BUF + 4 * ROWS / 4];  // 3 operand buffers (144 KiB), then per tile parity |x|^2, shifts
  float* s_sq0 = (float*)(lds + NB * BUF);
  int32_t* s_sh0 = (int32_t*)(lds + NB * BUF) + 2 * ROWS;

  const int total = tm * tn, G = gridDim.x;
  auto valid = [&](int L, int& x, int& y) {
    xcd_tile_of32(L, tm, tn, x, y);
    return !(sym && y < 2 * x);
  };
  int tx = 0, ty = 0, L = blockIdx.x;
  while (L < total && !valid(L, tx, ty)) L += G;
  if (L >= total) return;  // uniform: no barrier reached

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, hl = lane >> 5, qi = lane & 3;
  const int64_t rstride = (int64_t)nkb * 8;
  int m0 = tx * TM, n0 = ty * TN;

  // DMA geometry: wave w fills A rows 32 w + 8 i + (lane >> 3) (i = 0..3) and B
  // rows 16 w + 8 i + (lane >> 3) (i = 0..1); lane position p = lane & 7 takes
  // the global chunk p ^ ((row >> 1) & 7) (the read-side swizzle, TM % 16 == 0)
  const int l3 = lane >> 3;
  int arow[4], brow[2], ach[4], bch[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    arow[i] = 32 * wave + 8 * i + l3;
    ach[i] = (lane & 7) ^ ((arow[i] >> 1) & 7);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    brow[i] = 16 * wave + 8 * i + l3;
    bch[i] = (lane & 7) ^ ((brow[i] >> 1) & 7);
  }
  const u4* srca;
  const u4* srcb;
  auto set_src = [&](int a0, int b0) {
    srca = A + (int64_t)(a0 + 32 * wave + l3) * rstride;
    srcb = B + (int64_t)(b0 + 16 * wave + l3) * rstride;
  };
  auto dma = [&](int kb, int buf) {
    u4* dst = lds + buf * BUF;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srca + (int64_t)(8 * i) * rstride + (int64_t)kb * 8 + ach[i]),
                                       (__attribute__((address_space(3))) void*)(dst + (32 * wave + 8 * i) * CPR),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void*)(srcb + (int64_t)(8 * i) * rstride + (int64_t)kb * 8 + bch[i]),
          (__attribute__((address_space(3))) void*)(dst + (TM + 16 * wave + 8 * i) * CPR), 16, 0, 0);
  };
  auto row_data = [&](int a0, int b0, float& q, int32_t& h) {
    if (tid < ROWS) {
      const int ri = tid < TM ? min(a0 + tid, M - 1) : min(b0 + (tid - TM), N - 1);
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
  __syncthreads();  // row data of the first tile (no DMA in flight yet)
  set_src(m0, n0);
  dma(0, 0);
  if (nkb > 1) dma(1, 1);

  int par = 0;
  int pend = 0;  // store instructions each lane issued after the current tile's first two DMAs (0, 16 or 32)
  f16v H[2][2], PQ[2][2];
  while (true) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) H[a][b][r] = PQ[a][b][r] = 0.f;
    int cb = 0;  // buffer of block kb (kb % 3)
    for (int kb = 0; kb < nkb; ++kb) {
      // block kb's DMA is the oldest in flight but for the previous tile's
      // stores (blocks 0 and 1: between the DMAs of blocks 1 and 2)
      const bool ahead = kb + 1 < nkb;
      const int st = kb < 2 ? pend : 0;
      if (ahead) {
        if (st == 32) asm volatile("s_waitcnt vmcnt(38)" ::: "memory");
        else if (st == 16) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kb + 2 < nkb) dma(kb + 2, cb == 0 ? 2 : cb - 1);  // the buffer of block kb - 1: every wave is past it
      const u4* buf = lds + cb * BUF;
      // operand offsets recomputed per block from an opaque lane id (kept live
      // across the loop they cost ~40 registers)
      int klane = lane;
      asm volatile("" : "+v"(klane));
      const int sw = ((klane & 31) >> 1) & 7, hl = klane >> 5;
      const int ra0 = (wm * 64 + (klane & 31)) * CPR, ra1 = ra0 + 32 * CPR;
      const int rb0 = (TM + wn * 64 + (klane & 31)) * CPR, rb1 = rb0 + 32 * CPR;
      // H: k16 steps, lane half hl supplies h chunk 2 ks + hl (k slots 8 hl ..)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = (2 * ks + hl) ^ sw;
        const h8 b0 = __builtin_bit_cast(h8, buf[rb0 + ch]), b1 = __builtin_bit_cast(h8, buf[rb1 + ch]);
        const h8 a0 = __builtin_bit_cast(h8, buf[ra0 + ch]), a1 = __builtin_bit_cast(h8, buf[ra1 + ch]);
        H[0][0] = mfma32_f16(a0, b0, H[0][0]);
        H[0][1] = mfma32_f16(a0, b1, H[0][1]);
        H[1][0] = mfma32_f16(a1, b0, H[1][0]);
        H[1][1] = mfma32_f16(a1, b1, H[1][1]);
      }
      // PQ: one MFMA per 8-wide k chunk c, A' = [h_a(c) | l_a(c)], B' = [l_b(c) | h_b(c)]:
      // h_a l_b + l_a h_b in one accumulator, K-half swap symmetric
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int ca = ((hl ? 4 : 0) + c) ^ sw, cbk = ((hl ? 0 : 4) + c) ^ sw;
        const h8 b0 = __builtin_bit_cast(h8, buf[rb0 + cbk]), b1 = __builtin_bit_cast(h8, buf[rb1 + cbk]);
        const h8 a0 = __builtin_bit_cast(h8, buf[ra0 + ca]), a1 = __builtin_bit_cast(h8, buf[ra1 + ca]);
        PQ[0][0] = mfma32_f16(a0, b0, PQ[0][0]);
        PQ[0][1] = mfma32_f16(a0, b1, PQ[0][1]);
        PQ[1][0] = mfma32_f16(a1, b0, PQ[1][0]);
        PQ[1][1] = mfma32_f16(a1, b1, PQ[1][1]);
      }
      cb = cb == 2 ? 0 : cb + 1;
    }
    // ---- tile boundary (no DMA in flight: the last block waited vmcnt(0)) ----
    int nL = L + G, ntx = tx, nty = ty;
    while (nL < total && !valid(nL, ntx, nty)) nL += G;
    const bool has_next = nL < total;
    const int nm0 = ntx * TM, nn0 = nty * TN;
    float nq = 0.f;
    int32_t nh = 0;
    if (has_next) row_data(nm0, nn0, nq, nh);
    const float* s_sq = s_sq0 + par * ROWS;
    const int32_t* s_sh = s_sh0 + par * ROWS;
    // the epilogue's lane-dependent offsets are recomputed per tile (an opaque
    // copy of the lane id): hoisted out of the tile loop they would stay live
    // across the k loop and push it past 256 registers
    int elane = lane;
    asm volatile("" : "+v"(elane));
    const int ehl = elane >> 5, eqi = elane & 3;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int cbr = TM + wn * 64 + 32 * b + (elane & 31);
      const float bsq = s_sq[cbr];
      const int bsh = s_sh[cbr];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lr = wm * 64 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * ehl;
          const float dot = ldexpf(H[a][b][r] + PQ[a][b][r], -(s_sh[lr] + bsh));
          H[a][b][r] = rbf_from_dot(s_sq[lr], bsq, dot, gamma);
        }
    }
    if (has_next && tid < ROWS) {
      s_sq0[(par ^ 1) * ROWS + tid] = nq;
      s_sh0[(par ^ 1) * ROWS + tid] = nh;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done with this tile's operand buffers
    asm volatile("" ::: "memory");
    if (has_next) {
      set_src(nm0, nn0);
      dma(0, 0);
      if (nkb > 1) dma(1, 1);
    }
    asm volatile("" ::: "memory");  // the stores stay behind the DMAs
    // this wave's 128-row block and what it stores
    const int rblk = 2 * tx + (wm >> 1);
    const bool direct = !sym || ty >= rblk, mirror = sym && ty > rblk;
    const int wr0 = m0 + wm * 64, wc0 = n0 + wn * 64;  // the wave's 64 x 64 outputs
    const bool interior = wr0 + 64 <= M && wc0 + 64 <= N && nkb >= 3;
    if (interior) {
      if (mirror) {  // transposed: a lane's 4 consecutive rows -> 16 B of out[col][row ..]
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int col = wc0 + 32 * b + (elane & 31);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              f4 v;
              v.x = H[a][b][4 * g + 0];
              v.y = H[a][b][4 * g + 1];
              v.z = H[a][b][4 * g + 2];
              v.w = H[a][b][4 * g + 3];
              *(f4*)(out + (int64_t)col * ldo + wr0 + 32 * a + 8 * g + 4 * ehl) = v;
            }
          }
      }
      if (direct) {  // quad transposes: lane i of a quad takes row +i, columns 4q .. 4q + 3
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              float v[4] = {H[a][b][4 * g + 0], H[a][b][4 * g + 1], H[a][b][4 * g + 2], H[a][b][4 * g + 3]};
              quad_transpose4(v, eqi);
              const int row = wr0 + 32 * a + 8 * g + 4 * ehl + eqi;
              const int col = wc0 + 32 * b + ((elane & 31) & ~3);
              f4 o;
              o.x = v[0];
              o.y = v[1];
              o.z = v[2];
              o.w = v[3];
              *(f4*)(out + (int64_t)row * ldo + col) = o;
            }
      }
      pend = (direct ? 16 : 0) + (mirror ? 16 : 0);
    } else {
      if (direct) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = wr0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * ehl;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              const int col = wc0 + 32 * b + (elane & 31);
              if (row < M && col < N) out[row * ldo + col] = H[a][b][r];
            }
          }
      }
      if (mirror) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int col = wc0 + 32 * b + (elane & 31);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int row = wr0 + 32 * a + 8 * g + 4 * ehl;
              if (col < M) {
#pragma unroll
                for (int c = 0; c < 4; ++c)
                  if (row + c < N) out[(int64_t)col * ldo + row + c] = H[a][b][4 * g + c];
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

}  // namespace dev

namespace launch {

bool rbf_gram_wide_supported(int64_t M, int64_t N, int dp, int64_t ldo) {
  const int64_t tm = (M + 255) / 256, tn = (N + 127) / 128;
  return (dp + 31) / 32 >= 3 && ldo % 4 == 0 && tm * tn < (1ll << 31);
}

void rbf_gram_wide(const void* A, const int32_t* Ash, const float* Asq, int64_t M, const void* B, const int32_t* Bsh,
                   const float* Bsq, int64_t N, int dp, float gamma, float* out, int64_t ldo, hipStream_t s,
                   bool symmetric) {
  if (M <= 0 || N <= 0) return;
  DPSVM_CHECK(rbf_gram_wide_supported(M, N, dp, ldo), "rbf_gram_wide: unsupported shape");
  static const int cus8 = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(8, n / 8 * 8);
  }();
  const int64_t tm = (M + 255) / 256, tn = (N + 127) / 128;
  const int64_t tiles = symmetric ? tm * tn / 2 + tm : tm * tn;  // an upper bound of the valid tiles
  const int grid = (int)std::min<int64_t>(cus8, (tiles + 7) / 8 * 8);
  dev::rbf_gram_wide_kernel<<<dim3((unsigned)grid), dev::kWideThreads, 0, s>>>(
      (const dev::u4*)A, Ash, Asq, (int)M, (const dev::u4*)B, Bsh, Bsq, (int)N, (dp + 31) / 32, gamma, out,
      (int)ldo, symmetric ? 1 : 0, (int)tm, (int)tn);
  post_launch("rbf_gram_wide", s);
}

}  // namespace launch
}  // namespace dpsvm
