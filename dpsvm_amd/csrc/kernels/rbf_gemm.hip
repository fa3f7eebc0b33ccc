// RBF GEMM on fp32 MFMA (v_mfma_f32_32x32x2_f32: exact f32, 64 FLOP/clk/SIMD).
//
// Two fused epilogues over the same LDS-tiled main loop (C = A . B^T):
//   STORE   : out[i][j] = exp(-g * max(|a_i|^2 + |b_j|^2 - 2 c_ij, 0))
//             -> the whole resident Gram shard in one launch (dense cache mode)
//   PREDICT : partial[s][i] = sum_{j in split s} coef_j * exp(...)
//             -> decision values / training accuracy in one launch.
//   ROWS    : STORE with row indirection — A row i is X row a_rows[i], output
//             row i goes to line out_rows[i], M read on the device (*m_dev):
//             the kernel rows of a working set's cache misses in one launch
//             (the working-set cache engine, ws_*.hip).
//             Replaces the reference's n x (cublasSgemv + thrust::transform_reduce)
//             launches (svmTrain.cu:633-665, K12/K13).
//
// Tiling: 128x128 block tile, BK = 16, 256 threads = 4 waves (2x2), each wave
// 64x64 = 2x2 MFMA 32x32 tiles (64 accumulator registers).  ROWS with a short
// row set (<= 64 rows per tile) uses a 64x256 tile (4 waves 1x4): with 128x128
// the waves of the dead row half sit on SIMDs 2-3 (waves are dealt to SIMDs
// in order), which then issue no MFMA at all — half the CU's matrix rate.  A/B tiles are
// staged k-major in LDS (+4 float pad) through registers, double buffered so
// the next tile's global loads overlap the current tile's 32 MFMAs per wave.
// Operand maps (32x32x2 f32): A lane l -> (row l&31, k l>>5); B lane l ->
// (k l>>5, col l&31); C reg r of lane l -> (row (r&3)+8(r>>2)+4(l>>5), col l&31).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "dpsvm/common.hpp"
#include "device_util.hpp"
#include "kernels.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace dev {

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int GEMM_THREADS = 256;

enum Epi { EPI_STORE = 0, EPI_PREDICT = 1, EPI_ROWS = 2 };

// Tile shapes (4 waves; each wave MI x NJ MFMA 32x32 tiles = 64 accumulators):
//   <128, 2, 2>  128x128, waves 2x2     STORE (incl. symmetric) / PREDICT
//   < 64, 2, 2>   64x256, waves 1x4     ROWS (row sets of 33-64 rows per tile)
//   < 32, 1, 4>   32x512, waves 1x4     ROWS variant padding rows to 32 (measured
//                                       slower than 64x256, not launched)
template <int EPI, int TM = 128, int MI = 2, int NJ = 2>
__global__ __launch_bounds__(GEMM_THREADS, EPI == EPI_STORE ? 3 : 2) void rbf_gemm_kernel(
    const float* __restrict__ A, const float* __restrict__ Asq, int64_t M, int lda,
    const float* __restrict__ B, const float* __restrict__ Bsq, int64_t N, int ldb, int dp,
    float gamma, float* __restrict__ out, int64_t ldo, const float* __restrict__ coef,
    int n_tiles_per_split, int sym, const int32_t* __restrict__ a_rows = nullptr,
    const int32_t* __restrict__ out_rows = nullptr, const int32_t* __restrict__ m_dev = nullptr) {
  // sym (STORE, B == A, N == M): only tiles on/above the diagonal are computed;
  // each off-diagonal tile also writes its transpose.  K(i,j) and K(j,i) are
  // bit-identical (same products in the same k order, commutative norm sum).
  // Tile of this workgroup.  STORE: XCD-aware order — workgroups are dealt
  // round-robin over the 8 XCDs (linear id L runs on XCD L % 8), so the tile
  // sequence is cut in chunks of 64 and XCD x takes chunks x, x + 8, ...; a
  // chunk is an 8 x 8 block of tiles (groups of 8 tile-rows, column-major), so
  // an XCD's consecutive tiles share B panels and re-read A panels from its
  // L2, while every XCD still sees the whole matrix (balanced under the
  // symmetric mode's skipped lower triangle).  A bijection on the grid; the
  // tile math is unchanged: bit-identical output (every element is the same
  // MFMA k-sequence in every tile shape).
  constexpr int WM = TM / (32 * MI), WN = 4 / WM, TN = WN * 32 * NJ, LDA = TM + 4, LDB = TN + 4;
  static_assert(WM * WN == 4 && MI * NJ == 4, "4 waves of 2x2 / 1x4 MFMA tiles");
  static_assert((TM == 128 && MI == 2 && NJ == 2) || EPI == EPI_ROWS, "narrow tiles: ROWS epilogue only");
  constexpr int NA = TM >= 64 ? TM / 64 : 1;  // A float4 loads per thread (TM = 32: threads < 128)
  constexpr int NB = TN / 64;                 // B float4 loads per thread
  int64_t tx = blockIdx.x, ty = blockIdx.y;
  if (EPI == EPI_ROWS) M = *m_dev;
  if (EPI == EPI_STORE || EPI == EPI_ROWS) {
    const int64_t tm = gridDim.x, tn = gridDim.y, total = tm * tn;
    const int64_t L = blockIdx.x + (int64_t)blockIdx.y * tm;
    constexpr int64_t CH = 64;
    const int64_t full = total / (8 * CH) * (8 * CH);
    int64_t T = L;  // the tail past the last whole round keeps its order
    if (L < full) {
      const int64_t xcd = L % 8, local = L / 8;
      T = ((local / CH) * 8 + xcd) * CH + local % CH;
    }
    constexpr int64_t GM = 8;
    const int64_t first_m = (T / (GM * tn)) * GM;
    const int64_t gm = min(GM, tm - first_m);
    const int64_t in = T - first_m * tn;  // position inside the group (column-major)
    tx = first_m + in % gm;
    ty = in / gm;
  }
  if (EPI == EPI_STORE && sym && ty < tx) return;
  if (EPI == EPI_ROWS && tx * TM >= M) return;  // uniform: no barrier reached
  __shared__ __attribute__((aligned(16))) float As[2][BK][LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDB];
  __shared__ float red[EPI == EPI_PREDICT ? 2 : 1][EPI == EPI_PREDICT ? BM : 1];
  __shared__ float s_asq[EPI == EPI_ROWS ? TM : 1];      // ROWS: |x|^2 of the tile's rows
  __shared__ int32_t s_orow[EPI == EPI_ROWS ? TM : 1];   // ROWS: their output lines (-1: past M)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int rw = wm * 32 * MI, cw = wn * 32 * NJ;  // the wave's tile origin
  const int64_t m0 = tx * TM;
  const int64_t ntiles_total = (N + TN - 1) / TN;
  int64_t nt_begin, nt_end;
  if (EPI != EPI_PREDICT) {
    nt_begin = ty;
    nt_end = nt_begin + 1;
  } else {
    nt_begin = ty * n_tiles_per_split;
    nt_end = nt_begin + n_tiles_per_split;
    if (nt_end > ntiles_total) nt_end = ntiles_total;
  }
  // staging map: row r_ld0 + 64 i, k4 = tid & 3 (TM x 16 and TN x 16 floats)
  const int r_ld0 = tid >> 2, k4_ld = tid & 3;
  const bool a_ld = TM >= 64 || r_ld0 < TM;
  const int nk = dp / BK;  // dp is a multiple of 16

  if (EPI == EPI_ROWS && threadIdx.x < TM) {
    // the tile's row metadata once (read from LDS in the epilogue instead of
    // two dependent global loads per output element)
    const int64_t row = m0 + threadIdx.x;
    s_asq[threadIdx.x] = Asq[a_rows[min(row, M - 1)]];
    s_orow[threadIdx.x] = row < M ? out_rows[row] : -1;
  }

  float rowacc[MI][16];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) rowacc[i][r] = 0.f;

  for (int64_t nt = nt_begin; nt < nt_end; ++nt) {
    const int64_t n0 = nt * TN;
    f16v acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const float* ga[NA];
    const float* gb[NB];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int64_t ar = m0 + (a_ld ? r_ld0 : 0) + 64 * i;
      ga[i] = A + ar * (int64_t)lda + 4 * k4_ld;
      if (EPI == EPI_ROWS)  // rows past M repeat the last one (never stored)
        ga[i] = A + (int64_t)a_rows[min(ar, M - 1)] * lda + 4 * k4_ld;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) gb[i] = B + (n0 + r_ld0 + 64 * i) * (int64_t)ldb + 4 * k4_ld;
    f4 ra[NA], rb[NB];
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = *(const f4*)ga[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) rb[i] = *(const f4*)gb[i];
    auto stage = [&](int buf) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (a_ld) {
#pragma unroll
          for (int i = 0; i < NA; ++i) As[buf][4 * k4_ld + c][r_ld0 + 64 * i] = ra[i][c];
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) Bs[buf][4 * k4_ld + c][r_ld0 + 64 * i] = rb[i][c];
      }
    };
    __syncthreads();  // previous n-tile's readers are done with buffer 0
    stage(0);
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) {
        const int koff = (kt + 1) * BK;
#pragma unroll
        for (int i = 0; i < NA; ++i) ra[i] = *(const f4*)(ga[i] + koff);
#pragma unroll
        for (int i = 0; i < NB; ++i) rb[i] = *(const f4*)(gb[i] + koff);
      }
      // ROWS: a wave whose rows all lie past M only stages (uniform skip)
      const bool live = EPI != EPI_ROWS || m0 + rw < M;
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        if (!live) break;
        const int kr = 2 * kk + (lane >> 5);
        float av[MI], bv[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) av[i] = As[cur][kr][rw + 32 * i + (lane & 31)];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bv[j] = Bs[cur][kr][cw + 32 * j + (lane & 31)];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
      }
      if (more) stage(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }

    // ---- epilogue ----
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if (EPI == EPI_ROWS && m0 + rw + i * 32 >= M) continue;  // uniform: no exp for rows past M
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int64_t col = n0 + cw + j * 32 + (lane & 31);
        const float bsq = Bsq[col];
        float cf = 0.f;
        if (EPI == EPI_PREDICT) cf = col < N ? coef[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int lr = rw + i * 32 + rl;
          const int64_t row = m0 + lr;
          if (EPI == EPI_ROWS) {
            const int32_t orow = s_orow[lr];
            if (orow >= 0 && col < N) out[(int64_t)orow * ldo + col] = rbf_from_dot(s_asq[lr], bsq, acc[i][j][r], gamma);
            continue;
          }
          const float kv = rbf_from_dot(Asq[row], bsq, acc[i][j][r], gamma);
          if (EPI == EPI_STORE) {
            if (row < M && col < N) out[row * ldo + col] = kv;
            if (sym) acc[i][j][r] = kv;  // kept for the transposed store
          } else {
            rowacc[i][r] += cf * kv;
          }
        }
      }
    }
    if (EPI == EPI_STORE && sym && ty != tx) {
      // transposed tile: lane holds 4 consecutive rows per group -> 16-B stores
      // out[col][row .. row+3] (each store instruction: 32 rows x 32 B)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int64_t col = n0 + cw + j * 32 + (lane & 31);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int64_t row = m0 + rw + i * 32 + 8 * q + 4 * (lane >> 5);
            if (col >= M) continue;
            float* dst = out + col * ldo + row;
            if (row + 3 < N) {
              f4 v;
              v.x = acc[i][j][4 * q + 0];
              v.y = acc[i][j][4 * q + 1];
              v.z = acc[i][j][4 * q + 2];
              v.w = acc[i][j][4 * q + 3];
              *(f4*)dst = v;
            } else {
#pragma unroll
              for (int c = 0; c < 4; ++c)
                if (row + c < N) dst[c] = acc[i][j][4 * q + c];
            }
          }
        }
      }
    }
  }

  if (EPI == EPI_PREDICT) {
    // sum over the 32 columns held by lanes with equal (lane>>5), then over wn
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = rowacc[i][r];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 16, 64);
        rowacc[i][r] = v;
      }
    if ((lane & 31) == 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          red[wn][rw + i * 32 + rl] = rowacc[i][r];
        }
    }
    __syncthreads();
    if (tid < BM) {
      const int64_t row = m0 + tid;
      // out = partial [splits][ldo], ldo = M_pad
      out[ty * ldo + row] = red[0][tid] + red[1][tid];
    }
  }
}

__global__ void predict_reduce_kernel(const float* partial, int64_t M, int64_t ldp, int splits,
                                      float b, float* dec, const float* y, int32_t* correct) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool ok = false;
  if (i < M) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += partial[(int64_t)k * ldp + i];
    const float v = s - b;  // svmTrain.cu:652
    if (dec) dec[i] = v;
    if (y) ok = ((v < 0.f ? -1.f : 1.f) == y[i]);
  }
  if (correct) {
    const uint64_t m = __ballot(ok);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(correct, (int32_t)__popcll(m));
  }
}

}  // namespace dev

namespace launch {

static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

void rbf_gemm_store(const float* A, const float* Asq, int64_t M, int lda, const float* B,
                    const float* Bsq, int64_t N, int ldb, int dp, float gamma, float* out,
                    int64_t ldo, hipStream_t s, bool symmetric) {
  if (M <= 0 || N <= 0) return;
  DPSVM_CHECK(dp % 16 == 0, "rbf_gemm: dp must be a multiple of 16");
  DPSVM_CHECK(!symmetric || (A == B && Asq == Bsq && M == N && lda == ldb && ldo % 4 == 0),
              "rbf_gemm_store: symmetric mode needs B == A, N == M");
  const int64_t tm = (M + dev::BM - 1) / dev::BM, tn = (N + dev::BN - 1) / dev::BN;
  DPSVM_CHECK(tn < 65536, "rbf_gemm_store: N too large for grid.y");
  dev::rbf_gemm_kernel<dev::EPI_STORE><<<dim3((unsigned)tm, (unsigned)tn), dev::GEMM_THREADS, 0, s>>>(
      A, Asq, M, lda, B, Bsq, N, ldb, dp, gamma, out, ldo, nullptr, 1, symmetric ? 1 : 0);
  post_launch("rbf_gemm_store", s);
}

void rbf_rows_indexed(const float* X, const float* Xsq, const int32_t* a_rows, const int32_t* m_dev, int64_t M_max,
                      const float* B, const float* Bsq, int64_t N, int dp, float gamma, float* lines,
                      const int32_t* out_rows, int64_t ldl, hipStream_t s) {
  if (M_max <= 0 || N <= 0) return;
  DPSVM_CHECK(dp % 16 == 0, "rbf_rows_indexed: dp must be a multiple of 16");
  // 64x256 tiles (B, the columns, readable to a multiple of 256 rows).  The
  // 32x512 shape pads less (rows to 32) but ran slower (500k x 1024: 7.71 s vs
  // 6.43 s; covtype 8.22 vs 7.33: 5 LDS reads per 4 MFMAs, twice the B staging)
  const int64_t tm = (M_max + 63) / 64, tn = (N + 255) / 256;
  DPSVM_CHECK(tn < 65536, "rbf_rows_indexed: N too large for grid.y");
  dev::rbf_gemm_kernel<dev::EPI_ROWS, 64, 2, 2><<<dim3((unsigned)tm, (unsigned)tn), dev::GEMM_THREADS, 0, s>>>(
      X, Xsq, M_max, dp, B, Bsq, N, dp, dp, gamma, lines, ldl, nullptr, 1, 0, a_rows, out_rows, m_dev);
  post_launch("rbf_rows_indexed", s);
}

static int predict_splits(int64_t M, int64_t N) {
  const int64_t tm = (M + dev::BM - 1) / dev::BM, tn = (N + dev::BN - 1) / dev::BN;
  int64_t splits = (2048 + tm - 1) / tm;  // aim for >= 2048 workgroups (8 per CU)
  if (splits > tn) splits = tn;
  if (splits < 1) splits = 1;
  if (splits > 4096) splits = 4096;
  return (int)splits;
}

int64_t predict_scratch_floats(int64_t M, int64_t N) {
  return (int64_t)predict_splits(M, std::max<int64_t>(N, 1)) * round_up(std::max<int64_t>(M, 1), dev::BM);
}

bool predict_uses_split(int dp) {
  static const bool f32_only = [] {
    const char* e = std::getenv("DPSVM_PREDICT");  // A/B: f32 = the f32-input MFMA decision GEMM
    return e && std::string(e) == "f32";
  }();
  return !f32_only && dp >= 128;
}

void rbf_predict(const float* A, const float* Asq, int64_t M, int lda, const float* B,
                 const float* Bsq, const float* coef, int64_t N, int ldb, int dp, float gamma,
                 float b, float* partial, float* dec, const float* y, int32_t* correct,
                 hipStream_t s, int precision) {
  if (M <= 0) return;
  DPSVM_CHECK(dp % 16 == 0, "rbf_predict: dp must be a multiple of 16");
  const int64_t ldp = round_up(M, dev::BM);
  int splits = 1;
  if (N > 0) {
    const int64_t tm = ldp / dev::BM, tn = (N + dev::BN - 1) / dev::BN;
    splits = predict_splits(M, N);
    const int per = (int)((tn + splits - 1) / splits);
    splits = (int)((tn + per - 1) / per);
    if (precision == 2 || (precision == 0 && predict_uses_split(dp))) {
      // split-operand fp16 MFMA with LDS-DMA staging (fp32 accuracy, rbf_gemm_split.hip)
      rbf_predict_split(A, Asq, M, lda, B, Bsq, coef, N, ldb, dp, gamma, partial, ldp, splits, s);
    } else {
      dev::rbf_gemm_kernel<dev::EPI_PREDICT><<<dim3((unsigned)tm, (unsigned)splits), dev::GEMM_THREADS, 0, s>>>(
          A, Asq, M, lda, B, Bsq, N, ldb, dp, gamma, partial, ldp, coef, per, 0);
      post_launch("rbf_predict", s);
    }
  } else {
    HIP_CHECK(hipMemsetAsync(partial, 0, sizeof(float) * ldp, s));
  }
  dev::predict_reduce_kernel<<<dim3((unsigned)((M + 255) / 256)), 256, 0, s>>>(partial, M, ldp, splits, b,
                                                                             dec, y, correct);
  post_launch("predict_reduce", s);
}

}  // namespace launch
}  // namespace dpsvm
