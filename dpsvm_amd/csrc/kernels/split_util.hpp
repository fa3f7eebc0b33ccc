// Device helpers shared by the split-operand fp16 MFMA GEMMs
// (rbf_gemm_split.hip): operand vector types, the
// 32x32x16 f16 MFMA and the XCD-aware persistent tile order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_util.hpp"

namespace dpsvm {
namespace dev {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// K from a split GEMM's dot product — the epilogue of EVERY split kernel (the
// Gram, its indexed rows, the predictions, the recompute rounds), so they all
// agree bit for bit: the clamped |x|^2 expansion as rbf_from_dot, then exp on
// the hardware v_exp_f32 (__expf: a multiply by log2 e and one transcendental)
// instead of libm expf's ~10-instruction range reduction (~1 ulp apart)
__device__ __forceinline__ float rbf_split_value(float sq_a, float sq_b, float dot, float gamma) {
#pragma clang fp contract(off)
  float d2 = sq_a + sq_b - 2.0f * dot;
  d2 = d2 > 0.f ? d2 : 0.f;
  return __expf(-gamma * d2);
}

// Error-bounded one-product Gram (the adaptive split Gram, docs/DESIGN.md §13).
// The one-product dot product h_a.h_b differs from the three-product one by
// |h_a.l_b + l_a.h_b| <= 2u(1 + u)|a||b| (u = 2^-11, the fp16 rounding of the
// scaled rows, plus fp32 rounding far below it), so the two d^2 differ by at
// most D = 4.5 u |a||b| and the two K by at most K1 (e^{gamma D} - 1) <=
// 1.72 K1 E for E = gamma D <= 1.  Element (i, j) keeps the one-product value
// K1 when
//     s = R_i + R_j <= c1            (E <= 1)
//     t1 <= c0 - s                   (1.72 K1 E <= tau)
// with R = log2 |x| = split_log2norm(|x|^2), t1 the one-product exp2
// argument and c0 / c1 from split_cold_consts (host); every other element gets
// the three-product value.  The test reads only symmetric quantities (R_i + R_j
// commutes, t1 is the same expression as K's), so the choice is the same for
// (i, j) and (j, i) and in every tiling: the symmetric Gram, the sharded slabs
// and a hot-tile recompute store the same bits.
__device__ __forceinline__ float split_log2norm(float sq) { return 0.5f * __builtin_amdgcn_logf(sq); }
__device__ __forceinline__ bool split_cold(float t1, float s, float c0, float c1) {
  return (s <= c1) & (t1 <= c0 - s);
}

__device__ __forceinline__ f16v mfma32_f16(h8 a, h8 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// XCD-aware tile order in 32-bit arithmetic (persistent kernels: tm * tn <
// 2^31): linear id L runs on XCD L % 8; chunks of 64 tiles (8 x 8 tile
// blocks) are dealt so that an XCD's consecutive tiles share operand panels in
// its L2.  A bijection on the tm x tn grid.
__device__ __forceinline__ void xcd_tile_of32(int L, int tm, int tn, int& tx, int& ty) {
  const int total = tm * tn;
  constexpr int CH = 64, GM = 8;
  const int full = total / (8 * CH) * (8 * CH);
  int T = L;
  if (L < full) {
    const int xcd = L % 8, local = L / 8;
    T = ((local / CH) * 8 + xcd) * CH + local % CH;
  }
  const int first_m = (T / (GM * tn)) * GM;
  const int gm = min(GM, tm - first_m);
  const int in = T - first_m * tn;
  tx = first_m + in % gm;
  ty = in / gm;
}

}  // namespace dev
}  // namespace dpsvm
