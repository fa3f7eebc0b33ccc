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
