// Probe: is v_mfma_f32_32x32x16_f16 invariant under swapping the two 8-wide
// halves of its K dimension?  If D(A', B') with A' = [h_a | l_a], B' = [l_b | h_b]
// equals, bit for bit, D(A'', B'') with A'' = [h_b | l_b], B'' = [l_a | h_a]
// (transposed), the split GEMMs can fold P = h_a.l_b and Q = l_a.h_b into ONE
// accumulator and keep K(i, j) == K(j, i) bitwise (rbf_gemm_split.hip header).
//
// Build: hipcc --offload-arch=gfx950 -O3 bench/mfma_swap_probe.hip -o /tmp/mfma_swap_probe
// Prints the mismatch count over `trials` chains of `steps` MFMAs each.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// a: [trials][steps][32 rows][16] (h 0..7 | l 8..15), b: [trials][steps][32 cols][16]
// d1[t][i][j] from (A', B'), d2[t][j][i] from (A'', B'')
__global__ void probe(const _Float16* a, const _Float16* b, int steps, float* d1, float* d2, int control) {
  const int t = blockIdx.x, lane = threadIdx.x, r = lane & 31, hl = lane >> 5;
  f16v c1, c2;
  for (int q = 0; q < 16; ++q) c1[q] = c2[q] = 0.f;
  for (int s = 0; s < steps; ++s) {
    const _Float16* ar = a + (((size_t)t * steps + s) * 32 + r) * 16;
    const _Float16* br = b + (((size_t)t * steps + s) * 32 + r) * 16;
    h8 A1, B1, A2, B2;
    for (int k = 0; k < 8; ++k) {
      // A' row r: k-slots 0..7 = h_a, 8..15 = l_a  (lane half hl supplies slots 8 hl ..)
      A1[k] = hl == 0 ? ar[k] : ar[8 + k];
      // B' col r: slots 0..7 = l_b, 8..15 = h_b
      B1[k] = hl == 0 ? br[8 + k] : br[k];
      // A'' row r (= the b vectors as rows): h_b | l_b ; B'' col r (= a vectors): l_a | h_a
      A2[k] = hl == 0 ? br[k] : br[8 + k];
      B2[k] = hl == 0 ? ar[8 + k] : ar[k];
    }
    if (!control) {
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B1, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, B2, c2, 0, 0, 0);
    } else {
      // control (expected to mismatch): P then Q as two MFMAs on one accumulator
      h8 z = {};
      h8 A1l = hl ? A1 : z, A1h = hl ? z : A1, B1l = hl ? B1 : z, B1h = hl ? z : B1;
      h8 A2l = hl ? A2 : z, A2h = hl ? z : A2, B2l = hl ? B2 : z, B2h = hl ? z : B2;
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1h, B1h, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1l, B1l, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2h, B2h, c2, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2l, B2l, c2, 0, 0, 0);
    }
  }
  // output layout: lane l has column l & 31, rows (q & 3) + 8 (q >> 2) + 4 hl
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * hl, col = lane & 31;
    d1[((size_t)t * 32 + row) * 32 + col] = c1[q];  // D1[i = row][j = col]
    d2[((size_t)t * 32 + row) * 32 + col] = c2[q];  // D2[j = row][i = col]
  }
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 4096, steps = argc > 2 ? atoi(argv[2]) : 49;
  const int control = argc > 3 ? atoi(argv[3]) : 0;
  std::mt19937 rng(12345);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  const size_t na = (size_t)trials * steps * 32 * 16;
  std::vector<_Float16> a(na), b(na);
  for (size_t i = 0; i < na; i += 16)
    for (int k = 0; k < 8; ++k) {
      for (auto* v : {&a, &b}) {
        // split of x 2^s with |x 2^s| < 2^15: h = fp16(v), l = fp16(v - h)
        const float x = std::ldexp(u(rng), 14 + (int)(rng() % 2));
        const _Float16 h = (_Float16)x;
        (*v)[i + k] = h;
        (*v)[i + 8 + k] = (_Float16)(x - (float)h);
      }
    }
  _Float16 *da, *db;
  float *d1, *d2;
  hipMalloc(&da, na * 2);
  hipMalloc(&db, na * 2);
  hipMalloc(&d1, (size_t)trials * 1024 * 4);
  hipMalloc(&d2, (size_t)trials * 1024 * 4);
  hipMemcpy(da, a.data(), na * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), na * 2, hipMemcpyHostToDevice);
  probe<<<trials, 64>>>(da, db, steps, d1, d2, control);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  std::vector<float> h1((size_t)trials * 1024), h2((size_t)trials * 1024);
  hipMemcpy(h1.data(), d1, h1.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(h2.data(), d2, h2.size() * 4, hipMemcpyDeviceToHost);
  size_t mism = 0, total = 0;
  double maxrel = 0;
  for (int t = 0; t < trials; ++t)
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        const float x = h1[((size_t)t * 32 + i) * 32 + j], y = h2[((size_t)t * 32 + j) * 32 + i];
        ++total;
        if (memcmp(&x, &y, 4) != 0) {
          ++mism;
          maxrel = std::max(maxrel, (double)std::fabs(x - y) / (std::fabs(x) + 1e-30));
        }
      }
  printf("{\"control\": %d, \"trials\": %d, \"steps\": %d, \"elements\": %zu, \"mismatches\": %zu, \"max_rel_diff\": %.3g}\n", control, trials,
         steps, total, mism, maxrel);
  return 0;
}
