// Probe: how fast can the working-set f update (pass 1: d_f_j = sum over the
// round's changed rows k of c_k K(line_k, j)) stream its Gram rows, by access
// layout?  The production kernel (kernels/ws_select.hip, MODE 1) gives each
// thread one column (dword loads, 256 B per wave instruction), four
// partitions of the changed-row list per 1024-thread workgroup and 48 loads in
// flight per thread: 161 us for 3,072 rows x 60,000 columns (4.6 TB/s of row
// bytes, profiles/r3_pass1_bandwidth_notes.txt).  Variants here: VEC columns
// per thread (dword / dwordx2 / dwordx4 loads), loads in flight CH, list
// splits KS (workgroups per column group), and a contiguous streaming read of
// the same byte count as the roofline.
//
// Build: hipcc --offload-arch=gfx950 -O3 bench/pass1_layout_probe.hip -o /tmp/p1probe
// Run:   /tmp/p1probe [rows=60000] [cols=60000] [changed=3072] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

template <int VEC>
struct vt;
template <>
struct vt<1> {
  typedef float t;
};
template <>
struct vt<2> {
  typedef float t __attribute__((ext_vector_type(2)));
};
template <>
struct vt<4> {
  typedef float t __attribute__((ext_vector_type(4)));
};

__global__ void fill(float* g, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    g[i] = 0.25f + 1e-7f * (float)(i & 1023);
}

template <int VEC, int CH, int PARTS, int TPP = 256>
__global__ __launch_bounds__(TPP * PARTS) void pass1(const float* __restrict__ gram, int64_t ld, int ncols,
                                                     const int* __restrict__ lines, const float* __restrict__ coef,
                                                     int na, int G, int ks, float* __restrict__ out) {
  typedef typename vt<VEC>::t V;
  __shared__ int s_idx[4096];
  __shared__ float s_coef[4096];
  __shared__ V s_part[PARTS > 1 ? PARTS - 1 : 1][TPP];
  const int tid = threadIdx.x % TPP, part = threadIdx.x / TPP;
  const int grp = blockIdx.x % G, ksi = blockIdx.x / G;
  for (int k = threadIdx.x; k < na; k += TPP * PARTS) {
    s_idx[k] = lines[k];
    s_coef[k] = coef[k];
  }
  __syncthreads();
  const int col = (grp * TPP + tid) * VEC;
  const bool has = col < ncols;
  const int per = (na + PARTS * ks - 1) / (PARTS * ks);
  const int k_lo = min(na, (ksi * PARTS + part) * per), k_hi = min(na, k_lo + per);
  V acc = (V)0.f;
  for (int k0 = k_lo; k0 < k_hi; k0 += CH) {
    V kv[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int kk = min(k0 + u, k_hi - 1);
      kv[u] = has ? *(const V*)(gram + (int64_t)s_idx[kk] * ld + col) : (V)0.f;
    }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (k0 + u < k_hi) acc = acc + s_coef[k0 + u] * kv[u];
  }
  if (PARTS > 1) {
    if (part > 0) s_part[part - 1][tid] = acc;
    __syncthreads();
    if (part == 0)
      for (int p = 1; p < PARTS; ++p) acc = acc + s_part[p - 1][tid];
  }
  if (part == 0 && has) *(V*)(out + (int64_t)ksi * ncols + col) = acc;
}

// roofline: the same bytes read contiguously (rows 0 .. na-1 of the matrix)
__global__ __launch_bounds__(256) void stream(const float* __restrict__ g, size_t n4, float* __restrict__ out) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc = (f4)0.f;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) acc += ((const f4*)g)[i];
  if (acc.x + acc.y + acc.z + acc.w == -1.f) out[0] = acc.x;
}

template <int VEC, int CH, int PARTS, int TPP = 256>
static void run(const char* name, const float* g, int64_t ld, int ncols, const int* lines, const float* coef, int na,
                int ks, float* out, int reps, double bytes) {
  const int G = (ncols + TPP * VEC - 1) / (TPP * VEC);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(e0));
    pass1<VEC, CH, PARTS, TPP><<<G * ks, TPP * PARTS>>>(g, ld, ncols, lines, coef, na, G, ks, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 2) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  const float med = t[t.size() / 2];
  std::printf("{\"variant\": \"%s\", \"vec\": %d, \"ch\": %d, \"parts\": %d, \"tpp\": %d, \"ks\": %d, "
              "\"workgroups\": %d, \"us_median\": %.1f, \"us_min\": %.1f, \"TBps\": %.2f}\n",
              name, VEC, CH, PARTS, TPP, ks, G * ks, med, t[0], bytes / (med * 1e-6) / 1e12);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 60000;
  const int cols = argc > 2 ? atoi(argv[2]) : 60000;
  const int na = argc > 3 ? atoi(argv[3]) : 3072;
  const int reps = argc > 4 ? atoi(argv[4]) : 20;
  if (na > 4096 || cols % 4) {
    std::fprintf(stderr, "changed <= 4096, cols %% 4 == 0\n");
    return 2;
  }
  const size_t n = (size_t)rows * cols;
  float *g, *coef, *out;
  int* lines;
  CK(hipMalloc(&g, n * 4));
  CK(hipMalloc(&coef, na * 4));
  CK(hipMalloc(&lines, na * 4));
  CK(hipMalloc(&out, (size_t)16 * cols * 4));
  fill<<<4096, 256>>>(g, n);
  std::vector<int> perm(rows);
  std::iota(perm.begin(), perm.end(), 0);
  std::mt19937 rng(0);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<float> c(na);
  for (int k = 0; k < na; ++k) c[k] = 1e-2f * (float)((int)(rng() % 201) - 100);
  CK(hipMemcpy(lines, perm.data(), na * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(coef, c.data(), na * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  const double bytes = (double)na * cols * 4;
  // the production layout, then the variants
  run<1, 48, 4>("prod dword", g, cols, cols, lines, coef, na, 1, out, reps, bytes);
  run<1, 32, 4>("dword ch32", g, cols, cols, lines, coef, na, 1, out, reps, bytes);
  run<1, 48, 4>("dword ks2", g, cols, cols, lines, coef, na, 2, out, reps, bytes);
  run<2, 24, 4>("dwordx2 ks2", g, cols, cols, lines, coef, na, 2, out, reps, bytes);
  run<2, 16, 4>("dwordx2 ch16 ks2", g, cols, cols, lines, coef, na, 2, out, reps, bytes);
  run<4, 12, 4>("dwordx4 ks4", g, cols, cols, lines, coef, na, 4, out, reps, bytes);
  run<4, 8, 4>("dwordx4 ch8 ks4", g, cols, cols, lines, coef, na, 4, out, reps, bytes);
  run<4, 12, 4>("dwordx4 ks8", g, cols, cols, lines, coef, na, 8, out, reps, bytes);
  run<4, 12, 2>("dwordx4 p2 ks8", g, cols, cols, lines, coef, na, 8, out, reps, bytes);
  run<4, 16, 1>("dwordx4 p1 ch16 ks16", g, cols, cols, lines, coef, na, 16, out, reps, bytes);
  // 256 columns per workgroup as production (same slices per column), 4 columns per thread
  run<4, 12, 4, 64>("dwordx4 tpp64 ch12", g, cols, cols, lines, coef, na, 1, out, reps, bytes);
  run<4, 24, 4, 64>("dwordx4 tpp64 ch24", g, cols, cols, lines, coef, na, 1, out, reps, bytes);
  run<4, 32, 4, 64>("dwordx4 tpp64 ch32", g, cols, cols, lines, coef, na, 1, out, reps, bytes);
  run<2, 24, 4, 128>("dwordx2 tpp128 ch24", g, cols, cols, lines, coef, na, 1, out, reps, bytes);
  run<2, 48, 4, 128>("dwordx2 tpp128 ch48", g, cols, cols, lines, coef, na, 1, out, reps, bytes);
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    const size_t n4 = (size_t)na * cols / 4;
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipEventRecord(e0));
      stream<<<8192, 256>>>(g, n4, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) t.push_back(ms * 1e3f);
    }
    std::sort(t.begin(), t.end());
    std::printf("{\"variant\": \"contiguous stream (roofline)\", \"us_median\": %.1f, \"TBps\": %.2f}\n", t[t.size() / 2],
                bytes / (t[t.size() / 2] * 1e-6) / 1e12);
  }
  CK(hipFree(g));
  return 0;
}
