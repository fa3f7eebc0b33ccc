// dpsvm_amd — MI355X-native distributed RBF C-SVM trainer (modified SMO).
//
// Shared host/device definitions: error checking, parameters, order-preserving
// selection keys and the solver result record.
//
// Behavioural reference: farshid83/dpsvm
//   - algorithm / stop test / alpha update: svmTrainMain.cpp:235-310
//   - I-set classification:                  svmTrain.cu:41-95
//   - defaults (eps 1e-3, C 1, 150000 iters): svmTrainMain.cpp:60-136
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#if defined(__HIPCC__)
#define DPSVM_HD __host__ __device__ __forceinline__
#else
#define DPSVM_HD inline
#endif

namespace dpsvm {

// ---------------------------------------------------------------------------
// Errors
// ---------------------------------------------------------------------------
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] inline void fail(const std::string& msg) { throw Error(msg); }

#define DPSVM_CHECK(cond, msg)                                                   \
  do {                                                                           \
    if (!(cond)) ::dpsvm::fail(std::string("dpsvm: ") + (msg) + " [" __FILE__ ":" + \
                               std::to_string(__LINE__) + "]");                  \
  } while (0)

// ---------------------------------------------------------------------------
// Parameters
// ---------------------------------------------------------------------------
enum class ClipMode : int {
  Independent = 0,  // reference behaviour: both alphas clipped to [0,C] separately
                    // (svmTrainMain.cpp:294-295)
  Box = 1,          // LIBSVM-style joint [L,H] box, keeps sum(alpha*y) = 0
};

// host bound on one block of iterations when SolverParams::watchdog_s is 0 (auto)
constexpr double kWatchdogDefaultS = 1800.0;

struct SolverParams {
  float C = 1.0f;
  float gamma = -1.0f;        // <0 -> 1/d (reference uses integer 1/d == 0)
  float eps = 1e-3f;          // stop when !(b_lo > b_hi + 2 eps)
  int64_t max_iter = 150000;
  ClipMode clip = ClipMode::Independent;
  float tau = 1e-12f;         // eta floor
  // kernel-row cache
  int64_t cache_lines = 0;    // explicit number of lines (0 = auto)
  double cache_mb = 0.0;      // explicit size in MiB (0 = auto)
  double cache_frac = 0.80;   // auto: fraction of free HBM used for lines
  int64_t host_cache_lines = 0;  // pinned host spill tier (lines); 0 = off
  // X-pass batching: extra speculative kernel rows computed on a miss
  int spec_rows = 14;
  // execution
  int graph_block = 64;       // SMO iterations captured per hipGraph
  bool use_graph = true;
  int x_mode = 0;             // 0 auto, 1 replicated, 2 partitioned
  int log_every = 0;
  bool verbose = false;
  // checkpoint
  int64_t checkpoint_every = 0;
  std::string checkpoint_path;
  // debugging
  bool sync_debug = false;    // device sync + error check after every launch
  bool force_collectives = false;  // run the per-iteration collective even at world 1 (tests RCCL/graph paths)
  // per-iteration key exchange of the dense fused mode: 0 auto (peer exchange
  // when world > 1 and its self test passes, else the communicator's
  // all-reduce), 1 communicator all-reduce, 2 peer exchange (required; also
  // at world 1 as a loopback, for tests)
  int exchange = 0;
  // iteration engine: 0 auto, 1 one launch per iteration (graphs), 2 persistent
  // kernel (persist_block iterations per launch; dense and cache mode)
  int persist = 0;
  int persist_block = 2048;
  // ---- engine / geometry selection (recorded in GpuSetupInfo and --metrics-json;
  //      every choice is a parameter, none comes from the environment) ----
  bool force_cache = false;   // kernel-row cache mode even when the Gram shard fits
  int cache_engine = 0;       // cache mode, one launch per iteration: 0 fused kernel, 1 rows/step/finalize chain
  // 0 production (kEngineTable: ws-dense, ws-cache, persistent-dense, fused-dense), 1 all — also the
  // quarantined pair-at-a-time engines for a Gram that is not resident or an X that is partitioned
  // (kQuarantineTable: persistent-cache, fused-cache, chain; tests and A/B probes only)
  int engines = 0;
  int cache_groups = 256;     // cache mode: workgroups per rank (one per CU: the X pass wants every CU)
  int rows_per_group = 0;     // rows per workgroup of the fused / persistent engines (0 auto; multiple of 256)
  // peer exchange (in-kernel key exchange of the fused / persistent engines)
  int xch_poll_batch = 0;     // publications watched per lane per poll round: 0 auto, 1, 2, 4
  int xch_sleep = 1;          // s_sleep(1) count between poll rounds
  int xch_stride = 4;         // u64 slots per exchange entry (>= 4; larger pads entries apart)
  int xch_mem = 0;            // receive buffer: 0 auto (uncached when world > 1), 1 uncached, 2 coarse
  double xch_timeout_s = 120.0;  // give-up bound of one in-kernel poll loop (then status 5)
  double watchdog_s = 0.0;       // host bound on one block of iterations (s); 0 = auto: 1800, and at
                                 // world > 1 adaptive (120 s for the first blocks, then 50x the slowest)
  // residency census of the persistent engines (tests: a grid of this many
  // workgroups instead of the engine's, > the device's capacity forces the
  // fallback to the one-launch-per-iteration engine)
  int census_groups = 0;
  bool verify_ranks = true;   // world > 1: cross-rank alpha digest after every solve
  // data-parallel policy when world > 1: 0 auto, 1 shard the rows, 2 every rank
  // solves the whole problem.  auto replicates only when the ranks sit on
  // distinct devices, the whole Gram fits one device and the one-device
  // persistent engine runs its fast geometry (<= 256 workgroups of <= 1024
  // rows): the SMO iteration is a latency chain, and sharding such a problem
  // adds a cross-device hop to every iteration while saving only the Gram
  // GEMM (docs/DESIGN.md "Multi-GPU").
  int dp_policy = 0;
  // solver: 0 auto, 1 pair-at-a-time SMO engines (the reference's trajectory),
  // 2 working-set rounds (ws engine, ws_*.hip: the reference's pair rule on
  // a q-row sub-problem in LDS, the same global stop test)
  int solver = 0;
  int ws_size = 192;          // working-set rows q (<= 192: the q x q sub-Gram lives in LDS)
  int ws_new = 0;             // rows replaced per one-block round (0: auto, ws_new_auto in device_state.hpp)
  float ws_rel = 0.3f;        // sub-problem tolerance: max(eps, ws_rel * global gap / 2), < 1
  int ws_blocks = 0;          // working-set engines: up to P disjoint q-row sub-problems per round (1..128,
                              // P x ws_size <= 6144; 0 auto from 50k rows: 128 x 48 rows on numerically diagonal
                              // ws-dense kernels, else 32 x 96 (3072 rows); below 50k rows 1).  Adaptive: halved
                              // after every damped round (coupled blocks), 1 after an independent-clip event,
                              // then the one-block round kernels (ws_*.hip)
  int ws_inner = 0;           // pair steps per round at most (0: 4 * ws_size)
  int ws_wss = 0;             // sub-problem pair choice: 1 the reference's first-order rule (max f over I_low),
                              // 2 second order (WSS2: max (f_lo - b_hi)^2 / eta); the stop test is unchanged;
                              // 0 auto: second order when a row sample's mean off-diagonal K > 0.1
  int ws_recompute = 0;       // ws-cache rounds without the row cache (ws_recompute.hip: kernel rows recomputed,
                              // fused into the f update): 0 auto (one rank, one block, d <= 64 padded), 1 on, 2 off
  int ws_block = 8;           // rounds per hipGraph block (the host stops at most ~2 blocks past convergence;
                              // the one-block switch stays on 32-round boundaries: same trajectories)
  float ws_t_halve = 0.9f;    // multi-block: a round damped below this line-search factor halves the block count
  int ws_clip_fallback = 1;   // multi-block, independent clipping: 1 = one block per round after a clip event
  // eta's K(i_hi, i_lo) in the pair-at-a-time dense engines: 0 from the two X
  // rows (explicit difference, the same tree in every engine: bit parity), 1
  // from the resident Gram (persistent dense engine with every column local;
  // one load in the Gram-row round trip instead of the X-row reads and a barrier)
  int eta = 0;
  // Gram / kernel-row GEMM arithmetic: 1 f32-input MFMA (rbf_gemm.hip), 2 fp16
  // MFMA over hi / lo split operands (rbf_gemm_split.hip: fp32 accuracy, 3/16 of
  // the MFMA time), 0 auto = split for the working-set engines, f32 for the
  // pair-at-a-time engines (the reference's trajectory)
  int gram_precision = 0;
  // adaptive split Gram (ws-dense resident Gram, docs/DESIGN.md §13): one-product tiles where every element is
  // provably within gram_cold_tau of the three-product value, the rest recomputed: 0 auto (on when a row
  // sample's elements all pass the bound), 1 on, 2 off
  int gram_adapt = 0;
  float gram_cold_tau = 0x1p-22f;
};


// Per-run result, gathered on every rank.
struct SolveResult {
  std::vector<float> alpha;   // length n (global)
  float b = 0.f, b_hi = 0.f, b_lo = 0.f;
  int64_t iters = 0;
  int status = 0;             // 1 converged, 2 max_iter, 3 no violating pair, 4 non-finite
  double t_setup = 0.0, t_solve = 0.0;
  double t_gram = 0.0;  // device time of the resident Gram GEMM inside t_solve (dense mode)
  // adaptive split Gram (gram_adapt, docs/DESIGN.md §13): tiles of the one-product pass and how many of them
  // held an element the error bound rejected (recomputed with all three products); -1: not adaptive
  int64_t gram_tiles = -1, gram_hot_tiles = -1;
  int64_t cache_hits = 0, cache_misses = 0, rows_computed = 0, x_passes = 0;
  int64_t host_hits = 0, spec_rows = 0;
  int64_t cache_lines = 0, host_cache_lines = 0;
  int world = 1;
  double verify_f_err = -1.0;  // DPSVM_VERIFY: max |f - f(alpha)| / (1 + |f(alpha)|), -1 = not run
  int64_t outer = 0;           // working-set engine: rounds
  // multi-block working-set rounds: blocks at the start / at the end (adaptive),
  // rounds completed when the count reached 1 (0: never), damped rounds
  int ws_blocks = 1, ws_blocks_end = 1;
  int64_t ws_p1_round = 0, ws_damped = 0;
  int shrink_phases = 0;       // solve_shrinking: device solves on the (active) rows
  // solve_shrinking: one entry per phase, "rows engine/dp_policy exchange rounds seconds" (';'-separated)
  std::string phase_log;
  bool converged() const { return status == 1; }
};

// ---------------------------------------------------------------------------
// Order-preserving selection keys.
//
// A key packs (f, global index) into one u64 so that an unsigned min over keys
// picks the smallest f and, on ties, the lowest global index (SURVEY Q15:
// deterministic on every rank).  b_lo = max f over I_low is encoded with -f.
// ---------------------------------------------------------------------------
constexpr uint64_t kKeyNone = ~0ull;

DPSVM_HD uint32_t f32_bits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}
DPSVM_HD float bits_f32(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
DPSVM_HD uint32_t f32_order(float f) {
  uint32_t u = f32_bits(f);
  if (u == 0x80000000u) u = 0u;  // -0 == +0
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
DPSVM_HD float order_f32(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return bits_f32(u);
}
DPSVM_HD uint64_t make_key(float f, uint32_t idx) {
  return ((uint64_t)f32_order(f) << 32) | (uint64_t)idx;
}
DPSVM_HD float key_value(uint64_t k) { return order_f32((uint32_t)(k >> 32)); }
DPSVM_HD uint32_t key_index(uint64_t k) { return (uint32_t)(k & 0xffffffffu); }

// I_up / I_low membership (svmTrain.cu:56-91; seq.cpp:469-493).
DPSVM_HD bool in_up(float a, float y, float C) {
  if (a == 0.0f) return y == 1.0f;
  if (a == C) return y != 1.0f;
  return true;
}
DPSVM_HD bool in_low(float a, float y, float C) {
  if (a == 0.0f) return y != 1.0f;
  if (a == C) return y == 1.0f;
  return true;
}

DPSVM_HD float clip01(float v, float lo, float hi) {
  // reference clip_value (svmTrain.cu:674-682); NaN falls through unchanged
  if (v < lo) return lo;
  if (v > hi) return hi;
  return v;
}

// One SMO pair update.  Shared by the CPU solver and the device finalize
// kernel so both paths round identically.  (svmTrainMain.cpp:282-299)
struct PairUpdate {
  float a_hi_new, a_lo_new, c_hi, c_lo;
};

DPSVM_HD PairUpdate pair_update(float a_hi_old, float a_lo_old, float y_hi, float y_lo, float b_hi,
                                float b_lo, float k_hl, float C, float tau, int clip_mode,
                                bool same) {
#if defined(__clang__)
#pragma clang fp contract(off)  // identical rounding wherever it is inlined
#endif
  float eta = (1.0f + 1.0f) - 2.0f * k_hl;  // K(hi,hi) + K(lo,lo) - 2 K(hi,lo); K(i,i) = 1
  if (!(eta >= tau)) eta = tau;
  float s = y_lo * y_hi;
  float a_lo_new = a_lo_old + (y_lo * (b_hi - b_lo) / eta);
  float a_hi_new;
  if (clip_mode == (int)ClipMode::Box && !same) {
    // Joint box on the line y_hi a_hi + y_lo a_lo = const.  When a_lo hits a
    // bound that comes from a_hi's own bound, a_hi is set to that bound exactly
    // (as LIBSVM does) so round-off cannot leave it a hair inside the box,
    // where it would keep being selected with a zero-length step.
    float L, H;
    float hi_at_L, hi_at_H;  // a_hi value implied when a_lo lands on L / H (-1: none)
    if (y_hi != y_lo) {
      const float dl = a_lo_old - a_hi_old;
      L = dl > 0.f ? dl : 0.f;
      hi_at_L = dl > 0.f ? 0.f : -1.f;
      H = C + dl < C ? C + dl : C;
      hi_at_H = C + dl < C ? C : -1.f;
    } else {
      const float sm = a_lo_old + a_hi_old;
      L = sm - C > 0.f ? sm - C : 0.f;
      hi_at_L = sm - C > 0.f ? C : -1.f;
      H = sm < C ? sm : C;
      hi_at_H = sm < C ? 0.f : -1.f;
    }
    if (a_lo_new <= L) {
      a_lo_new = L;
      a_hi_new = hi_at_L >= 0.f ? hi_at_L : a_hi_old + (s * (a_lo_old - a_lo_new));
    } else if (a_lo_new >= H) {
      a_lo_new = H;
      a_hi_new = hi_at_H >= 0.f ? hi_at_H : a_hi_old + (s * (a_lo_old - a_lo_new));
    } else {
      a_hi_new = a_hi_old + (s * (a_lo_old - a_lo_new));  // NaN-safe: NaN falls here
    }
    a_hi_new = clip01(a_hi_new, 0.0f, C);  // guards fp round-off only
  } else {
    a_hi_new = a_hi_old + (s * (a_lo_old - a_lo_new));
    a_lo_new = clip01(a_lo_new, 0.0f, C);
    a_hi_new = clip01(a_hi_new, 0.0f, C);
  }
  PairUpdate u;
  u.a_hi_new = a_hi_new;
  u.a_lo_new = a_lo_new;
  u.c_hi = (a_hi_new - a_hi_old) * y_hi;
  u.c_lo = (a_lo_new - a_lo_old) * y_lo;
  return u;
}

// Stop test of the reference do/while tail (svmTrainMain.cpp:310).
DPSVM_HD bool gap_open(float b_hi, float b_lo, float eps) { return b_lo > (b_hi + (2.0f * eps)); }

inline float resolve_gamma(float gamma, int d) { return gamma < 0.f ? 1.0f / (float)d : gamma; }

// Row padding for device X: multiples of 16 floats (one MFMA k-step of 4 lanes x float4).
constexpr int kFeatPad = 16;
inline int pad_features(int d) { return (d + kFeatPad - 1) / kFeatPad * kFeatPad; }

// Balanced contiguous sharding (fixes SURVEY Q9: sizes differ by at most 1).
// Reference: svmTrainMain.cpp:367-384.
struct Shard {
  int64_t offset = 0, size = 0;
};
inline Shard shard_of(int64_t n, int rank, int world) {
  int64_t base = n / world, rem = n % world;
  Shard s;
  s.size = base + (rank < rem ? 1 : 0);
  s.offset = rank * base + (rank < rem ? rank : rem);
  return s;
}

// Workgroup geometry of the fused / persistent engines (rows per workgroup, a
// multiple of 256 threads; workgroups per rank).  nl_max = largest shard.
//   cache mode: about `wgs` workgroups (one per CU: the X pass wants every CU);
//   dense mode: ~128 publishers over all ranks, <= 1024 rows per workgroup, more
//   rows (12 register rows per thread, <= 3072) only to keep every poll of the
//   key exchange one batch (world x workgroups <= 256) and <= 256 resident
//   workgroups per rank (profiles/r1_dense_rows_ab.txt).
struct Geometry {
  int64_t rows = 256, groups = 1;
};
inline int64_t geo_round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
inline Geometry make_geometry(int64_t nl_max, int64_t rows_min, int64_t wgs = 256) {
  Geometry g;
  const int64_t per = (nl_max + wgs - 1) / wgs;
  g.rows = std::max<int64_t>(256, geo_round_up(per, 256));
  g.rows = std::max(g.rows, rows_min);
  g.groups = std::max<int64_t>(1, (nl_max + g.rows - 1) / g.rows);
  return g;
}
inline int64_t dense_rows_min(int64_t nl_max, int world) {
  int64_t r = std::min<int64_t>(1024, geo_round_up(std::max<int64_t>(1, nl_max * world / 128), 256));
  if (world * ((nl_max + r - 1) / r) > 256) r = std::max(r, geo_round_up((nl_max * world + 255) / 256, 256));
  if ((nl_max + r - 1) / r > 256) r = geo_round_up((nl_max + 255) / 256, 256);
  return r;
}

}  // namespace dpsvm
