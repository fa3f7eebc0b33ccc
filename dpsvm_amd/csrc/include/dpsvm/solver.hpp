// SMO solvers (CPU oracle + MI355X device-resident), predictors, checkpoints.
//
// Reference call stacks: SURVEY §3.1 (GPU/MPI svmTrain), §3.2 (CPU seq),
// §3.3 (seq_test predictor).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "dpsvm/comm.hpp"
#include "dpsvm/common.hpp"
#include "dpsvm/io.hpp"

namespace dpsvm {

struct Progress {
  int64_t iter;
  float b_hi, b_lo;
  double elapsed;
  int64_t hits, misses;
};
using ProgressFn = std::function<void(const Progress&)>;

// Checkpoint: everything needed to continue SMO (alpha, f, iteration, last b's).
struct Checkpoint {
  int64_t n = 0;
  int d = 0;
  float C = 0, gamma = 0, eps = 0;
  int clip = 0;
  int64_t iter = 0;
  float b_hi = 0, b_lo = 0;
  std::vector<float> alpha;  // n
  std::vector<float> f;      // n (may be empty -> recomputed from alpha)
};
void write_checkpoint(const std::string& path, const Checkpoint& ck);
Checkpoint read_checkpoint(const std::string& path);
// Rejects a checkpoint written for another problem: a different n, d, C, gamma
// or clip mode (its f would be inconsistent with this kernel, its alphas may
// violate this box).  eps and max_iter may differ.
void check_resume(const Checkpoint& ck, int64_t n, int d, const SolverParams& p, float gamma);

// ---------------------------------------------------------------------------
// CPU solver (C10 seq / the no-GPU path and the test oracle).  X is replicated,
// f and the kernel-row cache are sharded by `comm` (nullptr = one rank).
// ---------------------------------------------------------------------------
SolveResult solve_cpu(const Dataset& ds, const SolverParams& p, Communicator* comm = nullptr,
                      const Checkpoint* resume = nullptr, const ProgressFn& progress = {});

// Decision values d(x) = sum_sv alpha y K(sv,x) - b  (svmTrain.cu:646-658)
std::vector<float> decision_cpu(const Model& m, const float* x, int64_t n, int d, int threads = 0);
// fraction of rows with sign(decision) == y  (>= 0 -> +1)
double accuracy_from_decision(const std::vector<float>& dec, const float* y, int64_t n);

// ---------------------------------------------------------------------------
// Device-resident solver (one rank = one GPU).  Implementation: smo_gpu.hip.
// ---------------------------------------------------------------------------
struct GpuSetupInfo {
  int device = 0;
  std::string device_name;
  int64_t n = 0, n_local = 0, offset = 0;
  int d = 0, dp = 0;
  bool x_replicated = true;
  int64_t cache_lines = 0, host_cache_lines = 0;
  int blocks = 0;
  size_t bytes_device = 0;  // device memory held now (lines lent out by release_cache() do not count)
  std::string iteration;  // engine: "persistent-dense" | "fused-dense" | "persistent-cache" | "fused-cache" | "chain"
  std::string exchange;   // per-iteration key exchange: "none" | "allreduce" | "peer" | "loopback" (1 rank)
  std::string exchange_mem = "none";  // peer exchange receive buffer: "uncached" (across devices) | "coarse"
  // working-set engines: how a round's candidate lists, sub-Gram entries and
  // line-search partials cross ranks — "peer" (in-kernel pushes, no collective),
  // "collectives" (all-gather / sum all-reduce per round), "none" (one rank)
  std::string ws_exchange = "none";
  std::string dp_policy = "shard";    // "shard" (rows split over ranks) | "replicate" (every rank solves it all)
  int64_t rows_per_group = 0, groups = 0;  // fused / persistent geometry
  int poll_batch = 0;                 // publications per lane per poll round (peer exchange)
  int cus = 0, blocks_per_cu = 0;     // residency of the persistent kernel (occupancy API)
  std::string census = "n/a";         // residency census of the persistent grid: "ok" | "failed" | "n/a"
  std::string engine_note;            // why the engine was chosen / refused (fallbacks)
  std::string cache_note;             // cache_lines (-s N) raised to the working-set cache's minimum
  int ws_wss = 0;                     // working-set engines: sub-problem pair choice (1 first, 2 second order)
  std::string ws_rounds = "none";     // working-set engines: "graph" (launches per round) or "persistent"
  std::string ws_rows = "none";       // ws engines' kernel rows: "gram" (resident), "cache" (row cache), "recompute"
  std::string xch_selftest;            // peer exchange setup self test: "rank r: mapped=1 ping=1" or why refused
  std::string comm_kind;               // communicator backend: local | rccl | thread | callback
  int ws_blocks = 0, ws_q_max = 0;     // working-set rounds: blocks per round x rows per block (the union)
  std::string gram = "f32";           // Gram / kernel-row GEMM arithmetic: "f32" or "split-f16" (rbf_gemm_split.hip)
};

// true once the pair-cache plugin (libdpsvm_pairq.so, or the CLIs that link it)
// registered the quarantined pair-at-a-time cache / partitioned-X engines
bool quarantine_loaded();

class GpuSolver {
 public:
  // x: host row-major [n_x][d] where n_x = n (replicated) or the rank's shard
  // rows (partitioned, x_mode=2).  y: host, global n labels.
  GpuSolver(const SolverParams& p, Communicator* comm, int device);
  ~GpuSolver();
  GpuSolver(const GpuSolver&) = delete;
  GpuSolver& operator=(const GpuSolver&) = delete;

  GpuSetupInfo setup(const float* x, int64_t n_x_rows, int64_t n, int d, const float* y);
  SolveResult solve(const Checkpoint* resume = nullptr, const ProgressFn& progress = {});
  // After solve(): distributed training accuracy (each rank predicts its shard)
  double train_accuracy(const SolveResult& r);
  // decision values for rows of a host matrix using the trained SVs (any rank)
  std::vector<float> decision(const SolveResult& r, const float* x, int64_t n, int d);
  // after solve(): this rank's gradient f_j = sum_i alpha_i y_i K(i, j) - y_j
  // as the solver maintained it (its local rows)
  std::vector<float> gradient() const;
  // after solve(): the whole gradient on every rank (the shards all-gathered;
  // a collective at world > 1)
  std::vector<float> gradient_all();
  // the stop tolerance of the next solve() (kernel arguments updated, captured graphs rebuilt)
  void set_eps(float eps);
  // free the kernel-row cache / resident Gram until the next solve() (which
  // allocates it again): ShrinkingSolver lends its memory to a shrunk phase
  void release_cache();
  const GpuSetupInfo& info() const;
  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

// Shrinking (LIBSVM's heuristic, as problem reduction): phases of the device
// solver on the active rows only — free alphas and bounded ones that can still
// violate (f below b_lo on the up side, above b_hi on the low side) — each to
// its own stop test, then the inactive rows' gradient is brought up to date by
// one predict GEMM over the phase's alpha changes and the reference's stop
// test is evaluated on the whole problem.  x, y: host, all n rows (on every
// rank).  comm (world > 1): every rank calls; a phase is a multi-rank solve
// (dp policy of p), the inactive-row update split over the ranks.
SolveResult solve_shrinking(const SolverParams& p, int device, const float* x, int64_t n, int d, const float* y,
                            const Checkpoint* resume = nullptr, const ProgressFn& progress = {},
                            Communicator* comm = nullptr);

// The same, with the whole-problem solver set up once (X upload, cache or Gram
// sizing: the setup a plain solve does before its timed region) and kept for
// every whole-problem phase and every solve(); the shrunk phases' solvers use
// the memory it leaves (cache_frac).  x, y (host) must outlive the object.
class ShrinkingSolver {
 public:
  ShrinkingSolver(const SolverParams& p, Communicator* comm, int device);
  ~ShrinkingSolver();
  GpuSetupInfo setup(const float* x, int64_t n, int d, const float* y);
  SolveResult solve(const Checkpoint* resume = nullptr, const ProgressFn& progress = {});
  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

// shrink="auto" (library, svmTrain and bench default): shrinking phases where
// they pay — one GPU, working-set rounds, and a Gram that does not fit the
// device's cache budget (the ws-cache regime: covtype-shape 581k x 54).  On a
// resident Gram (the headline) a phase only adds setup work; measured in
// profiles/r4_shrink_auto_*.txt.
bool shrink_auto(const SolverParams& p, int64_t n, int d, int device, Communicator* comm = nullptr);

// Stand-alone GPU predictor (svmTest GPU path): model SVs resident on device,
// decision values of a host or device matrix via the MFMA predict kernel.
class GpuPredictor {
 public:
  // precision: 0 auto (split-operand GEMM from 128 padded features), 1 f32-input MFMA, 2 split-operand
  GpuPredictor(const Model& m, int device, int precision = 0);
  ~GpuPredictor();
  std::vector<float> decision(const float* x_host, int64_t n, int d);
  // device pointers, stream = hipStream_t as void*
  void decision_device(const float* x_dev, int64_t n, int d, int ld, float* out_dev, void* stream);
  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

// Low-level kernel entry points exposed for unit tests (device pointers).
namespace kernels {
void row_sqnorm(const float* x, int64_t n, int d, int ld, float* out, void* stream);
// known-bytes 16-B streaming read (FETCH_SIZE probe, bench/fetch_probe.py)
void stream_read(const void* x, int64_t bytes, float* out, int blocks, void* stream);
// K[q][j] = exp(-gamma * max(|x_j|^2 + |w_q|^2 - 2 x_j.w_q, 0)) for q < nq <= 16
void rbf_rows(const float* x, const float* xsq, int64_t n, int ld, const float* w, const float* wsq,
              int nq, float gamma, float* out, int64_t out_ld, void* stream);
// per-block selection partials over f/alpha/y (keys as in common.hpp)
void select_partials(const float* f, const float* alpha, const float* y, int64_t n, int64_t offset,
                     float C, uint64_t* partials, int* blocks_out, void* stream);
void predict(const float* x, const float* xsq, int64_t n, int ld, const float* sv,
             const float* svsq, const float* coef, int64_t nsv, int sv_ld, float gamma, float b,
             float* dec, void* stream);
int64_t compact_nonzero(const float* alpha, int64_t n, int* idx_out, void* stream);
// Gram block K[i][j] = K(a_i, b_j) (dense-mode GEMM; symmetric: b == a)
void rbf_gram(const float* a, const float* asq, int64_t m, const float* b, const float* bsq, int64_t n, int ld,
              float gamma, float* out, int64_t out_ld, bool symmetric, void* stream);
// the cache engines' X pass: out[q][j] = K(x_keys[q], x_j), q < nq <= 16, j < n
// (x: [rows >= G*rows_per_group][ld], xsq likewise; out rows >= G*rows_per_group)
// the working-set cache engine's row GEMM: out[out_rows[i]][j] = K(x[rows[i]], x_j), i < m, j < n
void rbf_rows_indexed(const float* x, const float* xsq, int64_t n, int ld, const int* rows, int m, float gamma,
                      float* out, int64_t out_ld, const int* out_rows, void* stream, bool split = false);
// diagnostics: the split row GEMM alone (operands split once), reps launches
// event-timed; returns ms per launch (bench/rows_probe.py)
std::vector<float> rbf_rows_indexed_split_bench(const float* x, const float* xsq, int64_t n, int ld, const int* rows,
                                                int m, float gamma, float* out, int64_t out_ld, const int* out_rows,
                                                int reps, void* stream);
// the same two GEMMs on fp16 MFMA over split operands (rbf_gemm_split.hip)
void rbf_gram_split(const float* a, const float* asq, int64_t m, const float* b, const float* bsq, int64_t n, int ld,
                    float gamma, float* out, int64_t out_ld, bool symmetric, void* stream,
                    float cold_tau = 0.f);
// the adaptive Gram of the calling thread's last rbf_gram_split / solve: (one-product tiles, hot tiles) or (-1, -1)
std::pair<int64_t, int64_t> gram_adapt_last();
void xpass_rows(const float* x, const float* xsq, int64_t n, int ld, const int* keys, int nq, float gamma,
                float* out, int64_t out_ld, int rows_per_group, void* stream);
// the fused / persistent engines' selection: per workgroup of rows_per_group rows
// the (up, low) keys of its rows -> keys_out[2 * groups]
void fused_select(const float* f, const float* alpha, const float* y, int64_t n, float C, int rows_per_group,
                  uint64_t* keys_out, void* stream);

// ---- working-set kernels (ws_*.hip), one launch each on crafted state
// (host vectors in and out; ws_kernel_entry.hip).  Reference counterparts:
// the selection / update functors svmTrain.cu:41-137, the pair rule
// svmTrainMain.cpp:255-299. ----
// ws_merge_multi: cand = [G][2][kWsCand] per-list keys (up, low), the previous
// union (newest first), the adaptive block count p_act of `blocks`
struct WsMergeProbe {
  std::vector<int32_t> uidx;  // the union, newest first
  std::vector<int32_t> idx;   // [blocks][q_max] block layout (-1: unused)
  std::vector<int32_t> qb;    // rows per block
  float b_hi = 0.f, b_lo = 0.f;
  int done = 0, p_round = 0;
};
WsMergeProbe ws_merge_multi_probe(const std::vector<uint64_t>& cand, int G, int blocks, int p_act, int q_max,
                                  int n_new, float eps, const std::vector<int32_t>& prev_union, int64_t iter,
                                  int64_t max_iter);
// ws_solve: P blocks; block p = qb[p] rows with sub-Gram K[p] ([q_max][q_max]),
// f / alpha / y (row a of block p is global row p q_max + a)
struct WsSolveProbe {
  std::vector<float> alpha;       // [P * q_max] after the solve (untouched rows 0)
  std::vector<int32_t> steps;     // pair steps per block
  std::vector<int32_t> apply_idx; // changed rows per block segment (concatenated, block order)
  std::vector<float> apply_coef;  // their (alpha_new - alpha_old) y
  std::vector<int32_t> nab;       // changed rows per block
  int64_t iter = 0, outer = 0, p1_round = 0;
  int done = 0, p_act = 0;
};
WsSolveProbe ws_solve_probe(const std::vector<float>& K, const std::vector<float>& f, const std::vector<float>& alpha,
                            const std::vector<float>& y, const std::vector<int32_t>& qb, int q_max, int blocks,
                            int p_round, float C, int clip, float eps, float rel, float eps_floor, float tau,
                            float b_hi, float b_lo, int inner_max, int64_t iter0, int64_t max_iter, int wss = 1);
// ws_select: the f update of a round's alpha changes (apply rows: lines into
// gram [L][ldg], coefficients) and the per-workgroup candidates.  blocks == 1:
// the one-pass kernel; blocks > 1: pass 1 (d_f, line-search partials) and pass 2
// (t, f += t d_f, alpha fix-up, candidates) with p_round blocks this round.
struct WsSelectProbe {
  std::vector<float> f, alpha, dalpha, dfs;
  std::vector<double> part;      // [G][2] d'Qd, g'd partials (two-pass mode)
  std::vector<uint64_t> cand;    // [G][2][kWsCand]
  int G = 0, rpt = 0, p_act = 0, n_damped = 0, nonfinite = 0;
  int p1G = 0;                   // pass-1 groups (= G; the wide pass 1: ceil(n / 1024)); part is [p1G][ks][2]
  float t = 1.f;
  int64_t p1_round = 0;
  std::vector<float> pass1_us;  // reps > 0: event times of repeated pass-1 launches
};
WsSelectProbe ws_select_probe(const std::vector<float>& gram, int64_t L, int64_t ldg, const std::vector<float>& f,
                              const std::vector<float>& alpha, const std::vector<float>& y,
                              const std::vector<float>& dalpha, const std::vector<int32_t>& apply_line,
                              const std::vector<float>& apply_coef, const std::vector<int32_t>& nab, int blocks,
                              int p_round, int p_act, int q_max, float C, int64_t outer, int ks = 0,
                              int reps = 0, bool wide = false);
}  // namespace kernels

int device_count();
std::string device_name(int dev);

}  // namespace dpsvm
