// Internal state of the device-resident SMO solver (one rank = one MI355X).
//
// Reference driver: svmTrainMain.cpp:142-365 + SvmTrain (svmTrain.cu:305-395).
// The solver is split by concern:
//   gpu_setup.hip     X placement, data-parallel policy, cache sizing, geometry,
//                     engine choice (incl. the residency census)
//   gpu_exchange.hip  in-kernel peer exchange buffers (IPC / peer mappings, ping),
//                     small collectives that work on device and host communicators
//   gpu_engines.hip   the iteration engines (seed + block of iterations / rounds)
//   gpu_solve.hip     the timed SMO loop, checkpoints, invariant checks
//   gpu_predict.hip   SV compaction, accuracy, decision values, GpuPredictor,
//                     kernel-level test entry points
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "dpsvm/device_state.hpp"
#include "dpsvm/solver.hpp"
#include "../kernels/kernels.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace gpu {

inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

template <class T>
T* dmalloc(size_t count, size_t* total) {
  void* p = nullptr;
  if (count == 0) count = 1;
  HIP_CHECK(hipMalloc(&p, count * sizeof(T)));
  *total += count * sizeof(T);
  return (T*)p;
}

// The pair a fused engine's last launch updated but has not committed to the
// alpha array yet (its record carries the new alphas): checkpoints apply it.
struct Pending {
  bool valid = false;
  int32_t i_hi = -1, i_lo = -1;
  float a_hi = 0.f, a_lo = 0.f;
  int64_t iter = 0;
  float b_hi = 0.f, b_lo = 0.f;
};

struct Engine;

}  // namespace gpu

struct GpuSolver::Impl {
  SolverParams p;
  Communicator* comm = nullptr;        // the solve's communicator (local when replicated)
  Communicator* outer = nullptr;       // the caller's communicator (== comm unless replicated)
  std::unique_ptr<Communicator> own_comm;
  int device = 0, rank = 0, world = 1;
  int outer_rank = 0, outer_world = 1;
  GpuSetupInfo info;
  hipStream_t stream = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  size_t bytes = 0;

  // device buffers
  float *x = nullptr, *xsq = nullptr, *y = nullptr, *alpha = nullptr, *f = nullptr;
  float* lines = nullptr;
  int32_t *slot_of = nullptr, *key_of = nullptr;
  uint8_t* ref = nullptr;  // CLOCK reference bits
  float *hlines_h = nullptr, *hlines_d = nullptr;  // pinned host tier (host / device view)
  int32_t *hslot_of = nullptr, *hkey_of = nullptr;
  int64_t H = 0;
  uint64_t* partials = nullptr;
  SmoCtrl* ctrl = nullptr;
  SmoStatus* status_h = nullptr;  // host view
  SmoStatus* status_d = nullptr;  // device view
  uint8_t *records = nullptr, *my_record = nullptr;
  uint64_t* pf = nullptr;          // fused engines: two partial buffers [2][2*Gf]
  FusedRec* rf = nullptr;          // dense / persistent engines: two records
  FusedCacheRec* rcf = nullptr;    // fused cache engine: two records
  int32_t* plru_meta = nullptr;    // persistent cache engine: private metadata per workgroup
  int64_t* plru_stats = nullptr;
  // peer exchange: own receive buffer (own allocation, IPC exported), device
  // table of every rank's buffer, IPC mappings to close
  bool xch = false;
  uint64_t* xbuf = nullptr;
  uint64_t** xpeer_d = nullptr;
  int64_t xregion = 0;             // u64 words of the two key parities (zeroed per solve)
  int64_t xstride = kXchGranules;  // u64 slots per exchange entry
  std::vector<void*> xopened;
  std::string xch_diag;
  std::string xch_mem = "none";    // receive-buffer memory kind
  int64_t Gf = 0, RBf = 0;         // fused / persistent geometry: workgroups, rows per workgroup
  // working-set engine (ws_*.hip): round control record, candidate keys
  WsArgs wsa{};
  int ws_q1 = 0;                    // the one-block rounds' q_max (multi-block rounds may use smaller blocks)
  WsCtrl* wsctrl = nullptr;
  uint64_t* wscand = nullptr;
  float* wsdfs = nullptr;           // multi-block rounds: d_f [nl], d_alpha [n], line-search partials [G][2]
  float* wsdalpha = nullptr;
  double* wspart = nullptr;
  uint64_t* wssorted = nullptr;     // multi-block merge: candidate keys per side, ascending
  float* wssub = nullptr;          // q_max x q_max sub-Gram + [3][kWsMax] f / alpha / y of the working set
  float *wsxq = nullptr, *wsxqsq = nullptr;  // partitioned X, cache mode: the misses' X rows / norms
  int32_t* wsiota = nullptr;                  //   (their GEMM row indices: 0..q_max-1)
  // fp16 split operands of the GEMMs (rbf_gemm_split.hip), rebuilt by every
  // solve inside the timed region: xs / xsh = the x_rows rows of x; wsxs /
  // wsxsh = the packed misses of partitioned ws-cache rounds
  bool gram_split = false;
  float gram_cold_tau = 0.f;  // > 0: the resident split Gram is adaptive (gram_adapt, docs/DESIGN.md §13)
  void* xs = nullptr;
  int32_t* xsh = nullptr;
  void* wsxs = nullptr;
  int32_t* wsxsh = nullptr;
  std::vector<uint8_t> h_wscand;   // host staging of the per-round collectives (host communicators)
  std::vector<float> h_wssub, h_wsxq;
  std::vector<uint8_t> h_wspart;
  uint64_t* stamps = nullptr;      // DPSVM_STAMPS diagnostics
  std::string stamps_path;
  std::vector<uint64_t> h_partials;  // host staging for host-memory communicators
  std::vector<uint8_t> h_records;

  SmoArgs args{};
  float gamma = 0.f;
  int64_t n = 0, nl = 0, off = 0, x_rows = 0, G = 0, ldl = 0, L = 0;
  int d = 0, dp = 0;
  bool replicated = true, dense = false;
  EngineKind kind = EngineKind::Chain;
  std::unique_ptr<gpu::Engine> engine;
  std::vector<float> h_y;

  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  // multi-block working-set rounds: the one-block round graph the engine
  // switches to once the adaptive block count reached 1 (built on first use)
  hipGraphExec_t gexec1 = nullptr;
  hipGraph_t graph1 = nullptr;
  // ws-cache rounds with the kernel rows recomputed (ws_recompute.hip)
  bool ws_recompute = false;

  ~Impl();

  bool collectives() const { return world > 1 || p.force_collectives; }
  bool device_comm() const { return world == 1 || comm->device_memory(); }
  bool fused() const { return kind != EngineKind::Chain; }
  bool persistent() const { return kind == EngineKind::PersistDense || kind == EngineKind::PersistCache; }
  bool working_set() const { return kind == EngineKind::WsDense || kind == EngineKind::WsCache; }
  // a working-set round still runs communicator collectives (candidates and
  // sub-Gram travel through the in-kernel peer exchange when it is set up;
  // partitioned-X ws-cache always sums its packed miss rows)
  bool ws_round_collectives() const {
    return collectives() && (wsa.xpeer == nullptr || (kind == EngineKind::WsCache && !replicated));
  }
  // device addresses inside the working-set control record (cache mode GEMM operands)
  int32_t* wsctrl_miss_row() const { return wsctrl ? wsctrl->miss_row : nullptr; }
  int32_t* wsctrl_miss_line() const { return wsctrl ? wsctrl->miss_line : nullptr; }
  int32_t* wsctrl_n_miss() const { return wsctrl ? &wsctrl->n_miss : nullptr; }

  SmoStatus read_status() const;
  // bound of the next wait_event (0: p.watchdog_s).  At world > 1 the solve
  // loop derives it from the measured block times (a dead peer is detected in
  // seconds, not at the 1800 s default)
  double wd_limit = 0.0;
  void init_ctrl(int64_t iter0, float b_hi, float b_lo);
  void wait_event(hipEvent_t e);

  // ---- gpu_exchange.hip ----
  // element-wise MIN over ranks of u64 device buffer (device or host communicator)
  void allreduce_keys(uint64_t* buf, int64_t count);
  void allgather_bytes(const void* send, void* recv, size_t bytes);  // host buffers
  // every rank of `c` agrees: true only if `mine` is true everywhere
  bool all_agree(bool mine, Communicator* c, int w);
  // region_words: u64 words of the exchange region (0: the SMO engines' key parities)
  bool setup_exchange(int64_t region_words = 0);
  // residency census of the chosen persistent engine (collective: agreed)
  bool census(EngineKind k);

  // ---- gpu_engines.hip ----
  void enqueue_iteration(int k);  // one iteration of a launch-per-iteration engine
  void build_graph(int iters);

  // ---- gpu_solve.hip ----
  void snapshot(const SmoStatus& st);
  std::vector<float> gather_f();
};

namespace gpu {

// One iteration engine.  prepare() resets engine state before the timed
// region; seed() runs at the start of the timed region (the
// dense engines compute the resident Gram there) and leaves the device state
// one block away from iteration iter0 + 1; run_block() enqueues B iterations
// (early-exit once the status record says done); pending() reports a pair
// whose alphas still sit in a record.
struct Engine {
  virtual ~Engine() = default;
  virtual EngineKind kind() const = 0;
  virtual int block(const SolverParams& p) const = 0;
  virtual void prepare(GpuSolver::Impl&) {}  // per-solve state reset, before the timed region
  virtual void seed(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo, SolveResult& res) = 0;
  virtual void run_block(GpuSolver::Impl& m, int B) = 0;
  // run_block(m, B) also takes B < block(): the last rounds before a predicted
  // convergence go one at a time (the host polls one launch behind, so the
  // rounds after convergence in the launches already queued are early exits)
  virtual bool shortens() const { return false; }
  // the status of the completed launches, `launched` iterations / rounds
  // enqueued so far (the one in flight included): engines may change what they
  // enqueue next — identically on every rank, so only from values that
  // completed launches wrote
  virtual void observe(GpuSolver::Impl&, const SmoStatus&, int64_t /*launched*/) {}
  virtual Pending pending(GpuSolver::Impl&) { return {}; }
  virtual double gram_seconds() { return 0.0; }
};

std::unique_ptr<Engine> make_engine(EngineKind k);

// ---- helpers shared by the production engines (gpu_engines.hip) and the
// quarantined pair-at-a-time cache / chain engines (gpu_engines_pairq.hip) ----
inline FusedRec seed_record(int64_t iter0, float b_hi, float b_lo) {
  FusedRec r;
  r.i_hi = r.i_lo = -1;  // no pending pair
  r.a_hi = r.a_lo = 0.f;
  r.iter = (int32_t)iter0;
  r.done = kRunning;
  r.b_hi = b_hi;
  r.b_lo = b_lo;
  return r;
}

inline Pending pending_of(const FusedRec& r) {
  Pending q;
  q.valid = true;
  q.i_hi = r.i_hi;
  q.i_lo = r.i_lo;
  q.a_hi = r.a_hi;
  q.a_lo = r.a_lo;
  q.iter = r.iter;
  q.b_hi = r.b_hi;
  q.b_lo = r.b_lo;
  return q;
}

// Blocks of launch-per-iteration engines: a hipGraph when the communicator is
// stream-ordered (or absent), else eager launches.
inline void run_launches(GpuSolver::Impl& m, int B) {
  if (m.gexec) {
    HIP_CHECK(hipGraphLaunch(m.gexec, m.stream));
  } else {
    for (int i = 0; i < B; ++i) m.enqueue_iteration(i);
  }
}

inline void maybe_graph(GpuSolver::Impl& m, int B) {
  const bool graphs = m.p.use_graph && m.device_comm() && !m.p.sync_debug && !sync_debug_env();
  if (!graphs) return;
  try {
    m.build_graph(B);
  } catch (const std::exception& e) {
    if (m.p.verbose) fprintf(stderr, "[dpsvm] graph capture failed (%s); eager launches\n", e.what());
  }
}

inline int even_block(const SolverParams& p) {
  // fused engines ping-pong two buffers: the parity must survive graph replays
  return std::max(2, (std::max(1, p.graph_block) + 1) / 2 * 2);
}

// The pair-at-a-time cache / partitioned-X engines (persistent-cache,
// fused-cache, chain: kQuarantineTable in device_state.hpp) are not part of
// the production module: they live in a plugin (dpsvm_amd/_pairq*.so; linked
// into the CLIs) that registers this table when it is loaded (engines="all").
// Production code reaches them only through quarantine().
struct QuarantineOps {
  std::unique_ptr<Engine> (*make_engine)(EngineKind k);
  void (*enqueue_iteration)(GpuSolver::Impl& m, int k);  // fused-cache / chain: one iteration
  // facts of the engine choice (gpu_setup.hip) and residency (census)
  bool (*fused_lru_supported)(int dp);
  bool (*persist_lru_supported)(int dp, int fused_rows, int fused_G);
  int64_t (*plru_stride_words)(int64_t n, int64_t L);
  int (*persist_lru_blocks_per_cu)(const SmoArgs& a);
  void (*persist_lru_census)(const SmoArgs& a, int groups, hipStream_t s);
  void (*preload)(hipStream_t s);
  // kernel-level test entry points (tests/test_kernels_gpu.py)
  void (*smo_rows)(const SmoArgs& a, hipStream_t s);
  void (*smo_step)(const SmoArgs& a, hipStream_t s);
  void (*xpass_rows)(const SmoArgs& a, const int* keys, int n_new, hipStream_t s);
};
void register_quarantine(const QuarantineOps* ops);
const QuarantineOps* quarantine();     // nullptr: the plugin is not loaded
const QuarantineOps& need_quarantine(const char* what);  // fails loudly when not loaded

}  // namespace gpu
}  // namespace dpsvm
