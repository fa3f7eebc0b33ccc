// Shrinking for the device solver, as problem reduction (one GPU, or every
// rank of a communicator running the same phases on its share).
//
// LIBSVM's shrinking heuristic in the reference's f-notation (f_j = sum_i
// alpha_i y_i K(i, j) - y_j, b_hi = min f over I_up, b_lo = max f over I_low;
// svmTrain.cu:41-95): a row whose alpha sits on a bound can only take part in
// a violating pair from one side — an up-only row (alpha = 0, y = +1 or
// alpha = C, y = -1) when f_j < b_lo, a low-only row (alpha = 0, y = -1 or
// alpha = C, y = +1) when f_j > b_hi.  Rows failing that test are shrunk: the
// reduced problem keeps the free rows and the rows that can still violate,
// with the shrunk alphas fixed (their contribution is already in every f).
//
// On the device the win is a smaller problem, not a masked one: every round of
// the working-set engines streams its changed rows' kernel lines over all rows
// (the f update), and the reduced problem's lines are |A| long (often short
// enough to make its Gram resident: ws-dense instead of ws-cache).  So a phase
// is a fresh GpuSolver on the active rows, resumed from the current alphas and
// gradient; afterwards the inactive rows' gradient is brought up to date by
// one predict GEMM over the phase's alpha changes
//     f_j += sum_{i changed} (alpha'_i - alpha_i) y_i K(i, j)     (j inactive)
// — the same incremental form the solver maintains, so no from-scratch
// recomputation (whose fp32 cancellation error with C = 2048 would exceed eps)
// — and the reference's stop test !(b_lo > b_hi + 2 eps) (svmTrainMain.cpp:310)
// is evaluated on the whole problem.  Phase 0 solves the whole problem to a
// loose tolerance; the last phase, if the shrunk ones keep failing the global
// test, solves the whole problem to eps.
//
// With a communicator (world > 1, X replicated): every rank runs this host
// loop on identical state.  A phase is one multi-rank GpuSolver (rows sharded
// or replicated by the dp policy), its gradient all-gathered; the inactive
// rows' update is split over the ranks (each predicts its slice of them) and
// all-gathered, so every rank continues from the same bits.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <memory>

#include <hip/hip_runtime.h>

#include "dpsvm/device_state.hpp"
#include "dpsvm/solver.hpp"
#include "../kernels/kernels.hpp"
#include "../runtime/hip_check.hpp"
#include "../runtime/trace.hpp"

namespace dpsvm {

namespace {

struct Extremes {
  float b_hi = 0.f, b_lo = 0.f;
  bool ok = false;
};

Extremes extremes(const std::vector<float>& f, const std::vector<float>& a, const float* y, float C) {
  Extremes e;
  float hi = INFINITY, lo = -INFINITY;
  for (size_t j = 0; j < f.size(); ++j) {
    if (in_up(a[j], y[j], C) && f[j] < hi) hi = f[j];
    if (in_low(a[j], y[j], C) && f[j] > lo) lo = f[j];
  }
  e.b_hi = hi;
  e.b_lo = lo;
  e.ok = std::isfinite(hi) && std::isfinite(lo);
  return e;
}

// rows that can still take part in a violating pair (LIBSVM's shrinking test)
std::vector<int64_t> active_rows(const std::vector<float>& f, const std::vector<float>& a, const float* y, float C,
                                 const Extremes& e) {
  std::vector<int64_t> act;
  for (int64_t j = 0; j < (int64_t)f.size(); ++j) {
    const bool up = in_up(a[j], y[j], C), low = in_low(a[j], y[j], C);
    const bool keep = (up && low) || (up && f[j] < e.b_lo) || (low && f[j] > e.b_hi);
    if (keep) act.push_back(j);
  }
  return act;
}

std::vector<float> gather_rows(const float* x, int d, const std::vector<int64_t>& rows) {
  std::vector<float> out(rows.size() * (size_t)d);
  for (size_t k = 0; k < rows.size(); ++k) std::copy(x + rows[k] * d, x + rows[k] * d + d, out.begin() + k * d);
  return out;
}

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// MIN over ranks of a flag (every rank must call)
bool comm_all(Communicator* comm, bool mine) {
  if (!comm || comm->size() == 1) return mine;
  uint64_t v = mine ? 1ull : 0ull;
  if (comm->device_memory()) {
    uint64_t* d = nullptr;
    hipStream_t st = nullptr;
    HIP_CHECK(hipStreamCreate(&st));
    HIP_CHECK(hipMalloc((void**)&d, 8));
    HIP_CHECK(hipMemcpy(d, &v, 8, hipMemcpyHostToDevice));
    comm->allreduce_min_u64(d, 1, st);
    HIP_CHECK(hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, st));
    sync_collective(comm, st, "shrink agreement");
    (void)hipFree(d);
    (void)hipStreamDestroy(st);
  } else {
    comm->allreduce_min_u64(&v, 1, nullptr);
  }
  return v == 1ull;
}

// This rank's slice of X resident on the device for the inactive rows' update
// (uploaded once: no host gather of the inactive rows per phase), with the
// decision buffer and a stream.
struct XSlice {
  int device = 0, dp = 0;
  Shard s;
  float* x = nullptr;
  float* out = nullptr;
  hipStream_t st = nullptr;
  XSlice(const float* xh, int64_t n, int d, int dev, int rank, int world) : device(dev), dp(pad_features(d)) {
    s = shard_of(n, rank, world);
    HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int64_t rows = (s.size + 127) / 128 * 128 + 128;  // whole 128-row tiles for the GEMM
    HIP_CHECK(hipMalloc((void**)&x, (size_t)rows * dp * 4));
    HIP_CHECK(hipMalloc((void**)&out, (size_t)rows * 4));
    HIP_CHECK(hipMemsetAsync(x, 0, (size_t)rows * dp * 4, st));
    if (s.size > 0)
      HIP_CHECK(hipMemcpy2DAsync(x, (size_t)dp * 4, xh + (size_t)s.offset * d, (size_t)d * 4, (size_t)d * 4,
                                 (size_t)s.size, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
  }
  ~XSlice() {
    (void)hipSetDevice(device);
    if (x) (void)hipFree(x);
    if (out) (void)hipFree(out);
    if (st) (void)hipStreamDestroy(st);
  }
  // df[s.offset ..) = sum_i dm.alpha_i dm.y_i K(x_i, x_j) for this rank's rows j
  void update(const Model& dm, int d, int precision, std::vector<float>& df) {
    if (s.size == 0) return;
    GpuPredictor pr(dm, device, precision);
    pr.decision_device(x, s.size, d, dp, out, st);
    HIP_CHECK(hipMemcpy(df.data() + s.offset, out, (size_t)s.size * 4, hipMemcpyDeviceToHost));
  }
};

// every rank's slice shard_of(n, r, world) of a length-n vector, all-gathered
// into `out` (each rank filled only its own slice)
void comm_allgather_slices(Communicator* comm, std::vector<float>& out) {
  const int world = comm->size(), rank = comm->rank();
  const int64_t n = (int64_t)out.size(), ld = (n + world - 1) / world;
  const Shard me = shard_of(n, rank, world);
  std::vector<float> loc((size_t)ld, 0.f), all((size_t)ld * world);
  std::copy(out.begin() + me.offset, out.begin() + me.offset + me.size, loc.begin());
  if (comm->device_memory()) {
    float* gb = nullptr;
    hipStream_t st = nullptr;
    HIP_CHECK(hipStreamCreate(&st));
    HIP_CHECK(hipMalloc((void**)&gb, (size_t)ld * world * 4));
    HIP_CHECK(hipMemcpy(gb + (size_t)rank * ld, loc.data(), (size_t)ld * 4, hipMemcpyHostToDevice));
    comm->allgather(gb + (size_t)rank * ld, gb, (size_t)ld * 4, st);
    HIP_CHECK(hipMemcpyAsync(all.data(), gb, all.size() * 4, hipMemcpyDeviceToHost, st));
    sync_collective(comm, st, "inactive-row all-gather");
    (void)hipFree(gb);
    (void)hipStreamDestroy(st);
  } else {
    comm->allgather(loc.data(), all.data(), (size_t)ld * 4, nullptr);
  }
  for (int r = 0; r < world; ++r) {
    const Shard s = shard_of(n, r, world);
    std::copy(all.begin() + (size_t)r * ld, all.begin() + (size_t)r * ld + s.size, out.begin() + s.offset);
  }
}

constexpr float kPhase0EpsScale = 50.f;   // phase 0: the whole problem to 50 eps
constexpr double kShrinkMaxFrac = 0.6;    // shrink only if the active set is at most 60% of the rows
constexpr int kMaxPhases = 8;             // then the whole problem to eps

}  // namespace

struct ShrinkingSolver::Impl {
  SolverParams p0, p;
  Communicator* comm = nullptr;
  int device = 0, world = 1, rank = 0;
  const float* x = nullptr;
  int64_t n = 0;
  int d = 0;
  float gamma = 0.f;
  std::vector<float> y;
  std::unique_ptr<GpuSolver> whole;  // every whole-problem phase (set up once)
  GpuSetupInfo info;
  std::unique_ptr<XSlice> xsl;  // this rank's X rows on the device, from the first shrunk phase on
};

ShrinkingSolver::ShrinkingSolver(const SolverParams& p0, Communicator* comm, int device) : impl_(new Impl) {
  auto& m = *impl_;
  m.world = comm ? comm->size() : 1;
  m.rank = comm ? comm->rank() : 0;
  DPSVM_CHECK(m.world == 1 || p0.x_mode != 2, "shrinking: every rank holds X (x_mode partitioned is not supported)");
  m.comm = m.world > 1 ? comm : nullptr;
  m.device = device;
  m.p0 = p0;
  m.p = p0;
  m.p.checkpoint_every = 0;  // the phases' own solvers do not checkpoint: the whole problem's state is
                             // written after every phase instead
  if (m.p.solver == 0) m.p.solver = 2;  // the phases are parts of a large problem: working-set rounds at any size
  // the inactive rows' gradient comes from the predict GEMM: the phases' kernel
  // values must come from the same arithmetic (f32 MFMA and split-operand
  // values differ by ~1e-5, which C-sized alpha changes turn into gradient
  // drift) — auto: the split GEMMs for both (the working-set engines' default:
  // round 3 ran the phases on the f32 GEMMs, 2x slower on synthetic-2m and
  // 1.4x per round on covtype's miss rows)
  if (m.p.gram_precision == 0) m.p.gram_precision = 2;
}

ShrinkingSolver::~ShrinkingSolver() = default;

GpuSetupInfo ShrinkingSolver::setup(const float* x, int64_t n, int d, const float* y_in) {
  auto& m = *impl_;
  DPSVM_CHECK(n >= 2 && d >= 1, "shrinking: need at least 2 samples and 1 feature");
  m.x = x;
  m.n = n;
  m.d = d;
  m.gamma = resolve_gamma(m.p.gamma, d);
  m.p.gamma = m.gamma;
  m.y.resize((size_t)n);
  for (int64_t j = 0; j < n; ++j) m.y[j] = y_in[j] > 0 ? 1.f : -1.f;
  m.xsl.reset();
  m.whole.reset();
  m.whole.reset(new GpuSolver(m.p, m.comm, m.device));
  m.info = m.whole->setup(x, n, n, d, m.y.data());
  return m.info;
}

SolveResult ShrinkingSolver::solve(const Checkpoint* resume, const ProgressFn& progress) {
  auto& m = *impl_;
  DPSVM_CHECK(m.whole != nullptr, "ShrinkingSolver::solve before setup");
  const SolverParams& p = m.p;
  const int64_t n = m.n;
  const int d = m.d, world = m.world, rank = m.rank;
  const float* x = m.x;
  const float gamma = m.gamma;
  const float C = p.C;
  const std::vector<float>& y = m.y;
  const double t_start = now();
  std::vector<float> alpha((size_t)n, 0.f), f((size_t)n);
  int64_t iters = 0;
  bool have_f = false;
  if (resume) {
    check_resume(*resume, n, d, p, gamma);
    alpha = resume->alpha;
    iters = resume->iter;
    if ((int64_t)resume->f.size() == n) {
      f = resume->f;
      have_f = true;
    }
  }
  if (!have_f && !resume)
    for (int64_t j = 0; j < n; ++j) f[j] = -y[j];

  SolveResult res;
  res.world = world;
  int phases = 0;
  int64_t rounds = 0, rows_computed = 0;
  double t_gram = 0.0;
  std::vector<int64_t> act;  // empty: every row
  bool full_to_eps = false;
  while (true) {
    const bool all = act.empty() || (int64_t)act.size() == n;
    const int64_t na = all ? n : (int64_t)act.size();
    // phase 0 (every row, the first time): a loose tolerance; later phases to eps
    const float eps_ph = (phases == 0 && !full_to_eps && (have_f || !resume)) ? p.eps * kPhase0EpsScale : p.eps;
    std::vector<float> xa, ya, aa, fa;
    if (!all) {
      xa = gather_rows(x, d, act);
      ya.resize((size_t)na);
      aa.resize((size_t)na);
      fa.resize((size_t)na);
      for (int64_t k = 0; k < na; ++k) {
        ya[k] = y[act[k]];
        aa[k] = alpha[act[k]];
        fa[k] = f[act[k]];
      }
    }
    const Extremes e0 = extremes(all ? f : fa, all ? alpha : aa, all ? y.data() : ya.data(), C);
    Checkpoint ck;
    ck.n = na;
    ck.d = d;
    ck.C = p.C;
    ck.gamma = gamma;
    ck.eps = eps_ph;
    ck.clip = (int)p.clip;
    ck.iter = iters;
    ck.b_hi = e0.b_hi;
    ck.b_lo = e0.b_lo;
    ck.alpha = all ? alpha : aa;
    if (have_f || phases > 0) ck.f = all ? f : fa;  // else recomputed from alpha by the solver
    const Checkpoint* ckp = (phases == 0 && !resume) ? nullptr : &ck;
    std::vector<float> f_new;
    SolveResult r;
    const double t_phase = now();
    double t_set = 0.0, t_grad = 0.0;
    std::string phase_engine;
    if (all) {
      // the whole problem: the solver set up once (setup())
      m.whole->set_eps(eps_ph);
      r = m.whole->solve(ckp, progress);
      const double tg = now();
      f_new = m.whole->gradient_all();
      t_grad = now() - tg;
      phase_engine = m.info.iteration + "/" + (world > 1 ? m.info.dp_policy + " " + m.info.exchange : std::string("local"));
    } else {
      SolverParams sp = p;
      sp.eps = eps_ph;
      {
        // the whole-problem solver holds its cache (cache_frac of the device):
        // when the phase's resident Gram (na x na / world columns) does not fit
        // what is left, lend it that memory until the next whole phase (which
        // allocates it again); agreed, so every rank's phase sees the same sizes
        HIP_CHECK(hipSetDevice(m.device));
        size_t freeb = 0, totalb = 0;
        HIP_CHECK(hipMemGetInfo(&freeb, &totalb));
        const int64_t cols = (na + world - 1) / world;
        const double need = (double)na * (double)((cols + 255) / 256 * 256) * 4.0;
        static const bool force_release = [] {  // tests: DPSVM_SHRINK_RELEASE=1 lends it for every phase
          const char* e = std::getenv("DPSVM_SHRINK_RELEASE");
          return e && e[0] == '1';
        }();
        const bool fits = need < p.cache_frac * (double)freeb - 512.0 * (1 << 20) && !force_release;
        if (!comm_all(m.comm, fits)) m.whole->release_cache();
      }
      GpuSolver s(sp, m.comm, m.device);
      const GpuSetupInfo si = s.setup(xa.data(), na, na, d, ya.data());
      t_set = now() - t_phase;
      phase_engine = si.iteration + "/" + (world > 1 ? si.dp_policy + " " + si.exchange : std::string("local"));
      r = s.solve(ckp, progress);
      const double tg = now();
      f_new = s.gradient_all();
      t_grad = now() - tg;
    }  // a shrunk phase's device memory is released before the next phase
    ++phases;
    {
      char buf[64];
      snprintf(buf, sizeof(buf), " %lld %.3f", (long long)r.outer, now() - t_phase);
      res.phase_log += (res.phase_log.empty() ? "" : ";") + std::to_string(na) + " " + phase_engine + buf;
    }
    if (trace::fault_throw_phase(m.rank) == phases)
      fail("fault injection: rank " + std::to_string(m.rank) + " throws after shrink phase " + std::to_string(phases));
    iters = r.iters;
    rounds += r.outer;
    rows_computed += r.rows_computed;
    t_gram += r.t_gram;
    double t_upd = 0.0;
    if (all) {
      alpha = r.alpha;
      f = f_new;
    } else {
      // the inactive rows' gradient: one predict GEMM over the phase's changes
      const double tu = now();
      Model dm;
      dm.gamma = gamma;
      dm.b = 0.f;
      dm.d = d;
      std::vector<int64_t> changed;
      for (int64_t k = 0; k < na; ++k)
        if (r.alpha[k] != aa[k]) {
          dm.alpha.push_back(r.alpha[k] - aa[k]);
          dm.y.push_back(ya[k]);
          changed.push_back(act[k]);
        }
      std::vector<char> is_act((size_t)n, 0);
      for (int64_t j : act) is_act[j] = 1;
      if (!changed.empty() && na < n) {
        // the change's contribution at every row of this rank's slice of X
        // (device-resident; the active rows' values are unused), all-gathered
        if (!m.xsl) m.xsl.reset(new XSlice(x, n, d, m.device, rank, world));
        dm.x = gather_rows(x, d, changed);
        std::vector<float> df((size_t)n, 0.f);
        m.xsl->update(dm, d, p.gram_precision, df);
        if (m.comm) comm_allgather_slices(m.comm, df);
        for (int64_t j = 0; j < n; ++j)
          if (!is_act[j]) f[j] += df[j];
      }
      for (int64_t k = 0; k < na; ++k) {
        alpha[act[k]] = r.alpha[k];
        f[act[k]] = f_new[k];
      }
      t_upd = now() - tu;
    }
    const Extremes e = extremes(f, alpha, y.data(), C);
    res.b_hi = e.b_hi;
    res.b_lo = e.b_lo;
    if (!m.p0.checkpoint_path.empty() && rank == 0) {
      // the whole problem after this phase (alpha, exact f): resumable by any
      // solver, with or without shrinking
      Checkpoint wck;
      wck.n = n;
      wck.d = d;
      wck.C = p.C;
      wck.gamma = gamma;
      wck.eps = p.eps;
      wck.clip = (int)p.clip;
      wck.iter = iters;
      wck.b_hi = e.b_hi;
      wck.b_lo = e.b_lo;
      wck.alpha = alpha;
      wck.f = f;
      write_checkpoint(m.p0.checkpoint_path, wck);
    }
    const bool open = e.ok && gap_open(e.b_hi, e.b_lo, p.eps);
    if (p.verbose && rank == 0)
      fprintf(stderr,
              "[dpsvm] shrink phase %d: %lld active rows, %lld rounds, %lld pair steps, %.3f s (setup %.3f, "
              "solve %.3f, gradient %.3f, inactive update %.3f s), global gap %g (status %d)\n",
              phases, (long long)na, (long long)r.outer, (long long)iters, now() - t_phase, t_set, r.t_solve, t_grad,
              t_upd, (double)(e.b_lo - e.b_hi), r.status);
    if (!e.ok) {
      res.status = kNoPair;
      break;
    }
    if (!open) {
      res.status = kConverged;
      break;
    }
    if (r.status == kMaxIter || iters >= p.max_iter) {
      res.status = kMaxIter;
      break;
    }
    if (r.status == kNonFinite || r.status == kCommFail) {
      res.status = r.status;
      break;
    }
    if (full_to_eps && all) {  // the whole problem solved to eps and still open: fp32 limit
      res.status = r.status;
      break;
    }
    act = active_rows(f, alpha, y.data(), C, e);
    if (phases >= kMaxPhases || (double)act.size() > kShrinkMaxFrac * (double)n) {
      act.clear();  // the whole problem to eps
      full_to_eps = true;
    }
  }
  res.alpha = alpha;
  res.iters = iters;
  res.outer = rounds;
  res.rows_computed = rows_computed;
  res.t_gram = t_gram;
  res.b = (res.b_hi + res.b_lo) / 2.f;
  res.t_solve = now() - t_start;
  res.shrink_phases = phases;
  return res;
}

SolveResult solve_shrinking(const SolverParams& p0, int device, const float* x, int64_t n, int d, const float* y_in,
                            const Checkpoint* resume, const ProgressFn& progress, Communicator* comm) {
  ShrinkingSolver s(p0, comm, device);
  s.setup(x, n, d, y_in);
  return s.solve(resume, progress);
}

namespace {
// the setup's cache budget (gpu_setup.hip) on this device: is the Gram block
// K(all n rows, cols columns) NOT resident?  (every line >= cols floats,
// padded to 256)
bool gram_exceeds_device(const SolverParams& p, int64_t n, int64_t cols, int device) {
  HIP_CHECK(hipSetDevice(device));
  size_t freeb = 0, totalb = 0;
  HIP_CHECK(hipMemGetInfo(&freeb, &totalb));
  double budget = p.cache_frac * (double)freeb - 256.0 * 1024 * 1024;
  if (p.cache_mb > 0) budget = std::min(budget, p.cache_mb * 1024.0 * 1024.0);
  const double ld = (double)((cols + 255) / 256 * 256);
  return (double)n * ld * 4.0 > budget;
}
}  // namespace

bool shrink_auto(const SolverParams& p, int64_t n, int d, int device, Communicator* comm) {
  (void)d;
  if (p.solver == 1) return false;                       // solver=smo: the reference's trajectory
  if (p.solver == 0 && n < kWsAutoRows) return false;    // auto below 50k rows: the pair engines
  if (p.force_cache) return false;                     // an explicit engine request (tests, probes)
  if (comm && comm->size() > 1) {
    if (p.x_mode == 2) return false;                     // the phases need X on every rank
    // a rank holds the columns of its row shard (dp shard; dp auto shards when
    // the whole Gram does not fit one device) or the whole Gram (dp replicate):
    // shrink only when that footprint is not resident on some rank's device
    // (covtype-ref at 8 ranks: 500k x 62.5k columns, 125 GB a rank, resident)
    const int64_t P = comm->size();
    const int64_t cols = p.dp_policy == 2 ? n : (n + P - 1) / P;
    return !comm_all(comm, !gram_exceeds_device(p, n, cols, device));  // any rank short of memory: shrink
  }
  return gram_exceeds_device(p, n, n, device);
}

}  // namespace dpsvm
