// Device solver setup: data-parallel policy, X placement, global vectors,
// kernel-row cache sizing (288 GB of HBM: the Gram shard is usually resident),
// workgroup geometry and the choice of iteration engine.
//
// Reference: SvmTrain::setup (svmTrain.cu:319-395: full X H2D per rank, n
// separate norm launches, 10 eager cache lines) and the shard tables of
// svmTrainMain.cpp:367-384.  Every decision that must match across ranks
// (dense vs cache mode, X placement, engine) is agreed by a collective, since
// free memory and residency can differ per device.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <chrono>
#include <thread>

#include <unistd.h>

#include "gpu_impl.hpp"
#include "../runtime/timer.hpp"

namespace dpsvm {

using gpu::dmalloc;
using gpu::round_up;

GpuSolver::Impl::~Impl() {
  if (device >= 0) (void)hipSetDevice(device);
  engine.reset();
  for (void* q : xopened) (void)hipIpcCloseMemHandle(q);
  if (xbuf) (void)hipFree(xbuf);
  if (xpeer_d) (void)hipFree(xpeer_d);
  if (gexec) (void)hipGraphExecDestroy(gexec);
  if (graph) (void)hipGraphDestroy(graph);
  if (gexec1) (void)hipGraphExecDestroy(gexec1);
  if (graph1) (void)hipGraphDestroy(graph1);
  for (void* ptr : {(void*)x, (void*)xsq, (void*)y, (void*)alpha, (void*)f, (void*)lines, (void*)slot_of,
                    (void*)key_of, (void*)ref, (void*)hslot_of, (void*)hkey_of, (void*)partials, (void*)ctrl,
                    (void*)records, (void*)my_record, (void*)pf, (void*)rf, (void*)rcf, (void*)stamps,
                    (void*)plru_meta, (void*)plru_stats, (void*)wsctrl, (void*)wscand, (void*)wssub, (void*)wsdfs, (void*)wsdalpha, (void*)wspart, (void*)wssorted,
                    (void*)wsxq, (void*)wsxqsq, (void*)wsiota, xs, (void*)xsh, wsxs, (void*)wsxsh})
    if (ptr) (void)hipFree(ptr);
  if (status_h) (void)hipHostFree(status_h);
  if (hlines_h) (void)hipHostFree(hlines_h);
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
  if (stream) (void)hipStreamDestroy(stream);
}

SmoStatus GpuSolver::Impl::read_status() const {
  SmoStatus s;
  std::atomic_thread_fence(std::memory_order_acquire);
  memcpy(&s, (const void*)status_h, sizeof(s));
  return s;
}

void GpuSolver::Impl::init_ctrl(int64_t iter0, float b_hi, float b_lo) {
  SmoCtrl c;
  memset(&c, 0, sizeof(c));
  c.iter = (int32_t)iter0;
  c.line_hi = c.line_lo = -1;
  c.b_hi = b_hi;
  c.b_lo = b_lo;
  HIP_CHECK(hipMemcpyAsync(ctrl, &c, sizeof(c), hipMemcpyHostToDevice, stream));
  memset(status_h, 0, sizeof(SmoStatus));
}

void GpuSolver::Impl::wait_event(hipEvent_t e) {
  // bounded wait with async-error polling (SURVEY §5.3 watchdog)
  auto t0 = Clock::now();
  const double limit = wd_limit > 0.0 ? wd_limit : (p.watchdog_s > 0.0 ? p.watchdog_s : kWatchdogDefaultS);
  int spins = 0;
  while (true) {
    hipError_t q = hipEventQuery(e);
    if (q != hipSuccess && q != hipErrorNotReady) HIP_CHECK(q);
    if (world > 1) {
      // also after a completed event: kernels of an aborted communicator exit
      // and their events complete, and the next block must not relaunch a
      // graph whose collective nodes point at the freed communicator
      std::string err = comm->async_error();
      if (!err.empty()) {
        comm->abort();
        fail("collective failed on rank " + std::to_string(rank) + ": " + err);
      }
    }
    if (q == hipSuccess) return;
    if (secs_since(t0) > limit) {
      if (world > 1) comm->abort();
      fail("watchdog: SMO block did not finish within " + std::to_string(limit) + " s");
    }
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

GpuSolver::GpuSolver(const SolverParams& p, Communicator* comm, int device) : impl_(new Impl) {
  auto& m = *impl_;
  m.p = p;
  if (!comm) {
    m.own_comm = make_local_comm();
    comm = m.own_comm.get();
  }
  m.comm = m.outer = comm;
  m.rank = m.outer_rank = comm->rank();
  m.world = m.outer_world = comm->size();
  m.device = device;
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&m.ev[0], hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&m.ev[1], hipEventDisableTiming));
}

GpuSolver::~GpuSolver() = default;

void GpuSolver::set_eps(float eps) {
  auto& m = *impl_;
  DPSVM_CHECK(eps > 0.f && std::isfinite(eps), "set_eps: eps must be > 0");
  if (eps == m.p.eps) return;
  HIP_CHECK(hipSetDevice(m.device));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  m.p.eps = eps;
  m.args.eps = eps;
  m.wsa.eps = eps;
  m.wsa.eps_floor = m.p.ws_rel * eps;
  // the captured graphs hold the old kernel arguments: recaptured by the next solve
  if (m.gexec) (void)hipGraphExecDestroy(m.gexec);
  if (m.graph) (void)hipGraphDestroy(m.graph);
  if (m.gexec1) (void)hipGraphExecDestroy(m.gexec1);
  if (m.graph1) (void)hipGraphDestroy(m.graph1);
  m.gexec = m.gexec1 = nullptr;
  m.graph = m.graph1 = nullptr;
}
const GpuSetupInfo& GpuSolver::info() const { return impl_->info; }

void GpuSolver::release_cache() {
  auto& m = *impl_;
  if (!m.lines) return;
  HIP_CHECK(hipSetDevice(m.device));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  // the captured graphs hold the lines' address: recaptured by the next solve
  if (m.gexec) (void)hipGraphExecDestroy(m.gexec);
  if (m.graph) (void)hipGraphDestroy(m.graph);
  if (m.gexec1) (void)hipGraphExecDestroy(m.gexec1);
  if (m.graph1) (void)hipGraphDestroy(m.graph1);
  m.gexec = m.gexec1 = nullptr;
  m.graph = m.graph1 = nullptr;
  HIP_CHECK(hipFree(m.lines));
  m.lines = nullptr;
  m.args.lines = nullptr;
  m.wsa.gram = nullptr;
  // bytes_device is what the solver holds now (the lines are lent out)
  m.bytes -= (size_t)m.L * m.ldl * sizeof(float);
  m.info.bytes_device = m.bytes;
}

namespace {

// Fast geometry of the one-device persistent dense engine: <= 256 workgroups
// of <= 1024 rows (4 register rows per thread, one poll batch per 64 lanes).
constexpr int64_t kReplicateMaxRows = 256 * 1024;

// every rank on its own physical device (PCI bus id; one node)?
bool distinct_devices(GpuSolver::Impl& m) {
  struct Id {
    char bus[32];
  } me{};
  if (hipDeviceGetPCIBusId(me.bus, sizeof(me.bus), m.device) != hipSuccess) {
    (void)hipGetLastError();
    snprintf(me.bus, sizeof(me.bus), "pid%d-dev%d", (int)getpid(), m.device);
  }
  std::vector<Id> all((size_t)m.world);
  m.allgather_bytes(&me, all.data(), sizeof(Id));
  for (int a = 0; a < m.world; ++a)
    for (int b = a + 1; b < m.world; ++b)
      if (strncmp(all[a].bus, all[b].bus, sizeof(Id::bus)) == 0) return false;
  return true;
}

// mean off-diagonal kernel value K(x_a, x_b) over a deterministic sample of up
// to 96 rows (fixed stride, float64): how strongly the rows of a working set
// couple — ~0 when K ~ I (MNIST-shape at gamma 0.25), ~0.85 for covtype-shape
constexpr double kWsW2Coupling = 0.1;
constexpr double kWsUncoupled = 1e-4;  // below: the blocks of a round are independent (64 blocks of 48 rows)
double mean_offdiag_kernel(const float* xh, int64_t rows, int d, float gamma) {
  const int64_t s = std::min<int64_t>(96, rows);
  if (s < 2) return 0.0;
  const int64_t stride = rows / s;
  double acc = 0.0;
  for (int64_t a = 0; a < s; ++a)
    for (int64_t b = a + 1; b < s; ++b) {
      const float* xa = xh + (size_t)(a * stride) * d;
      const float* xb = xh + (size_t)(b * stride) * d;
      double d2 = 0.0;
      for (int k = 0; k < d; ++k) {
        const double t = (double)xa[k] - (double)xb[k];
        d2 += t * t;
      }
      acc += std::exp(-(double)gamma * d2);
    }
  return acc / (double)(s * (s - 1) / 2);
}

// adaptive split Gram (gram_adapt auto, docs/DESIGN.md §13): true when every
// off-diagonal pair of the coupling sample (96 rows, float64) passes the
// one-product error bound with a 4x margin — K (e^E - 1) <= tau / 4 with
// E = gamma 4.5 2^-11 |a| |b| <= 1 — so that few tiles of the Gram hold an
// element the bound rejects (each costs a three-product recompute).  Any
// rejected element is still recomputed: this only predicts the cost.
bool gram_cold_sample_ok(const float* xh, int64_t rows, int d, float gamma, float tau) {
  const int64_t s = std::min<int64_t>(96, rows);
  if (s < 2 || !(gamma > 0.f) || !(tau > 0.f)) return false;
  const int64_t stride = rows / s;
  const double e = 4.5 * std::ldexp(1.0, -11) * (double)gamma;
  std::vector<double> nrm((size_t)s);
  for (int64_t a = 0; a < s; ++a) {
    const float* xa = xh + (size_t)(a * stride) * d;
    double q = 0.0;
    for (int k = 0; k < d; ++k) q += (double)xa[k] * (double)xa[k];
    nrm[(size_t)a] = std::sqrt(q);
  }
  for (int64_t a = 0; a < s; ++a)
    for (int64_t b = a + 1; b < s; ++b) {
      const float* xa = xh + (size_t)(a * stride) * d;
      const float* xb = xh + (size_t)(b * stride) * d;
      double d2 = 0.0;
      for (int k = 0; k < d; ++k) {
        const double t = (double)xa[k] - (double)xb[k];
        d2 += t * t;
      }
      const double E = e * nrm[(size_t)a] * nrm[(size_t)b];
      if (!(E <= 1.0) || std::exp(-(double)gamma * d2) * std::expm1(E) > 0.25 * (double)tau) return false;
    }
  return true;
}

// the most ranks any one device carries (collective: every rank calls it)
int max_device_sharing(GpuSolver::Impl& m) {
  struct Id {
    char bus[32];
  } me{};
  if (hipDeviceGetPCIBusId(me.bus, sizeof(me.bus), m.device) != hipSuccess) {
    (void)hipGetLastError();
    snprintf(me.bus, sizeof(me.bus), "pid%d-dev%d", (int)getpid(), m.device);
  }
  std::vector<Id> all((size_t)m.world);
  m.allgather_bytes(&me, all.data(), sizeof(Id));
  int most = 1;
  for (int a = 0; a < m.world; ++a) {
    int k = 0;
    for (int b = 0; b < m.world; ++b) k += strncmp(all[a].bus, all[b].bus, sizeof(Id::bus)) == 0;
    most = std::max(most, k);
  }
  return most;
}

// ws-cache without the cache (ws_recompute.hip): with short rows (d <= 64
// padded) a round's kernel rows are cheaper to recompute inside the f update
// than to write into cache lines and read back (covtype-shape 581k rows:
// profiles/r5_ws_recompute_ab.txt).  One rank; the one-block rounds (a
// multi-block engine's multi-block rounds keep the cache).
void ws_recompute_setup(GpuSolver::Impl& m) {
  WsArgs& w = m.wsa;
  m.ws_recompute = false;
  m.info.ws_rows = m.kind == EngineKind::WsDense ? "gram" : "cache";
  if (m.kind != EngineKind::WsCache) return;
  int mode = m.p.ws_recompute;  // 0 auto, 1 on, 2 off
  if (const char* e = std::getenv("DPSVM_WS_RECOMPUTE")) mode = std::atoi(e);  // A/B runs
  if (mode == 2 || !m.gram_split || !launch::ws_recompute_supported(w, m.dp)) return;
  m.ws_recompute = true;
  m.info.ws_rows = "recompute";
}

}  // namespace

GpuSetupInfo GpuSolver::setup(const float* xh, int64_t n_x_rows, int64_t n, int d, const float* yh) {
  auto& m = *impl_;
  HIP_CHECK(hipSetDevice(m.device));
  DPSVM_CHECK(n >= 2 && d >= 1, "need at least 2 samples and 1 feature");
  DPSVM_CHECK(n < (int64_t)1 << 31, "n must fit in 31 bits (packed selection keys)");
  DPSVM_CHECK(m.p.C > 0.f, "C must be > 0");
  DPSVM_CHECK(m.p.rows_per_group % kFusedThreads == 0 && m.p.rows_per_group >= 0,
              "rows_per_group must be a multiple of 256");
  m.n = n;
  m.d = d;
  m.dp = pad_features(d);
  m.gamma = resolve_gamma(m.p.gamma, d);
  size_t freeb = 0, totalb = 0;
  HIP_CHECK(hipMemGetInfo(&freeb, &totalb));

  // ---- data-parallel policy (world > 1): shard the rows or solve it all ----
  if (m.world > 1 && m.p.dp_policy != 1 && n_x_rows == n && m.p.x_mode != 2) {
    bool rep = m.p.dp_policy == 2;
    if (!rep) {
      const bool distinct = distinct_devices(m);  // collective: every rank calls it
      const double gram_bytes = (double)n * (double)round_up(n, 256) * 4.0;
      const bool fits = gram_bytes + (double)n * m.dp * 4.0 < m.p.cache_frac * (double)freeb - 512.0 * (1 << 20);
      rep = distinct && fits && n <= kReplicateMaxRows && !m.p.force_cache && m.p.persist != 1 &&
            m.p.exchange != 1 && !m.p.force_collectives && m.p.use_graph;
      rep = m.all_agree(rep, m.comm, m.world);
    }
    if (rep) {
      // every rank solves the whole problem on its own device: no per-iteration
      // communication; the caller's communicator still verifies the result
      m.own_comm = make_local_comm();
      m.comm = m.own_comm.get();
      m.rank = 0;
      m.world = 1;
      m.info.dp_policy = "replicate";
    }
  }

  const Shard sh = shard_of(n, m.rank, m.world);
  m.nl = sh.size;
  m.off = sh.offset;
  const int64_t nl_max = (n + m.world - 1) / m.world;
  m.G = std::max<int64_t>(1, (nl_max + kStepRows - 1) / kStepRows);
  // fused / persistent geometry, rows per workgroup a multiple of 256.  Cache
  // mode: ~cache_groups workgroups (the X pass wants every CU).  Dense mode:
  // ~128 publishers over all ranks, <= 1024 rows per workgroup (dense_rows_min,
  // common.hpp; profiles/r1_dense_rows_ab.txt).  rows_per_group overrides both.
  const int64_t wgs = std::max(1, m.p.cache_groups);
  auto geometry = [&](int64_t rows_min) {
    if (m.p.rows_per_group > 0) {
      const int64_t r = m.p.rows_per_group;
      return std::pair<int64_t, int64_t>(r, std::max<int64_t>(1, (nl_max + r - 1) / r));
    }
    const Geometry g = make_geometry(nl_max, rows_min, wgs);
    return std::pair<int64_t, int64_t>(g.rows, g.groups);
  };
  const auto geo_cache = geometry(0);
  const auto geo_dense = geometry(dense_rows_min(nl_max, m.world));
  m.RBf = geo_cache.first;
  m.Gf = geo_cache.second;
  // lines cover every row a kernel may write (the fused X pass writes whole
  // 256-row tiles) under either geometry
  m.ldl = std::max<int64_t>({m.G * kStepRows, geo_cache.first * geo_cache.second, geo_dense.first * geo_dense.second});

  // ---- X placement ----
  if (n_x_rows == n) {
    m.replicated = m.p.x_mode != 2;
  } else {
    DPSVM_CHECK(n_x_rows == m.nl, "x must hold all n rows (replicated) or this rank's shard rows");
    m.replicated = false;
  }
  if (m.world == 1 && m.p.x_mode == 2) m.replicated = false;
  if (m.replicated && m.p.x_mode == 0 && m.world > 1) {
    // auto: replicate unless X would take more than 40% of free HBM (agreed)
    const double xbytes = (double)n * m.dp * 4.0;
    m.replicated = m.all_agree(xbytes <= 0.4 * (double)freeb, m.comm, m.world);
    DPSVM_CHECK(m.replicated || n_x_rows == n, "internal: partition fallback needs full x");
  }
  const int64_t x_row0 = m.replicated ? 0 : m.off;
  // + 512 zero rows: the row GEMM (rbf_rows_indexed, 32x512 tiles) reads the
  // owned rows to a multiple of 512
  m.x_rows = m.replicated ? round_up(std::max<int64_t>(n, m.off + m.ldl), 128) + 512 : m.ldl + 512;
  m.x = dmalloc<float>((size_t)m.x_rows * m.dp, &m.bytes);
  HIP_CHECK(hipMemsetAsync(m.x, 0, (size_t)m.x_rows * m.dp * 4, m.stream));
  {
    const float* src = xh;
    int64_t rows = n_x_rows;
    if (!m.replicated && n_x_rows == n) {
      src = xh + (size_t)m.off * d;
      rows = m.nl;
    }
    if (rows > 0)
      HIP_CHECK(hipMemcpy2DAsync(m.x, (size_t)m.dp * 4, src, (size_t)d * 4, (size_t)d * 4, (size_t)rows,
                                 hipMemcpyHostToDevice, m.stream));
  }
  // ---- global vectors (n padded so padded local rows index in-bounds) ----
  const int64_t n_pad = round_up(std::max<int64_t>(n, m.off + m.ldl), 128) + 512;
  m.xsq = dmalloc<float>((size_t)n_pad, &m.bytes);
  m.y = dmalloc<float>((size_t)n_pad, &m.bytes);
  m.alpha = dmalloc<float>((size_t)n_pad, &m.bytes);
  HIP_CHECK(hipMemsetAsync(m.xsq, 0, n_pad * 4, m.stream));
  HIP_CHECK(hipMemsetAsync(m.y, 0, n_pad * 4, m.stream));
  HIP_CHECK(hipMemsetAsync(m.alpha, 0, n_pad * 4, m.stream));
  m.h_y.assign(yh, yh + n);
  for (auto& v : m.h_y) v = v > 0 ? 1.f : -1.f;
  HIP_CHECK(hipMemcpyAsync(m.y, m.h_y.data(), n * 4, hipMemcpyHostToDevice, m.stream));
  if (m.replicated) {
    launch::row_sqnorm(m.x, n, m.dp, m.dp, m.xsq, m.stream);  // one launch (was n)
  } else {
    // local norms, then all-gather the shards into the global vector
    float* loc = dmalloc<float>((size_t)m.ldl, &m.bytes);
    HIP_CHECK(hipMemsetAsync(loc, 0, m.ldl * 4, m.stream));
    launch::row_sqnorm(m.x, m.nl, m.dp, m.dp, loc, m.stream);
    std::vector<float> all((size_t)m.ldl * m.world), mine((size_t)m.ldl);
    if (m.world > 1 && m.comm->device_memory()) {
      float* gbuf = dmalloc<float>((size_t)m.ldl * m.world, &m.bytes);
      m.comm->allgather(loc, gbuf, m.ldl * 4, m.stream);
      HIP_CHECK(hipMemcpyAsync(all.data(), gbuf, all.size() * 4, hipMemcpyDeviceToHost, m.stream));
      sync_collective(m.comm, m.stream, "norm all-gather");
      (void)hipFree(gbuf);
    } else {
      HIP_CHECK(hipMemcpyAsync(mine.data(), loc, m.ldl * 4, hipMemcpyDeviceToHost, m.stream));
      HIP_CHECK(hipStreamSynchronize(m.stream));
      m.comm->allgather(mine.data(), all.data(), m.ldl * 4, nullptr);
    }
    std::vector<float> g((size_t)n, 0.f);
    for (int r = 0; r < m.world; ++r) {
      Shard s = shard_of(n, r, m.world);
      std::copy(all.begin() + (size_t)r * m.ldl, all.begin() + (size_t)r * m.ldl + s.size, g.begin() + s.offset);
    }
    HIP_CHECK(hipMemcpyAsync(m.xsq, g.data(), n * 4, hipMemcpyHostToDevice, m.stream));
    HIP_CHECK(hipStreamSynchronize(m.stream));
    (void)hipFree(loc);
  }
  m.f = dmalloc<float>((size_t)m.ldl, &m.bytes);
  HIP_CHECK(hipMemsetAsync(m.f, 0, m.ldl * 4, m.stream));
  m.partials = dmalloc<uint64_t>((size_t)2 * m.G, &m.bytes);
  m.ctrl = dmalloc<SmoCtrl>(1, &m.bytes);
  HIP_CHECK(hipHostMalloc((void**)&m.status_h, sizeof(SmoStatus), hipHostMallocMapped));
  HIP_CHECK(hipHostGetDevicePointer((void**)&m.status_d, m.status_h, 0));
  if (!m.replicated) {
    const int64_t rb = round_up((int64_t)sizeof(CandRecord) + 2LL * m.dp * 4, 64);
    m.my_record = dmalloc<uint8_t>((size_t)rb, &m.bytes);
    m.records = dmalloc<uint8_t>((size_t)rb * m.world, &m.bytes);
    HIP_CHECK(hipMemsetAsync(m.records, 0, rb * m.world, m.stream));
    m.args.rec_bytes = rb;
    m.h_records.assign((size_t)rb * m.world, 0);
  }
  m.h_partials.assign((size_t)2 * m.G, kKeyNone);
  // fp16 split operands of x for the split GEMMs (allocated before the cache is
  // sized from the free memory; released below if the engine runs f32 GEMMs)
  DPSVM_CHECK(m.p.gram_precision >= 0 && m.p.gram_precision <= 2, "gram_precision must be 0 (auto), 1 (f32) or 2 (split)");
  DPSVM_CHECK(m.p.engines == 0 || m.p.engines == 1, "engines must be 0 (production) or 1 (all)");
  DPSVM_CHECK(m.p.engines == 1 || (m.p.host_cache_lines == 0 && m.p.cache_engine == 0),
              "host_cache_lines and cache_engine=chain run on the quarantined pair-at-a-time cache engines: "
              "set engines=all (tests, A/B probes)");
  // production engines, solver auto: the working-set engines also below
  // kWsAutoRows rows when the Gram is not resident or X is partitioned
  const bool maybe_ws = m.p.solver == 2 || (m.p.solver == 0 && (n >= kWsAutoRows || m.p.engines == 0));
  if (m.p.gram_precision == 2 || (m.p.gram_precision == 0 && maybe_ws)) {
    m.xs = dmalloc<uint8_t>((size_t)m.x_rows * launch::split_row_u4(m.dp) * 16, &m.bytes);
    m.xsh = dmalloc<int32_t>((size_t)m.x_rows, &m.bytes);
  }
  HIP_CHECK(hipStreamSynchronize(m.stream));

  // ---- kernel-row cache sizing (288 GB HBM: the Gram shard is usually resident) ----
  HIP_CHECK(hipMemGetInfo(&freeb, &totalb));
  const double line_bytes = (double)m.ldl * 4.0;
  double budget = m.p.cache_frac * (double)freeb - 256.0 * 1024 * 1024;
  if (m.p.cache_mb > 0) budget = std::min(budget, m.p.cache_mb * 1024.0 * 1024.0);
  int64_t want_lines = (int64_t)(budget / line_bytes);
  if (m.p.cache_lines > 0) want_lines = std::min<int64_t>(want_lines, m.p.cache_lines);
  // working-set engines (solver=ws): with replicated X, or with partitioned X
  // (ws-dense builds its Gram block panel by panel from broadcast shards;
  // ws-cache packs the misses' X rows and sums them over ranks each round —
  // no engine step after the Gram reads a non-owned X row)
  const int ws_q = std::max(2, std::min(m.p.ws_size, kWsMax));
  // -s N: the reference takes any line count (default 10 lines,
  // svmTrainMain.cpp:71; cache.cu:49-60, 82-105), a pure speed knob.  The
  // production engines cap their lines at N; where the cap lies below the
  // working-set cache's minimum (the round's 2 x ws_size rows + the victim
  // window: production_line_cap, device_state.hpp) it is raised to that minimum, so a
  // reference command line runs instead of failing.  engines=all keeps the
  // count as given (the quarantined pair-at-a-time cache engines take any >= 2).
  {
    const int64_t cap = production_line_cap(m.p.cache_lines, ws_q, m.p.engines);
    if (cap > m.p.cache_lines && want_lines < cap) {
      want_lines = std::min<int64_t>(cap, (int64_t)(budget / line_bytes));
      m.info.cache_note = "cache_lines " + std::to_string(m.p.cache_lines) + " raised to " +
                          std::to_string(want_lines) + " (the working-set cache's minimum: 2 x ws_size + " +
                          std::to_string(kWsCacheWindow) + " lines)";
      if (m.outer_rank == 0) fprintf(stderr, "[dpsvm] note: %s\n", m.info.cache_note.c_str());
    }
  }
  // solver auto: the working-set engines from kWsAutoRows rows on (the pair-at-a-time
  // engines follow the reference's trajectory exactly and win on small problems;
  // on 500k-2M rows ws is 5-10x faster: profiles/r2_*_converged.json)
  const bool gram_fits = m.all_agree(want_lines >= n && !m.p.force_cache, m.comm, m.world);
  const bool want_ws = m.p.solver == 2 ||
                       (m.p.solver == 0 && (n >= kWsAutoRows || (m.p.engines == 0 && (!gram_fits || !m.replicated))));
  const bool ws_ok = want_ws && launch::ws_supported(nl_max, m.world, ws_q);
  m.dense = (m.replicated || ws_ok) && gram_fits;  // agreed: free memory can differ per device
  if (m.dense) {
    m.RBf = geo_dense.first;
    m.Gf = geo_dense.second;
  }
  // engine candidates.  Persistent engines need the in-kernel exchange (set up
  // below) and a co-resident grid (census); the one-launch-per-iteration
  // engines are the fallbacks.
  // the pair-at-a-time cache engines are a plugin (gpu_engines_pairq.hip), present
  // only when loaded (engines=all): production setups never pick them
  const gpu::QuarantineOps* qo = gpu::quarantine();
  DPSVM_CHECK(m.p.engines == 0 || qo != nullptr,
              "engines=all needs the quarantined pair-cache plugin (Python: dpsvm_amd._native.load_quarantine(); CLI: "
              "bin/svmTrainPairq)");
  const bool dp16 = m.dp >= 16 && m.dp % 16 == 0;  // the cache-mode X pass / row GEMM operand width
  const bool fused_lru_ok = !m.dense && m.replicated && qo && qo->fused_lru_supported(m.dp) && m.p.cache_engine == 0;
  // working-set engines: the resident Gram (ws-dense), or a kernel-row cache
  // whose missing rows come from one GEMM per round (ws-cache); rows sharded
  // over ranks at world > 1 (per-round candidate all-gather + sub-Gram sum)
  const bool ws_cand = ws_ok && m.dense;
  const bool wsc_cand = ws_ok && !m.dense && m.p.host_cache_lines == 0 &&
                        (!m.replicated || dp16);
  if (want_ws && !ws_ok)
    m.info.engine_note = "ws engines need <= " + std::to_string(kWsMaxRPT) + " rows per selection thread";
  const bool plru_cand = !wsc_cand && fused_lru_ok && m.p.host_cache_lines == 0 && m.p.persist != 1 && m.p.exchange != 1 &&
                         m.p.use_graph && !m.p.force_collectives &&
                         qo->persist_lru_supported(m.dp, (int)m.RBf, (int)m.Gf);
  if (plru_cand) {
    // every workgroup's private metadata copy comes out of the line budget (upper bound: L = n)
    const double meta_bytes = (double)m.Gf * qo->plru_stride_words(n, n) * 4.0;
    want_lines = std::min<int64_t>(want_lines, (int64_t)((budget - meta_bytes) / line_bytes));
  }
  const bool pdense_cand = !ws_cand && m.dense &&
                           (m.p.persist == 2 || (m.p.persist == 0 && m.p.exchange != 1 && m.p.use_graph &&
                                                 !m.p.force_collectives)) &&
                           m.RBf <= 12 * kFusedThreads && m.Gf <= 256;
  m.L = m.dense ? n : std::max<int64_t>(2, std::min<int64_t>(want_lines, n));
  DPSVM_CHECK(m.L * line_bytes <= (double)freeb, "not enough device memory for 2 kernel-row lines");
  m.lines = dmalloc<float>((size_t)m.L * m.ldl, &m.bytes);
  if (m.dense || fused_lru_ok) {
    m.pf = dmalloc<uint64_t>((size_t)4 * m.Gf, &m.bytes);
    m.rf = dmalloc<FusedRec>(2, &m.bytes);
    if (!m.dense) m.rcf = dmalloc<FusedCacheRec>(2, &m.bytes);
  }
  if (!m.dense) {
    m.slot_of = dmalloc<int32_t>((size_t)n, &m.bytes);
    m.key_of = dmalloc<int32_t>((size_t)m.L, &m.bytes);
    m.ref = dmalloc<uint8_t>((size_t)m.L, &m.bytes);
    if (m.p.host_cache_lines > 0) {
      // pinned host tier: a FIFO victim cache the row kernel spills to and
      // fetches from with zero-copy PCIe accesses (no host round trip)
      m.H = m.p.host_cache_lines;
      HIP_CHECK(hipHostMalloc((void**)&m.hlines_h, (size_t)m.H * m.ldl * 4, hipHostMallocMapped));
      HIP_CHECK(hipHostGetDevicePointer((void**)&m.hlines_d, m.hlines_h, 0));
      m.hslot_of = dmalloc<int32_t>((size_t)n, &m.bytes);
      m.hkey_of = dmalloc<int32_t>((size_t)m.H, &m.bytes);
    }
  }

  SmoArgs& a = m.args;
  a.x = m.x;
  a.xsq = m.xsq;
  a.y = m.y;
  a.alpha = m.alpha;
  a.f = m.f;
  a.lines = m.lines;
  a.ldl = m.ldl;
  a.slot_of = m.slot_of;
  a.key_of = m.key_of;
  a.ref = m.ref;
  a.hlines = m.hlines_d;
  a.hslot_of = m.hslot_of;
  a.hkey_of = m.hkey_of;
  a.H = (int32_t)m.H;
  a.partials = m.partials;
  a.ctrl = m.ctrl;
  a.status = m.status_d;
  a.records = m.records;
  a.my_record = m.my_record;
  a.n = n;
  a.nl = m.nl;
  a.off = m.off;
  a.x_row0 = x_row0;
  a.d = d;
  a.dp = m.dp;
  a.G = (int32_t)m.G;
  a.L = (int32_t)m.L;
  a.world = m.world;
  a.cache_mode = m.dense ? kCacheDense : kCacheLRU;
  a.partitioned = m.replicated ? 0 : 1;
  a.spec = (m.replicated && !m.dense) ? std::max(0, std::min(m.p.spec_rows, kNQ - 2)) : 0;
  a.clip = (int)m.p.clip;
  a.C = m.p.C;
  a.gamma = m.gamma;
  a.eps = m.p.eps;
  a.tau = m.p.tau;
  a.max_iter = m.p.max_iter;
  a.fused_rows = (int32_t)m.RBf;
  a.fused_G = (int32_t)m.Gf;
  a.stamps = nullptr;
  a.census = nullptr;
  a.census_ticks = 0;
  a.eta_gram = (m.p.eta == 1 && m.dense && m.nl == n) ? 1 : 0;
  if (const char* sp = std::getenv("DPSVM_STAMPS")) {  // diagnostics only (bench/stamps_report.py)
    m.stamps_path = std::string(sp) + ".rank" + std::to_string(m.rank);
    const size_t cnt = (size_t)kStampRing * 2 * kStampSlots;
    m.stamps = dmalloc<uint64_t>(cnt, &m.bytes);
    HIP_CHECK(hipMemsetAsync(m.stamps, 0, cnt * 8, m.stream));
    a.stamps = m.stamps;
  }

  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  HIP_CHECK(hipGetDeviceProperties(&prop, dev));
  m.info.device = dev;
  m.info.device_name = prop.name[0] ? std::string(prop.name) : std::string(prop.gcnArchName);
  if (m.info.device_name.empty() || m.info.device_name == " ") m.info.device_name = prop.gcnArchName;
  m.info.n = n;
  m.info.n_local = m.nl;
  m.info.offset = m.off;
  m.info.d = d;
  m.info.dp = m.dp;
  m.info.x_replicated = m.replicated;
  m.info.cache_lines = m.L;
  m.info.blocks = (int)m.G;

  // ---- per-iteration key exchange and engine ----
  a.xpeer = nullptr;
  a.xrank = 0;
  a.xworld = 0;
  a.xstride = kXchGranules;
  a.xpoll_kb = 0;
  a.xpoll_sleep = 1;
  a.xtimeout_ticks = 0;
  m.xch = false;
  const bool want_xch = (!ws_cand && !wsc_cand && m.dense && m.p.exchange != 1 && (m.world > 1 || m.p.exchange == 2)) ||
                        pdense_cand || plru_cand;
  // working-set engines at world > 1: the rounds' candidate lists and sub-Gram
  // rows through the same kind of receive buffers (ws_*.hip, "peer exchange")
  const bool wsc_fits_pre = wsc_cand && launch::ws_cache_supported(m.L, ws_q);
  int32_t ws_G = 0, ws_rpt = 0;
  if (ws_cand || wsc_cand) launch::ws_geometry(nl_max, m.world, &ws_G, &ws_rpt);
  // multi-block rounds (ws_blocks > 1): the union merge reads <= 256 candidate
  // lists, an even q_max.  At world > 1 they run over the in-kernel peer
  // exchange (candidate lists, the P sub-Grams' owned entries and the
  // line-search partials pushed into every rank's receive buffer: no collective
  // per round) or, when that is unavailable, over the communicator's
  // collectives (three per round; a device communicator, or exchange=allreduce)
  DPSVM_CHECK(m.p.ws_blocks >= 0 && m.p.ws_blocks <= kWsMaxBlocks,
              "ws_blocks must be 0 (auto) or 1.." + std::to_string(kWsMaxBlocks));
  const bool multi_comm = m.world == 1 || m.comm->device_memory() || m.p.exchange == 1;
  // ws_blocks auto (0): every block from kWsAutoBlocksRows rows on (the round's
  // fixed cost is amortised over P sub-problems; small problems need few rounds)
  // auto: kWsAutoBlocks (32) blocks of kWsMaxAll / 32 = 96 rows (the union
  // capacity over more, smaller sub-problems: each round's pair steps run on
  // more workgroups; headline 0.0308 vs 0.0371 s at 8 x 192,
  // profiles/r3_union3072_ab.txt), never larger than ws_size; the one-block
  // rounds the adaptive count falls back to keep ws_size rows
  static const int auto_blocks_env = [] {  // A/B: DPSVM_WS_AUTO_BLOCKS (2 .. kWsMaxBlocks)
    const char* e = std::getenv("DPSVM_WS_AUTO_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v >= 2 && v <= kWsMaxBlocks ? v : 0;
  }();
  // the coupling of a row sample (mean off-diagonal K, host, outside the timed
  // region; read by the auto choices below and by the pair choice): where the
  // kernel is numerically diagonal at working-set scale (MNIST-shape at gamma
  // 0.25: 1.7e-9; the structured mnist-parity: 4.3e-3; covtype-shape 0.85) the
  // blocks of a round do not interact, so blocks of 48 rows (one
  // row per solve lane: cheaper pair steps) beat 32 of 96 (headline
  // 0.0238-0.0240 vs 0.0241-0.0242 s); coupled data keeps 32 (mnist-parity
  // 0.0206 s with 32, 0.0422 s with 64: damped rounds; profiles/r5_blocks_64_vs_32_ab.txt)
  const double coupling = (ws_cand || wsc_cand) ? mean_offdiag_kernel(xh, n_x_rows, d, m.gamma) : 1.0;
  const bool uncoupled = m.all_agree(coupling < kWsUncoupled, m.comm, m.world);
  // the round's union: the rounds touch ~3.4 n rows in all whatever the union
  // (headline: 254 / 128 / 67 rounds at 768 / 1,536 / 3,072 rows), so a wider
  // union divides the rounds' fixed cost (~50 us: selection, rank, merge, launch
  // gaps) — uncoupled ws-dense rounds take kWsMaxAll rows (128 blocks of 48;
  // profiles/r5_union6144_ab.txt), everything else kWsAutoUnion
  static const int union_env = [] {  // A/B: DPSVM_WS_UNION (kWsAutoUnion or kWsMaxAll)
    const char* e = std::getenv("DPSVM_WS_UNION");
    const int v = e ? atoi(e) : 0;
    return v == kWsAutoUnion || v == kWsMaxAll ? v : 0;
  }();
  const bool wide_ok = uncoupled && ws_cand;
  const int auto_union = union_env > 0 ? (wide_ok ? union_env : kWsAutoUnion) : wide_ok ? kWsMaxAll : kWsAutoUnion;
  const int auto_blocks = auto_blocks_env > 0 ? auto_blocks_env
                          : uncoupled         ? auto_union / 48
                                              : kWsAutoBlocks;
  const int auto_q = std::min(ws_q, auto_union / auto_blocks) & ~1;
  const bool blocks_auto = m.p.ws_blocks == 0;
  int want_blocks = !blocks_auto ? m.p.ws_blocks
                                 : (n >= kWsAutoBlocksRows ? std::min(auto_blocks, auto_union / auto_q) : 1);
  const int mb_q = blocks_auto ? auto_q : ws_q;  // rows per block of the multi-block rounds
  // ranks sharing one device (rehearsals; 1 on distinct devices) and the wave
  // slots the peer exchange's spinning consumers may take (below)
  int xch_share = 1, xch_cus = 0;
  if (m.world > 1) {
    xch_share = max_device_sharing(m);  // collective
    HIP_CHECK(hipDeviceGetAttribute(&xch_cus, hipDeviceAttributeMultiprocessorCount, m.device));
  }
  auto xch_waves = [&](int blocks) { return (int64_t)xch_share * (64 + 16 * std::max(1, blocks)) + 1024; };
  // an auto union whose spinning solve workgroups (one per block, every rank)
  // would not leave the ranks sharing a device room for their producers: halve
  // the block count until they fit (4 ranks on one GPU: 64 blocks, 8 ranks: 32,
  // over the peer exchange, rather than one block per round over host
  // collectives).  Distinct devices (share 1) always fit 128 blocks.
  // (collectives — exchange=allreduce, force_collectives — spin on nothing: the wide union stays)
  if (m.world > 1 && blocks_auto && want_blocks > 1 && m.p.exchange != 1 && !m.p.force_collectives) {
    while (want_blocks > 8 && !m.all_agree(xch_waves(want_blocks) <= (int64_t)xch_cus * 32, m.comm, m.world))
      want_blocks /= 2;
  }
  // (only where working-set rounds can run: solver=smo or a small problem ignores ws_blocks)
  DPSVM_CHECK(!(ws_cand || wsc_cand) || want_blocks <= 1 || want_blocks * mb_q <= kWsMaxAll,
              "ws_blocks x ws_size must be <= " + std::to_string(kWsMaxAll) + " (the round's union capacity)");
  // ws-cache takes them too when its cache holds the union's lines plus the
  // victim window (L >= 2 P q_max + 4096; agreed: L follows each device's free memory)
  const bool wsc_multi = wsc_fits_pre && launch::ws_cache_multi_supported(m.L, want_blocks, mb_q);
  // (unions past kWsAutoUnion: ws-dense only — the cache merge's line tables
  // hold kWsAutoUnion rows)
  bool multi_elig = want_blocks > 1 && (ws_cand || wsc_multi) && mb_q % 2 == 0 &&
                    (int64_t)ws_G * m.world <= kWsMaxGroups && (want_blocks * mb_q <= kWsAutoUnion || ws_cand);
  if (m.world > 1) multi_elig = m.all_agree(multi_elig, m.comm, m.world);
  // Residency of the ws peer exchange with ranks sharing a device (rehearsals;
  // on distinct devices share = 1).  No producer ever waits: selection, gather
  // and pass-1 workgroups push into every rank's receive buffer and return.  The
  // spinning consumers of one rank are the collect kernels (<= 16 workgroups of
  // 4 waves) and the solve (one workgroup of 16 waves per block), so the share
  // ranks' consumers plus one rank's full-size producer kernel (1024 waves) must
  // fit the device's wave slots for every rank's producers to keep running —
  // one-block and multi-block rounds alike.
  bool xch_resident = true;
  if (m.world > 1) {
    const int64_t waves = xch_waves(want_blocks);
    xch_resident = m.all_agree(waves <= (int64_t)xch_cus * 32, m.comm, m.world);
    if (!xch_resident && m.p.exchange != 2 && (ws_cand || wsc_fits_pre))
      m.info.engine_note = "ws peer exchange refused: " + std::to_string(xch_share) + " ranks share a device (" +
                           std::to_string(waves) + " spinning + producer waves > " + std::to_string(xch_cus * 32) +
                           " wave slots): collectives";
  }
  const bool ws_peer_base = (ws_cand || wsc_fits_pre) && m.p.exchange != 1 && !m.p.force_collectives &&
                            (m.world > 1 || m.p.exchange == 2);  // exchange=peer at world 1: loopback (tests)
  // multi-block rounds over the peer exchange (partitioned X in cache mode sums
  // the miss rows by an all-reduce: that engine keeps the collectives)
  // multi-block pass 1: the wide layout by default (1024-column groups, 16-B
  // row loads: headline round 227.5 -> 212.9 us, 0.0257 -> 0.0248 s,
  // profiles/r5_pass1_wide_ab.txt), or the selection geometry (G groups of
  // rpt x 256 columns; DPSVM_PASS1=v1 for A/B runs)
  static const bool p1_sel = [] {
    const char* e = std::getenv("DPSVM_PASS1");
    return e && std::string(e) == "v1";
  }();
  const bool p1v4 = !p1_sel;
  const int p1G = p1v4 ? launch::ws_pass1_v4_groups(nl_max) : ws_G;
  const int ks_mb = p1v4 ? launch::ws_pass1_v4_splits(p1G) : launch::ws_pass1_splits(p1G);
  bool multi_peer = false;
  if (ws_peer_base && multi_elig && !(wsc_cand && !m.replicated) && (xch_resident || m.p.exchange == 2)) {
    const int64_t G_all = (int64_t)ws_G * m.world;
    const bool ok = m.setup_exchange(ws_xch_words_multi(G_all, (int64_t)p1G * m.world, ks_mb, want_blocks, mb_q, ws_q));
    DPSVM_CHECK(ok || m.p.exchange != 2,
                "peer exchange requested (exchange=peer) but its self test failed (" + m.xch_diag + ")");
    if (ok) {
      m.xch = true;
      multi_peer = true;
    } else {
      m.info.engine_note = "peer exchange refused: " + m.xch_diag + " (multi-block rounds use the collectives)";
    }
  }
  const bool multi_ok = multi_elig && (multi_peer || (multi_comm && m.p.exchange != 2));
  const bool want_ws_xch = ws_peer_base && !multi_ok && (xch_resident || m.p.exchange == 2);
  if (want_ws_xch) {
    const bool ok = m.setup_exchange(ws_xch_words((int64_t)ws_G * m.world, ws_q));
    DPSVM_CHECK(ok || m.p.exchange != 2,
                "peer exchange requested (exchange=peer) but its self test failed (" + m.xch_diag + ")");
    if (ok) m.xch = true;
    else m.info.engine_note = "peer exchange refused: " + m.xch_diag + " (working-set rounds use the collectives)";
  } else if (want_xch) {
    const bool ok = m.setup_exchange();
    DPSVM_CHECK(ok || (m.p.exchange != 2 && m.p.persist != 2),
                "peer exchange requested (exchange=peer / persist=on) but its self test failed (" + m.xch_diag + ")");
    if (ok) {
      m.xch = true;
      a.xpeer = m.xpeer_d;
      a.xrank = m.rank;
      a.xworld = m.world;
      a.xstride = (int32_t)m.xstride;
      a.xpoll_kb = m.p.xch_poll_batch;
      a.xpoll_sleep = std::max(0, m.p.xch_sleep);
      a.xtimeout_ticks = (int64_t)(std::max(1e-6, m.p.xch_timeout_s) * 1e8);
    } else if (m.info.engine_note.empty()) {
      m.info.engine_note = "peer exchange refused: " + m.xch_diag;
    }
  }
  const bool wsc_fits = wsc_cand && launch::ws_cache_supported(m.L, ws_q);
  if (wsc_cand && !wsc_fits)
    m.info.engine_note = "ws-cache needs >= " + std::to_string(2 * ws_q + 512) + " lines";
  EngineFacts facts;
  facts.ws_dense = ws_cand;
  facts.ws_cache = wsc_fits;
  facts.dense = m.dense;
  facts.cache_replicated = fused_lru_ok;
  facts.persistent = (m.dense ? pdense_cand : plru_cand) && m.xch;
  facts.quarantine = m.p.engines == 1;
  if (!choose_engine(facts, &m.kind)) {
    std::string why = m.p.solver == 1 ? "solver=smo (pair-at-a-time) needs the resident Gram and replicated X"
                                      : "no working-set engine fits this configuration";
    if (!m.info.engine_note.empty()) why += " (" + m.info.engine_note + ")";
    DPSVM_CHECK(false, why + "; the pair-at-a-time cache / partitioned-X engines are quarantined: set engines=all");
  }
  if (m.persistent() && !m.census(m.kind)) {
    DPSVM_CHECK(m.p.persist != 2, "persistent engine requested (persist=on) but its grid is not co-resident (" +
                                      m.info.engine_note + ")");
    m.kind = m.dense ? EngineKind::FusedDense : EngineKind::FusedCache;
    if (m.kind == EngineKind::FusedCache && m.xch) {
      // the exchange was set up for the persistent cache engine only; the fused
      // cache engine combines keys through its records (and the all-reduce)
      m.xch = false;
      a.xpeer = nullptr;
      a.xrank = 0;
      a.xworld = 0;
    }
  }
  if (m.kind == EngineKind::PersistCache) {
    a.plru_stride = gpu::need_quarantine("the persistent-cache engine").plru_stride_words(n, m.L);
    m.plru_meta = dmalloc<int32_t>((size_t)m.Gf * a.plru_stride, &m.bytes);
    m.plru_stats = dmalloc<int64_t>(8, &m.bytes);
    a.plru_meta = m.plru_meta;
  } else {
    a.plru_meta = nullptr;
    a.plru_stride = 0;
  }
  // split GEMMs: the working-set engines (auto), or every dense Gram (split);
  // the pair-at-a-time cache engines compute rows in their own f32 X pass
  m.gram_split = m.xs && (m.working_set() || (m.p.gram_precision == 2 && m.dense));
  if (m.xs && !m.gram_split) {
    (void)hipFree(m.xs);
    (void)hipFree(m.xsh);
    m.xs = nullptr;
    m.xsh = nullptr;
  }
  m.info.gram = m.gram_split ? "split-f16" : "f32";
  {
    // adaptive split Gram for the resident ws-dense Gram (gram_adapt: 0 auto, 1 on, 2 off;
    // A/B: DPSVM_GRAM_ADAPT overrides)
    static const int adapt_env = [] {
      const char* e = std::getenv("DPSVM_GRAM_ADAPT");
      return e ? atoi(e) : -1;
    }();
    const int mode = adapt_env >= 0 ? adapt_env : m.p.gram_adapt;
    DPSVM_CHECK(mode >= 0 && mode <= 2, "gram_adapt must be 0 (auto), 1 (on) or 2 (off)");
    DPSVM_CHECK(m.p.gram_cold_tau > 0.f && m.p.gram_cold_tau <= 1e-3f, "gram_cold_tau must be in (0, 1e-3]");
    // (the one-product pass needs >= 5 split blocks a row: dp > 128; shorter rows keep the three-product Gram)
    // and the adaptive kernels' indexing (rbf_gemm_store_split's idx_adapt)
    const bool cand = m.gram_split && m.kind == EngineKind::WsDense && mode != 2 && m.gamma > 0.f && m.dp > 128 &&
                      (int64_t)(n + 512) * ((m.dp + 31) / 32) * 8 < (1ll << 31) && m.ldl < (1ll << 22);
    const bool ok = cand && (mode == 1 || gram_cold_sample_ok(xh, n_x_rows, d, m.gamma, m.p.gram_cold_tau));
    m.gram_cold_tau = m.all_agree(ok, m.comm, m.world) ? m.p.gram_cold_tau : 0.f;
    if (m.gram_cold_tau > 0.f) m.info.gram = "split-f16-adaptive";
  }
  if (m.working_set()) {
    WsArgs& w = m.wsa;
    w = WsArgs{};
    w.gram = m.lines;
    w.ldg = m.ldl;
    w.cache = m.kind == EngineKind::WsCache ? 1 : 0;
    w.L = (int32_t)m.L;
    w.slot_of = m.slot_of;
    w.key_of = m.key_of;
    w.y = m.y;
    w.alpha = m.alpha;
    w.f = m.f;
    w.n = n;
    w.nl = m.nl;
    w.off = m.off;
    w.G = ws_G;
    w.p1G = ws_G;  // multi-block rounds may take the wide pass-1 geometry below
    w.rpt = ws_rpt;
    w.world = m.world;
    w.G_all = w.G * m.world;
    w.q_max = ws_q;
    // >= 2 new rows: the global maximal violating pair (up rank 0, low rank 0)
    // is always in the set, so every round makes progress
    // defaults measured on the MNIST-shape headline (profiles/r2_ws_param_sweep.txt)
    w.n_new = ws_new_auto(m.p.ws_new, ws_q, m.dp);
    w.inner_max = m.p.ws_inner > 0 ? m.p.ws_inner : 4 * ws_q;
    DPSVM_CHECK(m.p.ws_wss >= 0 && m.p.ws_wss <= 2, "ws_wss must be 0 (auto), 1 (first order) or 2 (second order)");
    if (m.p.ws_wss > 0) {
      w.wss = m.p.ws_wss;
    } else {
      // auto: second order where the kernel couples rows (mean off-diagonal K of
      // a row sample: covtype-shape 0.85, synthetic-2m 0.85 -> WSS2 converges
      // covtype-200k in 21.2 s vs 27.7 s; MNIST-shape 0.0000, adult 0.0002 ->
      // WSS2 only adds ~0.25 us per pair step; profiles/r3_wss2_*.txt)
      w.wss = m.all_agree(coupling > kWsW2Coupling, m.comm, m.world) ? 2 : 1;
    }
    m.info.ws_wss = w.wss;
    DPSVM_CHECK(m.p.ws_t_halve >= 0.f && m.p.ws_t_halve <= 1.f, "ws_t_halve must be in [0, 1]");
    w.t_halve = m.p.ws_t_halve;
    w.clip_fallback = m.p.ws_clip_fallback ? 1 : 0;
    DPSVM_CHECK(m.p.ws_rel >= 0.f && m.p.ws_rel < 1.f, "ws_rel must be in [0, 1)");
    w.rel_local = m.p.ws_rel;
    static const float rel_local_env = [] {  // A/B: DPSVM_WS_REL_LOCAL (the gap fraction only; the floor keeps ws_rel)
      const char* e = std::getenv("DPSVM_WS_REL_LOCAL");
      return e ? (float)atof(e) : -1.f;
    }();
    if (rel_local_env > 0.f && rel_local_env < 1.f) w.rel_local = rel_local_env;
    // sub-problem tolerance ws_rel * max(eps, gap / 2): floored at ws_rel * eps
    // rather than eps, rounds near the end keep taking steps (adult-shape:
    // 0.230 -> 0.206 s; headline unchanged; profiles/r2_ws_param_sweep2.txt)
    w.eps_floor = m.p.ws_rel * m.p.eps;
    w.C = m.p.C;
    w.eps = m.p.eps;
    w.tau = m.p.tau;
    w.clip = (int)m.p.clip;
    w.max_iter = m.p.max_iter;
    // multi-block rounds (adaptive block count, ws_*.hip)
    w.blocks = 1;
    m.ws_q1 = ws_q;
    if (want_blocks > 1) {
      if (multi_ok) {
        w.blocks = want_blocks;
        w.q_max = mb_q;
        w.inner_max = m.p.ws_inner > 0 ? m.p.ws_inner : 4 * mb_q;
      }
      else if (m.p.ws_blocks > 1) m.info.engine_note += std::string(m.info.engine_note.empty() ? "" : "; ") +
                                 "ws_blocks > 1 needs an even ws_size, <= 256 candidate lists, the peer exchange or a "
                                 "device communicator, and (ws-cache) >= 2 P ws_size + 4096 lines: one block per round";
    }
    // multi-block rounds replace the whole union each round by default (measured on the
    // headline at P = 8: 3/4 q new 0.0506 s, all new 0.0493 s; profiles/r2_ws_blocks_sweep.txt)
    if (w.blocks > 1 && m.p.ws_new <= 0) w.n_new = w.q_max;
    // keys per selection list: the union's half per side over the lists with
    // room to spare (8 cover 3,072-row unions: 1,880 a side on the headline's 235)
    w.ncand = w.blocks * w.q_max > kWsAutoUnion ? kWsCand : kWsCandStd;
    // blocks of <= 64 rows at world 1 on the resident Gram: the solve loads its
    // q x q block itself (A/B: DPSVM_WS_DIRECT_SUB=0; 96-row blocks measured
    // slower that way in round 4: 9,216 loads a workgroup, profiles/r4_direct_subgram_ab.txt)
    static const int direct_env = [] {  // 0 off, 1 blocks of <= 64 rows (default), 2 <= 96 (A/B)
      const char* e = std::getenv("DPSVM_WS_DIRECT_SUB");
      return e ? atoi(e) : 1;
    }();
    const int direct_q = direct_env == 2 ? 96 : direct_env == 1 ? 64 : 0;
    w.direct_sub = w.blocks > 1 && w.q_max <= direct_q && m.world == 1 && !w.cache && !m.xch ? 1 : 0;
    w.rank = m.rank;
    w.aux_stride = w.blocks * kWsMax;
    // candidate lists: [world][G][2][kWsCand] (this rank's block is the all-gather source)
    m.wscand = dmalloc<uint64_t>((size_t)w.G_all * 2 * kWsCand, &m.bytes);
    m.wsctrl = dmalloc<WsCtrl>(1, &m.bytes);
    // sub-Gram [q_max][q_max] then aux [f | alpha | y]: the first q_max^2 + kWsMax
    // floats are the per-round sum all-reduce at world > 1
    // (multi-block: P sub-Grams, then P aux blocks)
    // (the one-block rounds' view: ws_size rows, gpu_engines.hip one_block)
    const size_t sub_floats = std::max((size_t)w.blocks * ((size_t)w.q_max * w.q_max + 3 * kWsMax),
                                       (size_t)ws_q * ws_q + 3 * kWsMax);
    m.wssub = dmalloc<float>(sub_floats, &m.bytes);
    HIP_CHECK(hipMemsetAsync(m.wssub, 0, sub_floats * 4, m.stream));
    w.cand = m.wscand;
    w.cand_out = m.wscand + (size_t)m.rank * w.G * 2 * kWsCand;
    w.subg = m.wssub;
    w.aux = m.wssub + (size_t)w.blocks * w.q_max * w.q_max;
    if (w.blocks > 1) {
      w.ks = ks_mb;
      w.p1G = p1G;
      w.p1v4 = p1v4 ? 1 : 0;
      m.wsdfs = dmalloc<float>((size_t)w.ks * m.nl, &m.bytes);
      m.wsdalpha = dmalloc<float>((size_t)n, &m.bytes);
      m.wspart = dmalloc<double>((size_t)2 * w.world * w.p1G * w.ks, &m.bytes);
      m.wssorted = dmalloc<uint64_t>((size_t)2 * kWsMaxGroups * kWsCand, &m.bytes);
      w.sorted = m.wssorted;
      HIP_CHECK(hipMemsetAsync(m.wsdalpha, 0, (size_t)n * 4, m.stream));
      w.dfs = m.wsdfs;
      w.dalpha = m.wsdalpha;
      w.part = m.wspart;
    }
    w.ctrl = m.wsctrl;
    w.status = m.status_d;
    w.stamps = m.stamps;
    if (m.xch) {
      w.xpeer = m.xpeer_d;
      w.xrank = m.rank;
      if (w.blocks > 1) {  // ws_xch_words_multi: candidates (kWsCand keys a side), partials, sub-Gram rows
        w.xcw = 4 * kWsCand;
        w.xpart = ws_xch_cand_words_multi(w.G_all);
        w.xsub = w.xpart + ws_xch_part_words((int64_t)w.world * w.p1G, w.ks);
        w.xsub_rows = (int64_t)w.blocks * w.q_max;  // the one-block view: its own q_max (gpu_engines.hip)
      } else {  // ws_xch_words
        w.xcw = 4 * kWsCand1;
        w.xsub = 2 * (int64_t)w.G_all * 4 * kWsCand1;
        w.xsub_rows = w.q_max;
      }
      w.xtimeout_ticks = (int64_t)(std::max(1e-6, m.p.xch_timeout_s) * 1e8);
    }
    if (w.cache && !m.replicated) {
      const int64_t rows = std::max<int64_t>((int64_t)w.blocks * w.q_max, ws_q);  // the round's misses at most
      m.wsxq = dmalloc<float>((size_t)rows * m.dp, &m.bytes);
      m.wsxqsq = dmalloc<float>((size_t)rows, &m.bytes);
      m.wsiota = dmalloc<int32_t>((size_t)rows, &m.bytes);
      if (m.gram_split) {
        m.wsxs = dmalloc<uint8_t>((size_t)rows * launch::split_row_u4(m.dp) * 16, &m.bytes);
        m.wsxsh = dmalloc<int32_t>((size_t)rows, &m.bytes);
      }
      std::vector<int32_t> io((size_t)rows);
      for (int64_t i = 0; i < rows; ++i) io[i] = (int32_t)i;
      HIP_CHECK(hipMemcpyAsync(m.wsiota, io.data(), io.size() * 4, hipMemcpyHostToDevice, m.stream));
      HIP_CHECK(hipStreamSynchronize(m.stream));
    }
    m.info.ws_rounds = "graph";
    ws_recompute_setup(m);
  }
  m.engine = gpu::make_engine(m.kind);
  m.info.iteration = engine_name(m.kind);
  m.info.exchange_mem = m.xch ? m.xch_mem : "none";
  m.info.exchange = m.xch ? (m.world > 1 ? "peer" : "loopback")
                          : (m.world > 1 || m.p.force_collectives ? "allreduce" : "none");
  if (m.working_set()) {
    m.info.ws_exchange = m.wsa.xpeer ? (m.world > 1 ? "peer" : "loopback")
                                     : (m.collectives() ? "collectives" : "none");
    // partitioned X in cache mode also sums each round's packed miss rows
    if (m.wsa.xpeer && m.ws_round_collectives()) m.info.ws_exchange += "+rows-allreduce";
  }
  if (m.working_set()) {
    m.info.ws_blocks = m.wsa.blocks;
    m.info.ws_q_max = m.wsa.q_max;
  }
  m.info.xch_selftest = m.xch_diag;
  m.info.comm_kind = m.comm ? m.comm->name() : "local";
  m.info.rows_per_group = m.working_set() ? (int64_t)m.wsa.rpt * kWsSelThreads : m.fused() ? m.RBf : kStepRows;
  m.info.groups = m.working_set() ? m.wsa.G : m.fused() ? m.Gf : m.G;
  m.info.poll_batch = m.xch && !m.working_set() ? launch::poll_batch(a) : 0;
  m.info.bytes_device = m.bytes;
  return m.info;
}

}  // namespace dpsvm
