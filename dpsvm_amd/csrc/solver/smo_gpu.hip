// Device-resident distributed SMO driver (one rank = one MI355X).
//
// Reference driver: svmTrainMain.cpp:142-365 + SvmTrain (svmTrain.cu:305-395).
// MI355X-first differences:
//   * the iteration never returns to the host: kernels read the pair, alphas
//     and cache decisions from a device control record; blocks of iterations
//     are captured into one hipGraph (collectives included) and the host only
//     polls a pinned host-mapped status record one block behind;
//   * with 288 GB of HBM the whole Gram shard K[n][n_local] is usually resident
//     ("dense" mode, computed by one MFMA GEMM); otherwise an O(1) device LRU
//     of kernel-row lines, filled by a multi-row MFMA X pass (+ speculative
//     rows) on a miss;
//   * X is replicated when it fits (no row broadcast needed), or partitioned
//     with the winning rows travelling in an all-gathered candidate record;
//   * the per-iteration collective is one element-wise MIN all-reduce of packed
//     u64 keys (exact, deterministic tie-break) instead of a host float
//     Allgather with indices cast to float (svmTrainMain.cpp:244).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <atomic>
#include <thread>

#include <unistd.h>

#include "dpsvm/device_state.hpp"
#include "dpsvm/solver.hpp"
#include "../kernels/kernels.hpp"
#include "../runtime/hip_check.hpp"
#include "../runtime/timer.hpp"
#include "../runtime/trace.hpp"

namespace dpsvm {
namespace {

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

template <class T>
T* dmalloc(size_t count, size_t* total) {
  void* p = nullptr;
  if (count == 0) count = 1;
  HIP_CHECK(hipMalloc(&p, count * sizeof(T)));
  *total += count * sizeof(T);
  return (T*)p;
}

double watchdog_seconds() {
  const char* e = std::getenv("DPSVM_WATCHDOG_S");
  return e ? atof(e) : 1800.0;
}

}  // namespace

struct GpuSolver::Impl {
  SolverParams p;
  Communicator* comm = nullptr;
  std::unique_ptr<Communicator> own_comm;
  int device = 0, rank = 0, world = 1;
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
  uint64_t* pf = nullptr;  // dense fused mode: two partial buffers [2][2*Gf]
  FusedRec* rf = nullptr;  // dense fused mode: two records
  FusedCacheRec* rcf = nullptr;  // fused cache mode: two records
  // peer exchange (dense fused mode): own receive buffer (own allocation, IPC
  // exported), device table of every rank's buffer, IPC mappings to close
  bool xch = false;
  bool persist = false;  // dense mode: persistent kernel, persist_block iterations per launch
  bool persist_lru = false;  // cache mode: persistent kernel with private per-workgroup cache metadata
  int32_t* plru_meta = nullptr;
  int64_t* plru_stats = nullptr;
  uint64_t* xbuf = nullptr;
  uint64_t** xpeer_d = nullptr;
  int64_t xregion = 0;  // u64 words of the two key parities (zeroed per solve)
  int64_t xstride = kXchGranules;  // u64 slots per exchange entry
  std::vector<void*> xopened;
  std::string xch_diag;
  std::string xch_mem = "none";  // receive-buffer memory kind (uncached across devices)
  int64_t Gf = 0, RBf = 0;
  uint64_t* stamps = nullptr;  // DPSVM_STAMPS diagnostics
  std::string stamps_path;
  // host staging for host-memory communicators
  std::vector<uint64_t> h_partials;
  std::vector<uint8_t> h_records;

  SmoArgs args{};
  float gamma = 0.f;
  int64_t n = 0, nl = 0, off = 0, x_rows = 0, G = 0, ldl = 0, L = 0;
  int d = 0, dp = 0;
  bool replicated = true, dense = false;
  bool fused_lru = false;  // cache mode with one fused launch per iteration
  std::vector<float> h_y;

  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  int graph_iters = 0;

  ~Impl() {
    if (device >= 0) (void)hipSetDevice(device);
    for (void* q : xopened) (void)hipIpcCloseMemHandle(q);
    if (xbuf) (void)hipFree(xbuf);
    if (xpeer_d) (void)hipFree(xpeer_d);
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    for (void* ptr : {(void*)x, (void*)xsq, (void*)y, (void*)alpha, (void*)f, (void*)lines,
                      (void*)slot_of, (void*)key_of, (void*)ref, (void*)hslot_of, (void*)hkey_of,
                      (void*)partials, (void*)ctrl, (void*)records, (void*)my_record, (void*)pf, (void*)rf, (void*)rcf, (void*)stamps,
                      (void*)plru_meta, (void*)plru_stats})
      if (ptr) (void)hipFree(ptr);
    if (status_h) (void)hipHostFree(status_h);
    if (hlines_h) (void)hipHostFree(hlines_h);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
  }

  SmoStatus read_status() const {
    SmoStatus s;
    std::atomic_thread_fence(std::memory_order_acquire);
    memcpy(&s, (const void*)status_h, sizeof(s));
    return s;
  }

  bool device_comm() const { return world == 1 || comm->device_memory(); }

  void init_ctrl(int64_t iter0, float b_hi, float b_lo) {
    SmoCtrl c;
    memset(&c, 0, sizeof(c));
    c.iter = (int32_t)iter0;
    c.line_hi = c.line_lo = -1;
    c.b_hi = b_hi;
    c.b_lo = b_lo;
    c.hand = 0;
    c.hhand = 0;
    HIP_CHECK(hipMemcpyAsync(ctrl, &c, sizeof(c), hipMemcpyHostToDevice, stream));
    memset(status_h, 0, sizeof(SmoStatus));
  }

  // one SMO iteration on `stream` (no host synchronisation for device comms)
  // dense fused iteration k of a block (k even <-> reads buffer 1, writes 0)
  void enqueue_fused(int k) {
    const int wi = k & 1, ri = wi ^ 1;
    uint64_t* pout = pf + (size_t)wi * 2 * Gf;
    if (fused_lru)
      launch::smo_fused_lru(args, pf + (size_t)ri * 2 * Gf, pout, rcf + ri, rcf + wi, stream);
    else
      launch::smo_fused(args, 1, pf + (size_t)ri * 2 * Gf, pout, rf + ri, rf + wi, stream);
    if (collectives() && !xch) allreduce_keys(pout, 2 * Gf);
  }

  bool collectives() const { return world > 1 || p.force_collectives; }

  void allreduce_keys(uint64_t* buf, int64_t count) {
    if (comm->device_memory()) {
      comm->allreduce_min_u64(buf, (size_t)count, stream);
    } else {
      if ((int64_t)h_partials.size() < count) h_partials.resize((size_t)count);
      HIP_CHECK(hipMemcpyAsync(h_partials.data(), buf, 8 * count, hipMemcpyDeviceToHost, stream));
      HIP_CHECK(hipStreamSynchronize(stream));
      comm->allreduce_min_u64(h_partials.data(), (size_t)count, nullptr);
      HIP_CHECK(hipMemcpyAsync(buf, h_partials.data(), 8 * count, hipMemcpyHostToDevice, stream));
    }
  }

  bool fused() const { return dense || fused_lru; }

  // byte all-gather through the communicator (host or device memory)
  void allgather_bytes(const void* send, void* recv, size_t bytes) {
    if (world == 1) {
      memcpy(recv, send, bytes);
      return;
    }
    if (comm->device_memory()) {
      size_t tb = 0;
      uint8_t* d = dmalloc<uint8_t>(bytes * (world + 1), &tb);
      HIP_CHECK(hipMemcpy(d + bytes * world, send, bytes, hipMemcpyHostToDevice));
      comm->allgather(d + bytes * world, d, bytes, stream);
      HIP_CHECK(hipMemcpyAsync(recv, d, bytes * world, hipMemcpyDeviceToHost, stream));
      HIP_CHECK(hipStreamSynchronize(stream));
      (void)hipFree(d);
    } else {
      comm->allgather(send, recv, bytes, nullptr);
    }
  }

  // Peer exchange setup (collective over the communicator): receive buffers,
  // pointer / IPC-handle all-gather, mapping, and an in-kernel ping that every
  // rank must pass.  Returns false (everywhere) if any rank failed.
  bool setup_exchange() {
    struct alignas(16) XInfo {
      int64_t pid, device, ok;
      uint64_t ptr;
      hipIpcMemHandle_t handle;
    };
    XInfo me{};
    me.pid = (int64_t)getpid();
    me.device = device;
    me.ok = 1;
    const int64_t ping_words = 64;
    xstride = kXchGranules;
    if (const char* e = std::getenv("DPSVM_XCH_STRIDE")) xstride = std::max(kXchGranules, atoi(e));
    xregion = (int64_t)2 * world * Gf * xstride;
    try {
      DPSVM_CHECK(world <= 64, "peer exchange supports at most 64 ranks");
      launch::preload_fused_kernels(stream);
      launch::preload_persist_kernel(stream);
      launch::preload_persist_lru_kernel(stream);
      // own allocation (IPC export).  Ranks on other devices write it over xGMI:
      // uncached device memory, so no L2 of this device can hold a stale line of
      // a granule a peer rewrote (coarse-grained memory is only coherent within
      // one device); DPSVM_XCH_MEM=coarse keeps plain hipMalloc memory
      const size_t xbytes = (size_t)(xregion + ping_words) * 8;
      const char* xm = std::getenv("DPSVM_XCH_MEM");
      const std::string xms = xm ? xm : "";
      const bool uncached = (world > 1 || xms == "uncached") && xms != "coarse";
      const bool got_uc = uncached && hipExtMallocWithFlags((void**)&xbuf, xbytes, hipDeviceMallocUncached) == hipSuccess;
      if (!got_uc) {
        (void)hipGetLastError();
        xbuf = nullptr;
        HIP_CHECK(hipMalloc((void**)&xbuf, xbytes));
      }
      xch_mem = got_uc ? "uncached" : "coarse";
      HIP_CHECK(hipMemset(xbuf, 0, (size_t)(xregion + ping_words) * 8));
      HIP_CHECK(hipDeviceSynchronize());
      me.ptr = (uint64_t)xbuf;
      if (world > 1) HIP_CHECK(hipIpcGetMemHandle(&me.handle, xbuf));
    } catch (const std::exception& e) {
      if (p.verbose) fprintf(stderr, "[dpsvm] peer exchange unavailable on rank %d: %s\n", rank, e.what());
      me.ok = 0;
    }
    std::vector<XInfo> all((size_t)world);
    allgather_bytes(&me, all.data(), sizeof(XInfo));
    bool ok = true;
    for (const auto& r : all) ok &= r.ok != 0;
    for (int r = 0; r < world; ++r) {
      // rank threads of one process on one device: their streams may share a
      // hardware queue, so one spinning kernel can block the other's forever
      if (r != rank && all[r].pid == me.pid && all[r].device == me.device) {
        ok = false;
        xch_diag = "ranks " + std::to_string(rank) + " and " + std::to_string(r) + " share a device in one process";
      }
    }
    std::vector<uint64_t*> ptrs((size_t)world, nullptr);
    if (ok) {
      try {
        for (int r = 0; r < world; ++r) {
          if (r == rank) {
            ptrs[r] = xbuf;
          } else if (all[r].pid == me.pid) {  // rank thread of this process: direct pointer
            ptrs[r] = (uint64_t*)all[r].ptr;
            if (all[r].device != device) {
              const hipError_t e = hipDeviceEnablePeerAccess((int)all[r].device, 0);
              if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
              (void)hipGetLastError();
            }
          } else {  // other process: dmabuf IPC mapping (xGMI peer memory)
            void* q = nullptr;
            HIP_CHECK(hipIpcOpenMemHandle(&q, all[r].handle, hipIpcMemLazyEnablePeerAccess));
            xopened.push_back(q);
            ptrs[r] = (uint64_t*)q;
          }
        }
        size_t tb = 0;
        xpeer_d = dmalloc<uint64_t*>((size_t)world, &tb);
        HIP_CHECK(hipMemcpy(xpeer_d, ptrs.data(), world * sizeof(uint64_t*), hipMemcpyHostToDevice));
      } catch (const std::exception& e) {
        if (p.verbose) fprintf(stderr, "[dpsvm] peer mapping failed on rank %d: %s\n", rank, e.what());
        ok = false;
      }
    }
    // in-kernel self test (a rank that failed above does not ping: the others time out)
    size_t tb = 0;
    int32_t* okd = dmalloc<int32_t>(2, &tb);
    uint64_t* agree = dmalloc<uint64_t>(1, &tb);
    HIP_CHECK(hipMemset(okd, 0, 8));
    if (world > 1) comm->barrier();
    if (ok) launch::xch_ping(xpeer_d, rank, world, xregion, 1u, (int64_t)5e8 /* 5 s */, okd, stream);
    int32_t okh = 0;
    HIP_CHECK(hipMemcpyAsync(&okh, okd, 4, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    if (xch_diag.empty())
      xch_diag = "rank " + std::to_string(rank) + ": mapped=" + std::to_string((int)ok) + " ping=" + std::to_string(okh);
    const uint64_t mine = (ok && okh == 1) ? 0ull : 1ull;
    uint64_t v = ~mine;  // all ok -> every rank holds ~0; any failure -> some rank holds ~1 (smaller)
    HIP_CHECK(hipMemcpy(agree, &v, 8, hipMemcpyHostToDevice));
    if (world > 1) allreduce_keys(agree, 1);
    HIP_CHECK(hipMemcpyAsync(&v, agree, 8, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    (void)hipFree(okd);
    (void)hipFree(agree);
    const bool all_ok = v == ~0ull;
    if (!all_ok) {
      for (void* q : xopened) (void)hipIpcCloseMemHandle(q);
      xopened.clear();
      if (xbuf) (void)hipFree(xbuf);
      if (xpeer_d) (void)hipFree(xpeer_d);
      xbuf = nullptr;
      xpeer_d = nullptr;
    }
    if (world > 1) comm->barrier();
    return all_ok;
  }

  void enqueue_iteration(int k) {
    if (fused()) {
      enqueue_fused(k);
      return;
    }
    launch::smo_rows(args, stream);
    launch::smo_step(args, stream);
    if (collectives()) {
      if (replicated) {
        if (comm->device_memory()) {
          comm->allreduce_min_u64(partials, 2 * (size_t)G, stream);
        } else {
          HIP_CHECK(hipMemcpyAsync(h_partials.data(), partials, 16 * G, hipMemcpyDeviceToHost, stream));
          HIP_CHECK(hipStreamSynchronize(stream));
          comm->allreduce_min_u64(h_partials.data(), 2 * (size_t)G, nullptr);
          HIP_CHECK(hipMemcpyAsync(partials, h_partials.data(), 16 * G, hipMemcpyHostToDevice, stream));
        }
      } else {
        launch::smo_local_record(args, stream);
        const size_t rb = (size_t)args.rec_bytes;
        if (comm->device_memory()) {
          comm->allgather(my_record, records, rb, stream);
        } else {
          HIP_CHECK(hipMemcpyAsync(h_records.data() + rank * rb, my_record, rb, hipMemcpyDeviceToHost, stream));
          HIP_CHECK(hipStreamSynchronize(stream));
          comm->allgather(h_records.data() + rank * rb, h_records.data(), rb, nullptr);
          HIP_CHECK(hipMemcpyAsync(records, h_records.data(), rb * world, hipMemcpyHostToDevice, stream));
        }
      }
    } else if (!replicated) {
      // single-rank partitioned (tests): the local record is the whole world
      launch::smo_local_record(args, stream);
      HIP_CHECK(hipMemcpyAsync(records, my_record, args.rec_bytes, hipMemcpyDeviceToDevice, stream));
    }
    launch::smo_finalize(args, stream);
  }

  void build_graph(int iters) {
    if (gexec) return;
    HIP_CHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
    try {
      for (int i = 0; i < iters; ++i) enqueue_iteration(i);
    } catch (...) {
      hipGraph_t g;
      (void)hipStreamEndCapture(stream, &g);
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
      throw;
    }
    HIP_CHECK(hipStreamEndCapture(stream, &graph));
    HIP_CHECK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
    graph_iters = iters;
  }

  // Checkpoint snapshot (stream drained by the caller): alpha is replicated,
  // the f shards are all-gathered; rank 0 writes.
  void snapshot(const SmoStatus& st) {
    Checkpoint ck;
    ck.n = n; ck.d = d; ck.C = p.C; ck.gamma = gamma; ck.eps = p.eps;
    ck.clip = (int)p.clip; ck.iter = st.iter; ck.b_hi = st.b_hi; ck.b_lo = st.b_lo;
    ck.alpha.resize((size_t)n);
    HIP_CHECK(hipMemcpy(ck.alpha.data(), alpha, n * 4, hipMemcpyDeviceToHost));
    if (fused()) {
      // the latest pair's alphas are still pending in the record of the last
      // kernel (blocks have even length: the last kernel wrote record 1)
      // (the record is exact; the host-mapped status refreshes every kStatusEvery)
      int32_t ih = -1, il = -1;
      float ah = 0.f, al = 0.f;
      if (dense || persist_lru) {
        FusedRec r;
        HIP_CHECK(hipMemcpy(&r, rf + 1, sizeof(r), hipMemcpyDeviceToHost));
        ih = r.i_hi; il = r.i_lo; ah = r.a_hi; al = r.a_lo;
        ck.iter = r.iter; ck.b_hi = r.b_hi; ck.b_lo = r.b_lo;
      } else {
        FusedCacheRec r;
        HIP_CHECK(hipMemcpy(&r, rcf + 1, sizeof(r), hipMemcpyDeviceToHost));
        ih = r.i_hi; il = r.i_lo; ah = r.a_hi; al = r.a_lo;
        ck.iter = r.iter; ck.b_hi = r.b_hi; ck.b_lo = r.b_lo;
      }
      if (ih >= 0) {
        ck.alpha[il] = al;
        ck.alpha[ih] = ah;
      }
    }
    std::vector<float> floc((size_t)ldl, 0.f), fall((size_t)ldl * world);
    HIP_CHECK(hipMemcpy(floc.data(), f, nl * 4, hipMemcpyDeviceToHost));
    if (world > 1) {
      if (comm->device_memory()) {
        size_t tb = 0;
        float* gb = dmalloc<float>((size_t)ldl * world, &tb);
        HIP_CHECK(hipMemcpy(gb + (size_t)rank * ldl, f, ldl * 4, hipMemcpyDeviceToDevice));
        comm->allgather(gb + (size_t)rank * ldl, gb, ldl * 4, stream);
        HIP_CHECK(hipMemcpyAsync(fall.data(), gb, fall.size() * 4, hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
        (void)hipFree(gb);
      } else {
        comm->allgather(floc.data(), fall.data(), ldl * 4, nullptr);
      }
    } else {
      fall = floc;
    }
    ck.f.assign((size_t)n, 0.f);
    for (int r = 0; r < world; ++r) {
      Shard s = shard_of(n, r, world);
      std::copy(fall.begin() + (size_t)r * ldl, fall.begin() + (size_t)r * ldl + s.size, ck.f.begin() + s.offset);
    }
    if (rank == 0) write_checkpoint(p.checkpoint_path, ck);
  }

  void wait_event(hipEvent_t e) {
    // bounded wait with async-error polling (SURVEY §5.3 watchdog)
    auto t0 = Clock::now();
    const double limit = watchdog_seconds();
    int spins = 0;
    while (true) {
      hipError_t q = hipEventQuery(e);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) HIP_CHECK(q);
      if (world > 1) {
        std::string err = comm->async_error();
        if (!err.empty()) {
          comm->abort();
          fail("collective failed on rank " + std::to_string(rank) + ": " + err);
        }
      }
      if (secs_since(t0) > limit) {
        if (world > 1) comm->abort();
        fail("watchdog: SMO block did not finish within " + std::to_string(limit) + " s");
      }
      if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
};

GpuSolver::GpuSolver(const SolverParams& p, Communicator* comm, int device) : impl_(new Impl) {
  auto& m = *impl_;
  m.p = p;
  if (!comm) {
    m.own_comm = make_local_comm();
    comm = m.own_comm.get();
  }
  m.comm = comm;
  m.rank = comm->rank();
  m.world = comm->size();
  m.device = device;
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&m.ev[0], hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&m.ev[1], hipEventDisableTiming));
}

GpuSolver::~GpuSolver() = default;
const GpuSetupInfo& GpuSolver::info() const { return impl_->info; }

GpuSetupInfo GpuSolver::setup(const float* xh, int64_t n_x_rows, int64_t n, int d, const float* yh) {
  auto& m = *impl_;
  HIP_CHECK(hipSetDevice(m.device));
  DPSVM_CHECK(n >= 2 && d >= 1, "need at least 2 samples and 1 feature");
  DPSVM_CHECK(n < (int64_t)1 << 31, "n must fit in 31 bits (packed selection keys)");
  DPSVM_CHECK(m.p.C > 0.f, "C must be > 0");
  m.n = n;
  m.d = d;
  m.dp = pad_features(d);
  m.gamma = resolve_gamma(m.p.gamma, d);
  const Shard sh = shard_of(n, m.rank, m.world);
  m.nl = sh.size;
  m.off = sh.offset;
  const int64_t nl_max = (n + m.world - 1) / m.world;
  m.G = std::max<int64_t>(1, (nl_max + kStepRows - 1) / kStepRows);
  // fused-iteration geometry, rows per workgroup a multiple of 256.  Cache mode:
  // <= ~256 workgroups (the X pass wants every CU).  Dense mode: the period is
  // set by the all-to-all key exchange, whose cost grows with the number of
  // publishers (world x G): ~128 publishers in all, <= 1024 rows per workgroup
  // (more only to keep one poll batch / <= 256 resident workgroups:
  // dense_rows_min, common.hpp).  Measured on 60k x 784, 1 GPU:
  // 235 workgroups 5.8-6.2 us per iteration, 118 -> 5.2 us (profiles/README.md).
  int64_t wgs = 256;  // cache mode: one workgroup per CU
  if (const char* e = std::getenv("DPSVM_CACHE_WGS")) wgs = std::max<int64_t>(1, atoll(e));
  auto geometry = [&](int64_t rows_min) {
    Geometry g = make_geometry(nl_max, rows_min, wgs);
    if (const char* e = std::getenv("DPSVM_FUSED_ROWS")) {  // override: rows per workgroup
      const int64_t r = atoll(e) / kFusedThreads * kFusedThreads;
      if (r > g.rows) g = make_geometry(nl_max, r, wgs);
    }
    return std::pair<int64_t, int64_t>(g.rows, g.groups);
  };
  const auto geo_cache = geometry(0);
  int64_t dense_rows = dense_rows_min(nl_max, m.world);
  if (const char* e = std::getenv("DPSVM_DENSE_ROWS"))  // tests: more publishers (multi-batch polls)
    dense_rows = std::max<int64_t>(kFusedThreads, std::min<int64_t>(3072, atoll(e) / kFusedThreads * kFusedThreads));
  auto geo_dense = geometry(dense_rows);
  if (std::getenv("DPSVM_DENSE_ROWS"))
    geo_dense = {dense_rows, std::max<int64_t>(1, (nl_max + dense_rows - 1) / dense_rows)};
  m.RBf = geo_cache.first;
  m.Gf = geo_cache.second;
  // lines cover every row a kernel may write (the fused X pass writes whole
  // 256-row tiles) under either geometry
  m.ldl = std::max<int64_t>({m.G * kStepRows, geo_cache.first * geo_cache.second,
                             geo_dense.first * geo_dense.second});

  // ---- X placement ----
  if (n_x_rows == n) {
    m.replicated = m.p.x_mode != 2;
  } else {
    DPSVM_CHECK(n_x_rows == m.nl, "x must hold all n rows (replicated) or this rank's shard rows");
    m.replicated = false;
  }
  if (m.world == 1 && m.p.x_mode == 2) m.replicated = false;
  size_t freeb = 0, totalb = 0;
  HIP_CHECK(hipMemGetInfo(&freeb, &totalb));
  if (m.replicated && m.p.x_mode == 0 && m.world > 1) {
    // auto: replicate unless X would take more than 40% of free HBM
    const double xbytes = (double)n * m.dp * 4.0;
    if (xbytes > 0.4 * (double)freeb) m.replicated = false;
    DPSVM_CHECK(m.replicated || n_x_rows == n, "internal: partition fallback needs full x");
  }
  const int64_t x_row0 = m.replicated ? 0 : m.off;
  m.x_rows = m.replicated ? round_up(std::max<int64_t>(n, m.off + m.ldl), 128) + 128 : m.ldl + 128;
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
  const int64_t n_pad = round_up(std::max<int64_t>(n, m.off + m.ldl), 128) + 128;
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
      HIP_CHECK(hipStreamSynchronize(m.stream));
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
  HIP_CHECK(hipStreamSynchronize(m.stream));

  // ---- kernel-row cache sizing (288 GB HBM: the Gram shard is usually resident) ----
  HIP_CHECK(hipMemGetInfo(&freeb, &totalb));
  const double line_bytes = (double)m.ldl * 4.0;
  double budget = m.p.cache_frac * (double)freeb - 256.0 * 1024 * 1024;
  if (m.p.cache_mb > 0) budget = std::min(budget, m.p.cache_mb * 1024.0 * 1024.0);
  int64_t want_lines = (int64_t)(budget / line_bytes);
  if (m.p.cache_lines > 0) want_lines = std::min<int64_t>(want_lines, m.p.cache_lines);
  m.dense = m.replicated && want_lines >= n;
  if (const char* e = std::getenv("DPSVM_FORCE_LRU")) if (e[0] == '1') m.dense = false;
  if (m.dense) {
    m.RBf = geo_dense.first;
    m.Gf = geo_dense.second;
  }
  // cache mode, persistent engine candidate: every workgroup's private metadata
  // copy comes out of the line budget (upper bound: L = n)
  const char* ple = std::getenv("DPSVM_PERSIST_LRU");
  const bool plru_cand = !m.dense && m.replicated && m.p.host_cache_lines == 0 && m.p.persist != 1 &&
                         !(ple && ple[0] == '0') && m.p.use_graph && !m.p.force_collectives &&
                         launch::smo_persist_lru_supported(m.dp, (int)m.RBf, (int)m.Gf);
  if (plru_cand) {
    const double meta_bytes = (double)m.Gf * launch::plru_stride_words(n, n) * 4.0;
    want_lines = std::min<int64_t>(want_lines, (int64_t)((budget - meta_bytes) / line_bytes));
  }
  m.L = m.dense ? n : std::max<int64_t>(2, std::min<int64_t>(want_lines, n));
  DPSVM_CHECK(m.L * line_bytes <= (double)freeb, "not enough device memory for 2 kernel-row lines");
  m.lines = dmalloc<float>((size_t)m.L * m.ldl, &m.bytes);
  // cache mode with replicated X: one fused launch per iteration
  // (DPSVM_LRU_KERNELS=3 keeps the rows/step/finalize chain, e.g. for A/B runs)
  const char* lk = std::getenv("DPSVM_LRU_KERNELS");
  m.fused_lru = !m.dense && m.replicated && launch::smo_fused_lru_supported(m.dp) && !(lk && lk[0] == '3');
  if (m.fused()) {
    m.pf = dmalloc<uint64_t>((size_t)4 * m.Gf, &m.bytes);
    if (m.dense || plru_cand) m.rf = dmalloc<FusedRec>(2, &m.bytes);
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
  if (const char* sp = std::getenv("DPSVM_STAMPS")) {
    m.stamps_path = std::string(sp) + ".rank" + std::to_string(m.rank);
    const size_t cnt = (size_t)kStampRing * 2 * kStampSlots;
    m.stamps = dmalloc<uint64_t>(cnt, &m.bytes);
    HIP_CHECK(hipMemset(m.stamps, 0, cnt * 8));
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
  m.info.iteration = m.dense ? "fused-dense" : (m.fused_lru ? "fused-cache" : "chain");
  // ---- per-iteration key exchange ----
  a.xpeer = nullptr;
  a.xrank = 0;
  a.xworld = 0;
  a.xstride = kXchGranules;
  a.xpoll_kb = 0;
  a.xpoll_sleep = 1;
  a.xtimeout_ticks = 0;
  m.xch = false;
  bool want_persist = false;
  if (m.dense && m.replicated) {
    const char* pe = std::getenv("DPSVM_PERSIST");
    int mode = m.p.persist;
    if (pe && pe[0]) mode = pe[0] == '1' ? 2 : 1;
    // auto: persistent unless the exchange is pinned to the communicator all-reduce
    // (and unless a test forces the per-iteration collective path or eager launches)
    want_persist = mode == 2 || (mode == 0 && m.p.exchange != 1 && m.p.use_graph && !m.p.force_collectives);
    // register-resident rows and one resident workgroup per CU (launch::smo_persist)
    want_persist = want_persist && m.RBf <= 12 * kFusedThreads && m.Gf <= 256;
  }
  // cache mode: the persistent cache engine (same exchange) unless the exchange
  // is pinned to the communicator all-reduce or the geometry does not fit it
  const bool want_plru = plru_cand && m.fused_lru && m.p.exchange != 1;
  if ((m.dense && ((m.p.exchange != 1 && (m.world > 1 || m.p.exchange == 2)) || want_persist)) || want_plru) {
    const bool ok = m.setup_exchange();
    DPSVM_CHECK(ok || (m.p.exchange != 2 && m.p.persist != 2),
                "peer exchange requested (exchange=2 / persist=2) but its self test failed (" + m.xch_diag + ")");
    if (ok) {
      double tmo = 120.0;
      if (const char* e = std::getenv("DPSVM_XCH_TIMEOUT_S")) tmo = std::max(1e-6, atof(e));  // tiny: tests
      m.xch = true;
      a.xpeer = m.xpeer_d;
      a.xrank = m.rank;
      a.xworld = m.world;
      a.xstride = (int32_t)m.xstride;
      const char* kb = std::getenv("DPSVM_XCH_KB");
      a.xpoll_kb = kb ? atoi(kb) : 0;
      const char* ps = std::getenv("DPSVM_XCH_SLEEP");
      a.xpoll_sleep = ps ? atoi(ps) : 1;
      a.xtimeout_ticks = (int64_t)(tmo * 1e8);
    }
  }
  m.info.exchange_mem = m.xch ? m.xch_mem : "none";
  m.info.exchange = m.xch ? (m.world > 1 ? "peer" : "loopback")
                          : (m.world > 1 || m.p.force_collectives ? "allreduce" : "none");
  m.persist = want_persist && m.xch;
  if (m.persist) m.info.iteration = "persistent-dense";
  m.persist_lru = want_plru && m.xch;
  a.plru_meta = nullptr;
  a.plru_stride = 0;
  if (m.persist_lru) {
    a.plru_stride = launch::plru_stride_words(n, m.L);
    m.plru_meta = dmalloc<int32_t>((size_t)m.Gf * a.plru_stride, &m.bytes);
    m.plru_stats = dmalloc<int64_t>(8, &m.bytes);
    a.plru_meta = m.plru_meta;
    m.info.iteration = "persistent-cache";
  }
  m.info.bytes_device = m.bytes;
  return m.info;
}

// Support-vector set (rows, |x|^2, alpha*y) gathered from a host alpha; every rank
// ends with all SVs (padded per-rank blocks in partitioned mode).
namespace {
struct SvSet {
  int64_t nsv = 0;
  float *sv = nullptr, *svsq = nullptr, *coef = nullptr;
  size_t bytes = 0;
  ~SvSet() {
    for (void* p : {(void*)sv, (void*)svsq, (void*)coef}) if (p) (void)hipFree(p);
  }
};
}  // namespace

static void build_svs(GpuSolver::Impl& m, const SolveResult& r, SvSet& s) {
  HIP_CHECK(hipMemcpyAsync(m.alpha, r.alpha.data(), m.n * 4, hipMemcpyHostToDevice, m.stream));
  std::vector<int32_t> local_idx;
  if (m.replicated) {
    size_t tb = 0;
    int32_t* idx = dmalloc<int32_t>((size_t)m.n, &tb);
    int32_t* cnt = dmalloc<int32_t>(1, &tb);
    int32_t* scratch = dmalloc<int32_t>((size_t)launch::compact_scratch_ints(m.n), &tb);
    launch::compact_positive(m.alpha, m.n, idx, cnt, scratch, m.stream);
    int32_t nsv = 0;
    HIP_CHECK(hipMemcpyAsync(&nsv, cnt, 4, hipMemcpyDeviceToHost, m.stream));
    HIP_CHECK(hipStreamSynchronize(m.stream));
    s.nsv = nsv;
    const int64_t pad = round_up(std::max<int64_t>(nsv, 1), 128) + 128;
    s.sv = dmalloc<float>((size_t)pad * m.dp, &s.bytes);
    s.svsq = dmalloc<float>((size_t)pad, &s.bytes);
    s.coef = dmalloc<float>((size_t)pad, &s.bytes);
    HIP_CHECK(hipMemsetAsync(s.sv, 0, (size_t)pad * m.dp * 4, m.stream));
    HIP_CHECK(hipMemsetAsync(s.svsq, 0, pad * 4, m.stream));
    HIP_CHECK(hipMemsetAsync(s.coef, 0, pad * 4, m.stream));
    launch::gather_sv(m.x, 0, m.xsq, m.alpha, m.y, idx, nsv, m.dp, s.sv, s.svsq, s.coef, m.stream);
    HIP_CHECK(hipStreamSynchronize(m.stream));
    for (void* p : {(void*)idx, (void*)cnt, (void*)scratch}) (void)hipFree(p);
  } else {
    // partitioned: each rank gathers its local SVs; all-gather padded blocks
    for (int64_t j = 0; j < m.nl; ++j)
      if (r.alpha[m.off + j] > 0.f) local_idx.push_back((int32_t)(m.off + j));
    std::vector<double> cnts((size_t)m.world, 0.0);
    cnts[m.rank] = (double)local_idx.size();
    if (m.world > 1) {
      if (m.comm->device_memory()) {
        size_t tb = 0;
        double* dc = dmalloc<double>((size_t)m.world, &tb);
        HIP_CHECK(hipMemcpy(dc, cnts.data(), m.world * 8, hipMemcpyHostToDevice));
        m.comm->allreduce_sum_f64(dc, m.world, m.stream);
        HIP_CHECK(hipMemcpyAsync(cnts.data(), dc, m.world * 8, hipMemcpyDeviceToHost, m.stream));
        HIP_CHECK(hipStreamSynchronize(m.stream));
        (void)hipFree(dc);
      } else {
        m.comm->allreduce_sum_f64(cnts.data(), m.world, nullptr);
      }
    }
    int64_t maxc = 0, total = 0;
    for (double c : cnts) { maxc = std::max<int64_t>(maxc, (int64_t)c); total += (int64_t)c; }
    const int64_t per = std::max<int64_t>(1, maxc);
    const int64_t pad = round_up(per * m.world, 128) + 128;
    s.sv = dmalloc<float>((size_t)pad * m.dp, &s.bytes);
    s.svsq = dmalloc<float>((size_t)pad, &s.bytes);
    s.coef = dmalloc<float>((size_t)pad, &s.bytes);
    HIP_CHECK(hipMemsetAsync(s.sv, 0, (size_t)pad * m.dp * 4, m.stream));
    HIP_CHECK(hipMemsetAsync(s.svsq, 0, pad * 4, m.stream));
    HIP_CHECK(hipMemsetAsync(s.coef, 0, pad * 4, m.stream));
    size_t tb = 0;
    int32_t* didx = dmalloc<int32_t>(std::max<size_t>(1, local_idx.size()), &tb);
    if (!local_idx.empty()) {
      HIP_CHECK(hipMemcpyAsync(didx, local_idx.data(), local_idx.size() * 4, hipMemcpyHostToDevice, m.stream));
      launch::gather_sv(m.x, m.args.x_row0, m.xsq, m.alpha, m.y, didx, (int64_t)local_idx.size(), m.dp,
                        s.sv + (size_t)m.rank * per * m.dp, s.svsq + m.rank * per, s.coef + m.rank * per,
                        m.stream);
    }
    HIP_CHECK(hipStreamSynchronize(m.stream));
    (void)hipFree(didx);
    if (m.world > 1) {
      // zero-padded blocks; coef = 0 on padding rows makes them inert
      auto gather = [&](float* buf, int64_t elems) {
        if (m.comm->device_memory()) {
          m.comm->allgather(buf + (size_t)m.rank * elems, buf, elems * 4, m.stream);
          HIP_CHECK(hipStreamSynchronize(m.stream));
        } else {
          std::vector<float> h((size_t)elems * m.world);
          HIP_CHECK(hipMemcpy(h.data() + (size_t)m.rank * elems, buf + (size_t)m.rank * elems, elems * 4,
                              hipMemcpyDeviceToHost));
          m.comm->allgather(h.data() + (size_t)m.rank * elems, h.data(), elems * 4, nullptr);
          HIP_CHECK(hipMemcpy(buf, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        }
      };
      gather(s.sv, per * m.dp);
      gather(s.svsq, per);
      gather(s.coef, per);
    }
    s.nsv = per * m.world;
    (void)total;
  }
}


// f-style decision values of this rank's rows without b: out_j = sum_i alpha_i y_i K(i, j)
// for j in [off, off + nl), from a host alpha (length n).  Used to rebuild f on resume and
// by the DPSVM_VERIFY consistency check; collective in partitioned mode (SV all-gather).
static void local_decision(GpuSolver::Impl& m, const std::vector<float>& alpha, float* out_dev) {
  SolveResult tmp;
  tmp.alpha = alpha;
  SvSet s;
  build_svs(m, tmp, s);
  size_t tb = 0;
  float* part = dmalloc<float>((size_t)launch::predict_scratch_floats(m.nl, s.nsv), &tb);
  const int64_t lrow = m.off - m.args.x_row0;
  launch::rbf_predict(m.x + (size_t)lrow * m.dp, m.xsq + m.off, m.nl, m.dp, s.sv, s.svsq, s.coef, s.nsv,
                      m.dp, m.dp, m.gamma, 0.f, part, out_dev, nullptr, nullptr, m.stream);
  HIP_CHECK(hipStreamSynchronize(m.stream));
  (void)hipFree(part);
}

SolveResult GpuSolver::solve(const Checkpoint* resume, const ProgressFn& progress) {
  auto& m = *impl_;
  HIP_CHECK(hipSetDevice(m.device));
  SolveResult res;
  res.world = m.world;
  res.cache_lines = m.L;
  auto ts0 = Clock::now();

  // ---- state init (alpha = 0, f = -y, empty cache) or resume ----
  int64_t iter0 = 0;
  float b_hi0 = 0.f, b_lo0 = 0.f;
  HIP_CHECK(hipMemsetAsync(m.alpha, 0, m.n * 4, m.stream));
  if (resume) {
    DPSVM_CHECK(resume->n == m.n && (int64_t)resume->alpha.size() == m.n, "checkpoint n mismatch");
    HIP_CHECK(hipMemcpyAsync(m.alpha, resume->alpha.data(), m.n * 4, hipMemcpyHostToDevice, m.stream));
    iter0 = resume->iter;
    b_hi0 = resume->b_hi;
    b_lo0 = resume->b_lo;
  }
  if (resume && (int64_t)resume->f.size() == m.n) {
    HIP_CHECK(hipMemcpyAsync(m.f, resume->f.data() + m.off, m.nl * 4, hipMemcpyHostToDevice, m.stream));
  } else if (resume) {
    // f_j = sum_i alpha_i y_i K(i, j) - y_j via the predict GEMM (b = 0)
    local_decision(m, resume->alpha, m.f);
    std::vector<float> fh((size_t)m.nl);
    HIP_CHECK(hipMemcpy(fh.data(), m.f, m.nl * 4, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < m.nl; ++j) fh[j] -= m.h_y[m.off + j];
    HIP_CHECK(hipMemcpy(m.f, fh.data(), m.nl * 4, hipMemcpyHostToDevice));
  } else {
    launch::init_f(m.y, m.off, m.nl, m.f, m.stream);
  }
  if (!m.dense) {
    launch::fill_i32(m.slot_of, m.n, -1, m.stream);
    launch::fill_i32(m.key_of, m.L, -1, m.stream);
    HIP_CHECK(hipMemsetAsync(m.ref, 0, m.L, m.stream));
    if (m.H > 0) {
      launch::fill_i32(m.hslot_of, m.n, -1, m.stream);
      launch::fill_i32(m.hkey_of, m.H, -1, m.stream);
    }
    if (m.persist_lru) {  // every workgroup's private copy: empty cache, hand 0
      launch::plru_init(m.plru_meta, m.args.plru_stride, m.Gf, m.n, m.L, m.stream);
      HIP_CHECK(hipMemsetAsync(m.plru_stats, 0, 8 * sizeof(int64_t), m.stream));
    }
  }
  m.init_ctrl(iter0, b_hi0, b_lo0);
  if (m.xch) HIP_CHECK(hipMemsetAsync(m.xbuf, 0, (size_t)m.xregion * 8, m.stream));  // tags restart at iter0 + 1
  HIP_CHECK(hipStreamSynchronize(m.stream));
  if (m.world > 1) m.comm->barrier();
  res.t_setup = secs_since(ts0);

  // ================= timed region: the SMO loop (svmTrainMain.cpp:206-314) =================
  trace::Range loop_range("dpsvm/solve");
  const int64_t fault_iter = trace::fault_nan_iter();
  bool fault_done = false;
  auto t0 = Clock::now();
  EventTimer gram_timer;
  if (m.persist_lru) {
    // seed: "no pending pair" record + initial keys published to the exchange
    FusedRec r0;
    r0.i_hi = r0.i_lo = -1;
    r0.a_hi = r0.a_lo = 0.f;
    r0.iter = (int32_t)iter0;
    r0.done = kRunning;
    r0.b_hi = b_hi0;
    r0.b_lo = b_lo0;
    HIP_CHECK(hipMemcpyAsync(m.rf + 1, &r0, sizeof(r0), hipMemcpyHostToDevice, m.stream));
    launch::smo_fused(m.args, 0, nullptr, m.pf + 2 * m.Gf, m.rf + 1, nullptr, m.stream);
  } else if (m.fused_lru) {
    // seed: record "no pending pair, empty cache" in buffer 1 + initial keys
    FusedCacheRec r0;
    memset(&r0, 0, sizeof(r0));
    r0.i_hi = r0.i_lo = -1;
    r0.iter = (int32_t)iter0;
    r0.done = kRunning;
    r0.b_hi = b_hi0;
    r0.b_lo = b_lo0;
    r0.hit_line[0] = r0.hit_line[1] = -1;
    for (int q = 0; q < kNQ; ++q) r0.line[q] = r0.key[q] = r0.old[q] = r0.hline[q] = r0.hold[q] = -1;
    HIP_CHECK(hipMemcpyAsync(m.rcf + 1, &r0, sizeof(r0), hipMemcpyHostToDevice, m.stream));
    uint64_t* p1 = m.pf + 2 * m.Gf;
    launch::smo_fused(m.args, 0, nullptr, p1, nullptr, nullptr, m.stream);
    if (m.collectives()) m.allreduce_keys(p1, 2 * m.Gf);
  }
  if (m.dense) {
    trace::Range gram_range("dpsvm/gram_gemm");
    // whole Gram shard K[i][j], i over all n rows, j over local rows: one MFMA GEMM
    gram_timer.start(m.stream);
    // one rank holds the whole (symmetric) Gram: compute half, mirror the rest
    const bool sym = m.off == 0 && m.nl == m.n && m.replicated;
    launch::rbf_gemm_store(m.x, m.xsq, m.n, m.dp, m.x + (size_t)m.off * m.dp, m.xsq + m.off, m.nl, m.dp,
                           m.dp, m.gamma, m.lines, m.ldl, m.stream, sym);
    gram_timer.stop(m.stream);
    res.rows_computed = m.n;
    res.x_passes = 1;
    // fused-iteration seed: record "no pending pair" in buffer 1 + initial keys
    FusedRec r0;
    r0.i_hi = r0.i_lo = -1;
    r0.a_hi = r0.a_lo = 0.f;
    r0.iter = (int32_t)iter0;
    r0.done = kRunning;
    r0.b_hi = b_hi0;
    r0.b_lo = b_lo0;
    HIP_CHECK(hipMemcpyAsync(m.rf + 1, &r0, sizeof(r0), hipMemcpyHostToDevice, m.stream));
    uint64_t* p1 = m.pf + 2 * m.Gf;
    launch::smo_fused(m.args, 0, nullptr, p1, m.rf + 1, nullptr, m.stream);
    if (m.collectives() && !m.xch) m.allreduce_keys(p1, 2 * m.Gf);
  }
  const bool graphs = m.p.use_graph && m.device_comm() && !m.p.sync_debug && !sync_debug_env();
  int B = std::max(1, m.p.graph_block);
  if (m.fused()) B = std::max(2, (B + 1) / 2 * 2);  // ping-pong parity must survive graph replays
  if (m.persist || m.persist_lru) B = std::max(1, m.p.persist_block);
  if (graphs && !m.persist && !m.persist_lru) {
    try {
      m.build_graph(B);
    } catch (const std::exception& e) {
      if (m.p.verbose) fprintf(stderr, "[dpsvm] graph capture failed (%s); eager launches\n", e.what());
    }
  }
  int64_t blocks = 0;
  const int64_t max_blocks = (m.p.max_iter - iter0) / B + 3;
  int64_t last_ck = iter0, last_log = iter0;
  SmoStatus st{};
  while (true) {
    if (m.persist) {
      launch::smo_persist(m.args, m.rf + 1, B, m.stream);
    } else if (m.persist_lru) {
      launch::smo_persist_lru(m.args, m.rf + 1, B, m.plru_stats, m.stream);
    } else if (m.gexec) {
      HIP_CHECK(hipGraphLaunch(m.gexec, m.stream));
    } else {
      for (int i = 0; i < B; ++i) m.enqueue_iteration(i);
    }
    HIP_CHECK(hipEventRecord(m.ev[blocks & 1], m.stream));
    if (blocks > 0) {
      m.wait_event(m.ev[(blocks - 1) & 1]);
      st = m.read_status();
      if (progress && m.p.log_every > 0 && st.iter / m.p.log_every != last_log / m.p.log_every) {
        last_log = st.iter;
        progress(Progress{st.iter, st.b_hi, st.b_lo, secs_since(t0), st.hits, st.misses});
      }
      if (st.done != kRunning) break;
      if (fault_iter >= 0 && !fault_done && st.iter >= fault_iter) {
        // DPSVM_FAULT=nan@K: poison f[0]; lands between two enqueued blocks
        static const float qnan = std::nanf("");
        HIP_CHECK(hipMemcpyAsync(m.f, &qnan, 4, hipMemcpyHostToDevice, m.stream));
        fault_done = true;
      }
      if (m.p.checkpoint_every > 0 && !m.p.checkpoint_path.empty() &&
          st.iter - last_ck >= m.p.checkpoint_every) {
        // drain the in-flight block, then snapshot (alpha replicated, f gathered)
        m.wait_event(m.ev[blocks & 1]);
        st = m.read_status();
        if (st.done == kRunning) {
          m.snapshot(st);
          last_ck = st.iter;
        }
      }
    }
    ++blocks;
    DPSVM_CHECK(blocks <= max_blocks + 2, "SMO loop did not terminate (internal error)");
  }
  m.wait_event(m.ev[blocks & 1]);  // the overshoot block (early-exit kernels)
  HIP_CHECK(hipStreamSynchronize(m.stream));
  res.t_solve = secs_since(t0);
  if (m.dense) res.t_gram = gram_timer.seconds();
  if (m.p.checkpoint_every > 0 && !m.p.checkpoint_path.empty()) {
    st = m.read_status();
    if (st.done == kMaxIter) m.snapshot(st);  // resumable continuation point
  }
  // ================= end of timed region =================

  if (trace::verify_enabled()) {
    // invariants: alpha in [0, C]; f consistent with alpha, i.e. the
    // incrementally updated f_j equals sum_i alpha_i y_i K(i, j) - y_j recomputed
    // from scratch (MFMA predict GEMM); float drift over 10^5 updates stays ~1e-5.
    std::vector<float> ah((size_t)m.n);
    HIP_CHECK(hipMemcpy(ah.data(), m.alpha, m.n * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < m.n; ++i)
      if (!(ah[i] >= 0.f && ah[i] <= m.p.C))
        fail("DPSVM_VERIFY: alpha[" + std::to_string(i) + "] = " + std::to_string(ah[i]) +
             " outside [0, C]");
    std::vector<float> fd((size_t)m.nl), fr((size_t)m.nl);
    HIP_CHECK(hipMemcpy(fd.data(), m.f, m.nl * 4, hipMemcpyDeviceToHost));
    size_t tb = 0;
    float* dref = dmalloc<float>((size_t)m.nl, &tb);
    local_decision(m, ah, dref);
    HIP_CHECK(hipMemcpy(fr.data(), dref, m.nl * 4, hipMemcpyDeviceToHost));
    (void)hipFree(dref);
    double err = 0.0;
    for (int64_t j = 0; j < m.nl; ++j) {
      const double ref = (double)fr[j] - m.h_y[m.off + j];
      const double e = std::fabs((double)fd[j] - ref) / (1.0 + std::fabs(ref));
      err = std::isfinite(e) ? std::max(err, e) : INFINITY;
    }
    res.verify_f_err = err;
    const char* te = std::getenv("DPSVM_VERIFY_FTOL");
    const double tol = te ? atof(te) : 1e-3;
    if (!(err <= tol))
      fail("DPSVM_VERIFY: f inconsistent with alpha (max relative error " + std::to_string(err) + ")");
  }
  if (m.collectives() && trace::verify_ranks_enabled()) {
    // cross-rank consistency: every rank must hold bit-identical alphas
    std::vector<float> ah((size_t)m.n);
    HIP_CHECK(hipMemcpy(ah.data(), m.alpha, m.n * 4, hipMemcpyDeviceToHost));
    const uint64_t h = trace::hash_floats(ah.data(), ah.size());
    uint64_t hk[2] = {h, ~h};
    if (m.comm->device_memory()) {
      size_t tb = 0;
      uint64_t* dk = dmalloc<uint64_t>(2, &tb);
      HIP_CHECK(hipMemcpy(dk, hk, 16, hipMemcpyHostToDevice));
      m.comm->allreduce_min_u64(dk, 2, m.stream);
      HIP_CHECK(hipMemcpyAsync(hk, dk, 16, hipMemcpyDeviceToHost, m.stream));
      HIP_CHECK(hipStreamSynchronize(m.stream));
      (void)hipFree(dk);
    } else {
      m.comm->allreduce_min_u64(hk, 2, nullptr);
    }
    if (hk[0] != h || ~hk[1] != h) fail("DPSVM_VERIFY: ranks hold different alphas (diverged)");
  }
  st = m.read_status();
  res.iters = st.iter;
  res.status = st.done;
  if (st.done == kCommFail)
    fail("peer exchange: a rank stopped publishing its selection keys (timeout after iteration " +
         std::to_string(st.iter) + ")");
  res.b_hi = st.b_hi;
  res.b_lo = st.b_lo;
  res.b = (st.b_lo + st.b_hi) / 2.0f;
  res.cache_hits = st.hits;
  res.cache_misses = st.misses;
  res.rows_computed += st.rows_computed;
  res.x_passes += st.x_passes;
  res.spec_rows = st.spec_rows;
  res.host_hits = st.host_hits;
  res.host_cache_lines = m.H;
  if (m.stamps) {
    std::vector<uint64_t> h((size_t)kStampRing * 2 * kStampSlots);
    HIP_CHECK(hipMemcpy(h.data(), m.stamps, h.size() * 8, hipMemcpyDeviceToHost));
    if (FILE* fp = fopen(m.stamps_path.c_str(), "wb")) {
      fwrite(h.data(), 8, h.size(), fp);
      fclose(fp);
    }
  }
  res.alpha.resize((size_t)m.n);
  HIP_CHECK(hipMemcpy(res.alpha.data(), m.alpha, m.n * 4, hipMemcpyDeviceToHost));
  return res;
}

// ---------------------------------------------------------------------------
// Distributed training accuracy: every rank compacts the SVs from the
// replicated alpha, predicts its own shard rows on MFMA, one sum all-reduce.
// Reference: rank 0 alone, n x (Sgemv + transform_reduce) (svmTrain.cu:633-665).
// ---------------------------------------------------------------------------
double GpuSolver::train_accuracy(const SolveResult& r) {
  auto& m = *impl_;
  HIP_CHECK(hipSetDevice(m.device));
  SvSet s;
  build_svs(m, r, s);
  size_t tb = 0;
  float* part = dmalloc<float>((size_t)launch::predict_scratch_floats(m.nl, s.nsv), &tb);
  int32_t* correct = dmalloc<int32_t>(1, &tb);
  HIP_CHECK(hipMemsetAsync(correct, 0, 4, m.stream));
  const int64_t lrow = m.off - m.args.x_row0;
  launch::rbf_predict(m.x + (size_t)lrow * m.dp, m.xsq + m.off, m.nl, m.dp, s.sv, s.svsq, s.coef, s.nsv,
                      m.dp, m.dp, m.gamma, r.b, part, nullptr, m.y + m.off, correct, m.stream);
  int32_t ok = 0;
  HIP_CHECK(hipMemcpyAsync(&ok, correct, 4, hipMemcpyDeviceToHost, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  (void)hipFree(part);
  (void)hipFree(correct);
  double tot = ok;
  if (m.world > 1) {
    if (m.comm->device_memory()) {
      double* dt = dmalloc<double>(1, &tb);
      HIP_CHECK(hipMemcpy(dt, &tot, 8, hipMemcpyHostToDevice));
      m.comm->allreduce_sum_f64(dt, 1, m.stream);
      HIP_CHECK(hipMemcpyAsync(&tot, dt, 8, hipMemcpyDeviceToHost, m.stream));
      HIP_CHECK(hipStreamSynchronize(m.stream));
      (void)hipFree(dt);
    } else {
      m.comm->allreduce_sum_f64(&tot, 1, nullptr);
    }
  }
  return tot / (double)m.n;
}

std::vector<float> GpuSolver::decision(const SolveResult& r, const float* xh, int64_t nt, int d) {
  auto& m = *impl_;
  DPSVM_CHECK(d == m.d, "feature count mismatch");
  HIP_CHECK(hipSetDevice(m.device));
  SvSet s;
  build_svs(m, r, s);
  std::vector<float> out((size_t)nt);
  const int64_t chunk = 1 << 20;
  size_t tb = 0;
  const int64_t cpad = round_up(std::min<int64_t>(nt, chunk), 128) + 128;
  float* dx = dmalloc<float>((size_t)cpad * m.dp, &tb);
  float* dsq = dmalloc<float>((size_t)cpad, &tb);
  float* ddec = dmalloc<float>((size_t)cpad, &tb);
  float* part = dmalloc<float>((size_t)launch::predict_scratch_floats(std::min<int64_t>(nt, chunk), s.nsv), &tb);
  for (int64_t r0 = 0; r0 < nt; r0 += chunk) {
    const int64_t rows = std::min(chunk, nt - r0);
    HIP_CHECK(hipMemsetAsync(dx, 0, (size_t)cpad * m.dp * 4, m.stream));
    HIP_CHECK(hipMemsetAsync(dsq, 0, cpad * 4, m.stream));
    HIP_CHECK(hipMemcpy2DAsync(dx, (size_t)m.dp * 4, xh + (size_t)r0 * d, (size_t)d * 4, (size_t)d * 4,
                               (size_t)rows, hipMemcpyHostToDevice, m.stream));
    launch::row_sqnorm(dx, rows, m.dp, m.dp, dsq, m.stream);
    launch::rbf_predict(dx, dsq, rows, m.dp, s.sv, s.svsq, s.coef, s.nsv, m.dp, m.dp, m.gamma, r.b, part,
                        ddec, nullptr, nullptr, m.stream);
    HIP_CHECK(hipMemcpyAsync(out.data() + r0, ddec, rows * 4, hipMemcpyDeviceToHost, m.stream));
  }
  HIP_CHECK(hipStreamSynchronize(m.stream));
  for (void* p : {(void*)dx, (void*)dsq, (void*)ddec, (void*)part}) (void)hipFree(p);
  return out;
}

// ---------------------------------------------------------------------------
// GpuPredictor (svmTest GPU path)
// ---------------------------------------------------------------------------
struct GpuPredictor::Impl {
  int device = 0;
  int d = 0, dp = 0;
  float gamma = 0.f, b = 0.f;
  int64_t nsv = 0;
  float *sv = nullptr, *svsq = nullptr, *coef = nullptr;
  hipStream_t stream = nullptr;
  ~Impl() {
    (void)hipSetDevice(device);
    for (void* p : {(void*)sv, (void*)svsq, (void*)coef}) if (p) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

GpuPredictor::GpuPredictor(const Model& mdl, int device) : impl_(new Impl) {
  auto& m = *impl_;
  m.device = device;
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking));
  m.d = std::max(1, mdl.d);
  m.dp = pad_features(m.d);
  m.gamma = mdl.gamma;
  m.b = mdl.b;
  m.nsv = mdl.nsv();
  const int64_t pad = round_up(std::max<int64_t>(m.nsv, 1), 128) + 128;
  size_t tb = 0;
  m.sv = dmalloc<float>((size_t)pad * m.dp, &tb);
  m.svsq = dmalloc<float>((size_t)pad, &tb);
  m.coef = dmalloc<float>((size_t)pad, &tb);
  HIP_CHECK(hipMemsetAsync(m.sv, 0, (size_t)pad * m.dp * 4, m.stream));
  HIP_CHECK(hipMemsetAsync(m.svsq, 0, pad * 4, m.stream));
  HIP_CHECK(hipMemsetAsync(m.coef, 0, pad * 4, m.stream));
  if (m.nsv) {
    HIP_CHECK(hipMemcpy2DAsync(m.sv, (size_t)m.dp * 4, mdl.x.data(), (size_t)mdl.d * 4, (size_t)mdl.d * 4,
                               (size_t)m.nsv, hipMemcpyHostToDevice, m.stream));
    std::vector<float> c((size_t)m.nsv);
    for (int64_t i = 0; i < m.nsv; ++i) c[i] = mdl.alpha[i] * mdl.y[i];
    HIP_CHECK(hipMemcpyAsync(m.coef, c.data(), m.nsv * 4, hipMemcpyHostToDevice, m.stream));
    launch::row_sqnorm(m.sv, m.nsv, m.dp, m.dp, m.svsq, m.stream);
  }
  HIP_CHECK(hipStreamSynchronize(m.stream));
}

GpuPredictor::~GpuPredictor() = default;

std::vector<float> GpuPredictor::decision(const float* xh, int64_t nt, int d) {
  auto& m = *impl_;
  DPSVM_CHECK(d == m.d || m.nsv == 0, "feature count mismatch between model and data");
  HIP_CHECK(hipSetDevice(m.device));
  std::vector<float> out((size_t)nt);
  if (nt == 0) return out;
  const int64_t chunk = 1 << 20;
  size_t tb = 0;
  const int64_t cpad = round_up(std::min<int64_t>(nt, chunk), 128) + 128;
  float* dx = dmalloc<float>((size_t)cpad * m.dp, &tb);
  float* dsq = dmalloc<float>((size_t)cpad, &tb);
  float* ddec = dmalloc<float>((size_t)cpad, &tb);
  float* part = dmalloc<float>((size_t)launch::predict_scratch_floats(std::min<int64_t>(nt, chunk), m.nsv), &tb);
  for (int64_t r0 = 0; r0 < nt; r0 += chunk) {
    const int64_t rows = std::min(chunk, nt - r0);
    HIP_CHECK(hipMemsetAsync(dx, 0, (size_t)cpad * m.dp * 4, m.stream));
    HIP_CHECK(hipMemcpy2DAsync(dx, (size_t)m.dp * 4, xh + (size_t)r0 * d, (size_t)d * 4, (size_t)d * 4,
                               (size_t)rows, hipMemcpyHostToDevice, m.stream));
    HIP_CHECK(hipMemsetAsync(dsq, 0, cpad * 4, m.stream));
    launch::row_sqnorm(dx, rows, m.dp, m.dp, dsq, m.stream);
    launch::rbf_predict(dx, dsq, rows, m.dp, m.sv, m.svsq, m.coef, m.nsv, m.dp, m.dp, m.gamma, m.b, part, ddec,
                        nullptr, nullptr, m.stream);
    HIP_CHECK(hipMemcpyAsync(out.data() + r0, ddec, rows * 4, hipMemcpyDeviceToHost, m.stream));
  }
  HIP_CHECK(hipStreamSynchronize(m.stream));
  for (void* p : {(void*)dx, (void*)dsq, (void*)ddec, (void*)part}) (void)hipFree(p);
  return out;
}

void GpuPredictor::decision_device(const float* x_dev, int64_t nt, int d, int ld, float* out_dev, void* stream) {
  auto& m = *impl_;
  DPSVM_CHECK(d == m.d, "feature count mismatch");
  DPSVM_CHECK(ld % 16 == 0 && ld >= m.dp, "decision_device: ld must be a multiple of 16 >= padded d");
  hipStream_t s = (hipStream_t)stream;
  size_t tb = 0;
  const int64_t pad = round_up(nt, 128) + 128;
  float* dsq = dmalloc<float>((size_t)pad, &tb);
  float* part = dmalloc<float>((size_t)launch::predict_scratch_floats(nt, m.nsv), &tb);
  HIP_CHECK(hipMemsetAsync(dsq, 0, pad * 4, s));
  launch::row_sqnorm(x_dev, nt, m.dp, ld, dsq, s);
  launch::rbf_predict(x_dev, dsq, nt, ld, m.sv, m.svsq, m.coef, m.nsv, m.dp, m.dp, m.gamma, m.b, part, out_dev,
                      nullptr, nullptr, s);
  HIP_CHECK(hipStreamSynchronize(s));
  (void)hipFree(dsq);
  (void)hipFree(part);
}

// ---------------------------------------------------------------------------
// kernel-level test entry points
// ---------------------------------------------------------------------------
namespace kernels {

void row_sqnorm(const float* x, int64_t n, int d, int ld, float* out, void* stream) {
  launch::row_sqnorm(x, n, d, ld, out, (hipStream_t)stream);
}

void rbf_rows(const float* x, const float* xsq, int64_t n, int ld, const float* w, const float* wsq, int nq,
              float gamma, float* out, int64_t out_ld, void* stream) {
  DPSVM_CHECK(nq >= 1 && nq <= kNQ, "rbf_rows: 1 <= nq <= 16");
  DPSVM_CHECK(ld % 16 == 0, "rbf_rows: ld must be a multiple of 16");
  hipStream_t s = (hipStream_t)stream;
  std::vector<float> hsq((size_t)nq);
  HIP_CHECK(hipMemcpyAsync(hsq.data(), wsq, nq * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  SmoCtrl c;
  memset(&c, 0, sizeof(c));
  c.nq = nq;
  c.n_compute = nq;  // all queries are kOpCompute (0) after the memset
  for (int q = 0; q < nq; ++q) {
    c.q_idx[q] = q;
    c.q_line[q] = q;
    c.q_sq[q] = hsq[q];
    c.q_ptr[q] = w + (size_t)q * ld;
  }
  size_t tb = 0;
  SmoCtrl* dc = dmalloc<SmoCtrl>(1, &tb);
  HIP_CHECK(hipMemcpyAsync(dc, &c, sizeof(c), hipMemcpyHostToDevice, s));
  SmoArgs a{};
  a.x = x;
  a.xsq = xsq;
  a.lines = out;
  a.ldl = out_ld;
  a.ctrl = dc;
  a.n = n;
  a.nl = n;
  a.off = 0;
  a.x_row0 = 0;
  a.dp = ld;
  a.d = ld;
  a.G = (int32_t)((n + kStepRows - 1) / kStepRows);
  a.gamma = gamma;
  launch::smo_rows(a, s);
  HIP_CHECK(hipStreamSynchronize(s));
  (void)hipFree(dc);
}

void select_partials(const float* f, const float* alpha, const float* y, int64_t n, int64_t offset, float C,
                     uint64_t* partials, int* blocks_out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  SmoCtrl c;
  memset(&c, 0, sizeof(c));
  c.line_hi = c.line_lo = -1;
  size_t tb = 0;
  SmoCtrl* dc = dmalloc<SmoCtrl>(1, &tb);
  HIP_CHECK(hipMemcpyAsync(dc, &c, sizeof(c), hipMemcpyHostToDevice, s));
  SmoArgs a{};
  a.f = const_cast<float*>(f);
  a.alpha = const_cast<float*>(alpha);
  a.y = y;
  a.ctrl = dc;
  a.partials = partials;
  a.nl = n;
  a.off = offset;
  a.C = C;
  a.G = (int32_t)((n + kStepRows - 1) / kStepRows);
  launch::smo_step(a, s);
  HIP_CHECK(hipStreamSynchronize(s));
  (void)hipFree(dc);
  if (blocks_out) *blocks_out = a.G;
}

void predict(const float* x, const float* xsq, int64_t n, int ld, const float* sv, const float* svsq,
             const float* coef, int64_t nsv, int sv_ld, float gamma, float b, float* dec, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  DPSVM_CHECK(ld == sv_ld && ld % 16 == 0, "predict: ld == sv_ld, multiple of 16");
  size_t tb = 0;
  float* part = dmalloc<float>((size_t)launch::predict_scratch_floats(n, nsv), &tb);
  launch::rbf_predict(x, xsq, n, ld, sv, svsq, coef, nsv, sv_ld, ld, gamma, b, part, dec, nullptr, nullptr, s);
  HIP_CHECK(hipStreamSynchronize(s));
  (void)hipFree(part);
}

void rbf_gram(const float* a, const float* asq, int64_t m, const float* b, const float* bsq, int64_t n, int ld,
              float gamma, float* out, int64_t out_ld, bool symmetric, void* stream) {
  launch::rbf_gemm_store(a, asq, m, ld, b, bsq, n, ld, ld, gamma, out, out_ld, (hipStream_t)stream, symmetric);
}

int64_t compact_nonzero(const float* alpha, int64_t n, int* idx_out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  size_t tb = 0;
  int32_t* cnt = dmalloc<int32_t>(1, &tb);
  int32_t* scratch = dmalloc<int32_t>((size_t)launch::compact_scratch_ints(n), &tb);
  launch::compact_positive(alpha, n, idx_out, cnt, scratch, s);
  int32_t h = 0;
  HIP_CHECK(hipMemcpyAsync(&h, cnt, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  (void)hipFree(cnt);
  (void)hipFree(scratch);
  return h;
}

}  // namespace kernels

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

std::string device_name(int dev) {
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, dev));
  std::string nm = p.name;
  while (!nm.empty() && nm.back() == ' ') nm.pop_back();
  return nm.empty() ? std::string(p.gcnArchName) : nm;
}

}  // namespace dpsvm
