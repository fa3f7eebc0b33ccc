// QUARANTINED engines: the pair-at-a-time SMO engines for a kernel-row cache
// (Gram not resident) or a partitioned X.  Not part of the production module
// (dpsvm_amd/_C): they are built into the plugin dpsvm_amd/_pairq*.so (and
// linked into the CLIs), which registers QuarantineOps (gpu_impl.hpp) when it
// is loaded — engines="all" / svmTrain --engines all: tests and A/B probes.
//
//   persistent-cache  one launch per persist_block iterations, private cache
//                     metadata per workgroup (kernels/smo_persist_lru.hip)
//   fused-cache       one launch per iteration incl. the CLOCK plan, the X pass
//                     and the pinned-host spill tier (kernels/smo_fused_lru.hip;
//                     SURVEY §5.7 — measured 4-25x slower than recomputing a row,
//                     profiles/r3_spill_vs_recompute_1gpu.json)
//   chain             rows / step / [collective] / finalize per iteration
//                     (kernels/smo_kernels.hip): the partitioned-X pair engine
//
// Why quarantined: with 288 GB per GPU the Gram of every problem the pair
// engines win on (< 50k rows) is resident, and the working-set engines are
// 5-10x faster where it is not (docs/DESIGN.md §2).  They stay the reference's
// exact trajectory (bit-identical to the dense pair engines, tested) for a Gram
// that does not fit.  Reference: cache.cu:49-105 (LRU row cache), svmTrain.cu:
// 190-302 (rows + f update), svmTrainMain.cpp:235-310 (the iteration).
#include <hip/hip_runtime.h>

#include <cstring>

#include "gpu_impl.hpp"

namespace dpsvm {
namespace gpu {
namespace {

// one iteration of the fused-cache or chain engine (the production module
// handles fused-dense itself).  Fused: iteration k of a block reads partial
// buffer / record k^1 and writes k&1.
void enqueue_pairq(GpuSolver::Impl& m, int k) {
  if (m.kind == EngineKind::FusedCache) {
    const int wi = k & 1, ri = wi ^ 1;
    uint64_t* pout = m.pf + (size_t)wi * 2 * m.Gf;
    launch::smo_fused_lru(m.args, m.pf + (size_t)ri * 2 * m.Gf, pout, m.rcf + ri, m.rcf + wi, m.stream);
    if (m.collectives() && !m.xch) m.allreduce_keys(pout, 2 * m.Gf);
    return;
  }
  DPSVM_CHECK(m.kind == EngineKind::Chain, "pair-cache plugin: not a plugin engine");
  launch::smo_rows(m.args, m.stream);
  launch::smo_step(m.args, m.stream);
  if (m.collectives()) {
    if (m.replicated) {
      m.allreduce_keys(m.partials, 2 * m.G);
    } else {
      launch::smo_local_record(m.args, m.stream);
      const size_t rb = (size_t)m.args.rec_bytes;
      if (m.comm->device_memory()) {
        m.comm->allgather(m.my_record, m.records, rb, m.stream);
      } else {
        HIP_CHECK(hipMemcpyAsync(m.h_records.data() + m.rank * rb, m.my_record, rb, hipMemcpyDeviceToHost, m.stream));
        HIP_CHECK(hipStreamSynchronize(m.stream));
        m.comm->allgather(m.h_records.data() + m.rank * rb, m.h_records.data(), rb, nullptr);
        HIP_CHECK(hipMemcpyAsync(m.records, m.h_records.data(), rb * m.world, hipMemcpyHostToDevice, m.stream));
      }
    }
  } else if (!m.replicated) {
    // single-rank partitioned (tests): the local record is the whole world
    launch::smo_local_record(m.args, m.stream);
    HIP_CHECK(hipMemcpyAsync(m.records, m.my_record, m.args.rec_bytes, hipMemcpyDeviceToDevice, m.stream));
  }
  launch::smo_finalize(m.args, m.stream);
}

struct PersistCache final : Engine {
  EngineKind kind() const override { return EngineKind::PersistCache; }
  int block(const SolverParams& p) const override { return std::max(1, p.persist_block); }
  void prepare(GpuSolver::Impl& m) override {  // every workgroup's private copy: empty cache, hand 0
    launch::plru_init(m.plru_meta, m.args.plru_stride, m.Gf, m.n, m.L, m.stream);
    HIP_CHECK(hipMemsetAsync(m.plru_stats, 0, 8 * sizeof(int64_t), m.stream));
  }
  void seed(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo, SolveResult&) override {
    const FusedRec r0 = seed_record(iter0, b_hi, b_lo);
    HIP_CHECK(hipMemcpyAsync(m.rf + 1, &r0, sizeof(r0), hipMemcpyHostToDevice, m.stream));
    launch::smo_fused(m.args, 0, nullptr, m.pf + 2 * m.Gf, m.rf + 1, nullptr, m.stream);
  }
  void run_block(GpuSolver::Impl& m, int B) override {
    launch::smo_persist_lru(m.args, m.rf + 1, B, m.plru_stats, m.stream);
  }
  Pending pending(GpuSolver::Impl& m) override {
    FusedRec r;
    HIP_CHECK(hipMemcpy(&r, m.rf + 1, sizeof(r), hipMemcpyDeviceToHost));
    return pending_of(r);
  }
};

struct FusedCache final : Engine {
  EngineKind kind() const override { return EngineKind::FusedCache; }
  int block(const SolverParams& p) const override { return even_block(p); }
  void seed(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo, SolveResult&) override {
    // record "no pending pair, empty cache" in buffer 1 + initial keys
    FusedCacheRec r0;
    memset(&r0, 0, sizeof(r0));
    r0.i_hi = r0.i_lo = -1;
    r0.iter = (int32_t)iter0;
    r0.done = kRunning;
    r0.b_hi = b_hi;
    r0.b_lo = b_lo;
    r0.hit_line[0] = r0.hit_line[1] = -1;
    for (int q = 0; q < kNQ; ++q) r0.line[q] = r0.key[q] = r0.old[q] = r0.hline[q] = r0.hold[q] = -1;
    HIP_CHECK(hipMemcpyAsync(m.rcf + 1, &r0, sizeof(r0), hipMemcpyHostToDevice, m.stream));
    uint64_t* p1 = m.pf + 2 * m.Gf;
    launch::smo_fused(m.args, 0, nullptr, p1, nullptr, nullptr, m.stream);
    if (m.collectives()) m.allreduce_keys(p1, 2 * m.Gf);
    maybe_graph(m, block(m.p));
  }
  void run_block(GpuSolver::Impl& m, int B) override { run_launches(m, B); }
  Pending pending(GpuSolver::Impl& m) override {
    FusedCacheRec r;
    HIP_CHECK(hipMemcpy(&r, m.rcf + 1, sizeof(r), hipMemcpyDeviceToHost));
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
};

struct Chain final : Engine {
  EngineKind kind() const override { return EngineKind::Chain; }
  int block(const SolverParams& p) const override { return std::max(1, p.graph_block); }
  void seed(GpuSolver::Impl& m, int64_t, float, float, SolveResult&) override { maybe_graph(m, block(m.p)); }
  void run_block(GpuSolver::Impl& m, int B) override { run_launches(m, B); }
};

std::unique_ptr<Engine> make_pairq(EngineKind k) {
  switch (k) {
    case EngineKind::PersistCache: return std::make_unique<PersistCache>();
    case EngineKind::FusedCache: return std::make_unique<FusedCache>();
    case EngineKind::Chain: return std::make_unique<Chain>();
    default: fail("pair-cache plugin: not a plugin engine");
  }
  return nullptr;
}

const QuarantineOps kOps = {
    make_pairq,
    enqueue_pairq,
    launch::smo_fused_lru_supported,
    launch::smo_persist_lru_supported,
    launch::plru_stride_words,
    launch::smo_persist_lru_blocks_per_cu,
    launch::smo_persist_lru_census,
    launch::preload_persist_lru_kernel,
    launch::smo_rows,
    launch::smo_step,
    launch::xpass_rows,
};

// registration when the plugin is loaded (dlopen) or linked (CLIs)
struct Register {
  Register() { register_quarantine(&kOps); }
} g_register;

}  // namespace
}  // namespace gpu
}  // namespace dpsvm
