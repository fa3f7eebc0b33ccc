// The iteration engines of the device solver.  Each one seeds the device
// state at the start of the timed region and then advances the SMO in blocks
// of iterations that never return to the host (the host polls a pinned status
// record one block behind).
//
//   persistent-dense  Gram resident; ONE launch runs persist_block iterations,
//                     keys exchanged in-kernel (smo_persist.hip)
//   fused-dense       Gram resident; one launch per iteration, blocks of launches
//                     replayed from a hipGraph (smo_fused.hip)
//   (persistent-cache, fused-cache and chain — the quarantined pair-at-a-time
//   cache / partitioned-X engines — live in the plugin gpu_engines_pairq.hip)
//   ws-dense          Gram resident; working-set rounds: one workgroup solves a
//                     q-row sub-problem from an LDS sub-Gram, one grid pass
//                     updates f and selects the next candidates (ws_*.hip)
//   ws-cache          kernel-row cache; working-set rounds whose missing rows
//                     come from one MFMA GEMM per round
//
// Reference per-iteration path: svmTrainMain.cpp:235-310 (host loop, >= 7
// blocking host<->device round trips, one MPI Allgather).
#include <hip/hip_runtime.h>

#include <atomic>

#include "gpu_impl.hpp"
#include "../runtime/timer.hpp"
#include "../runtime/trace.hpp"

namespace dpsvm {

// one SMO iteration of a launch-per-iteration engine on `stream` (no host
// synchronisation for device communicators).  Fused engines: iteration k of
// a block reads partial buffer / record k^1 and writes k&1.
void GpuSolver::Impl::enqueue_iteration(int k) {
  if (kind == EngineKind::FusedDense) {
    const int wi = k & 1, ri = wi ^ 1;
    launch::smo_fused(args, 1, pf + (size_t)ri * 2 * Gf, pf + (size_t)wi * 2 * Gf, rf + ri, rf + wi, stream);
    if (collectives() && !xch) allreduce_keys(pf + (size_t)wi * 2 * Gf, 2 * Gf);
    return;
  }
  // fused-cache / chain: the quarantined pair-at-a-time engines (plugin)
  gpu::need_quarantine("the fused-cache / chain iteration").enqueue_iteration(*this, k);
}

void GpuSolver::Impl::build_graph(int iters) {
  if (gexec) return;
  HIP_CHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
  try {
    for (int i = 0; i < iters; ++i) enqueue_iteration(i);
  } catch (...) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(stream, &g);
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    throw;
  }
  HIP_CHECK(hipStreamEndCapture(stream, &graph));
  HIP_CHECK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
}

namespace gpu {
namespace {

// The split GEMMs' fp16 operands of every x row this rank holds (part of the
// Gram / first-round work, so inside the timed region of every solve).
void split_x(GpuSolver::Impl& m) {
  if (m.gram_split) launch::split_rows_f16(m.x, m.x_rows, m.dp, m.dp, m.xs, m.xsh, m.stream);
}

// Dense engines: the whole Gram shard K[i][j] (i over all n rows, j over the
// local rows) by one MFMA GEMM inside the timed region.
struct DenseBase : Engine {
  EventTimer gram_timer;
  void gram(GpuSolver::Impl& m, SolveResult& res) {
    trace::Range gram_range("dpsvm/gram_gemm");
    gram_timer.start(m.stream);
    split_x(m);
    if (!m.replicated) {
      gram_panels(m);
    } else if (m.gram_split) {
      const bool sym = m.off == 0 && m.nl == m.n;
      const size_t ru = (size_t)launch::split_row_u4(m.dp) * 16;
      launch::rbf_gemm_store_split(m.xs, m.xsh, m.xsq, m.n, (const uint8_t*)m.xs + (size_t)m.off * ru, m.xsh + m.off,
                                   m.xsq + m.off, m.nl, m.dp, m.gamma, m.lines, m.ldl, m.stream, sym,
                                   m.gram_cold_tau);
    } else {
      // one rank holds the whole (symmetric) Gram: compute half, mirror the rest
      const bool sym = m.off == 0 && m.nl == m.n;
      launch::rbf_gemm_store(m.x, m.xsq, m.n, m.dp, m.x + (size_t)m.off * m.dp, m.xsq + m.off, m.nl, m.dp, m.dp,
                             m.gamma, m.lines, m.ldl, m.stream, sym);
    }
    gram_timer.stop(m.stream);
    res.rows_computed = m.n;
    res.x_passes = 1;
  }
  // Partitioned X (ws-dense only: no later step reads a non-owned X row): the
  // Gram block K(all rows, owned columns) panel by panel — rank r's shard is
  // broadcast into a panel buffer and multiplied against the owned rows.  Every
  // element is the same MFMA k-sequence as in the replicated launch
  // (bit-identical Gram).  One panel of X lives at a time.
  static void gram_panels(GpuSolver::Impl& m) {
    const int64_t prow = round_up(m.ldl, 128) + 512;
    size_t tb = 0;
    float* panel = dmalloc<float>((size_t)prow * m.dp, &tb);
    const size_t ru = (size_t)launch::split_row_u4(m.dp) * 16;
    void* pxs = m.gram_split ? (void*)dmalloc<uint8_t>((size_t)prow * ru, &tb) : nullptr;
    int32_t* pxsh = m.gram_split ? dmalloc<int32_t>((size_t)prow, &tb) : nullptr;
    HIP_CHECK(hipMemsetAsync(panel, 0, (size_t)prow * m.dp * 4, m.stream));
    std::vector<float> host;
    for (int r = 0; r < m.world; ++r) {
      const Shard s = shard_of(m.n, r, m.world);
      const size_t bytes = (size_t)s.size * m.dp * 4;
      if (r == m.rank) HIP_CHECK(hipMemcpyAsync(panel, m.x, bytes, hipMemcpyDeviceToDevice, m.stream));
      if (m.world > 1 && bytes > 0) {
        if (m.comm->device_memory()) {
          m.comm->broadcast(panel, bytes, r, m.stream);
        } else {
          host.resize(bytes / 4);
          HIP_CHECK(hipMemcpyAsync(host.data(), panel, bytes, hipMemcpyDeviceToHost, m.stream));
          HIP_CHECK(hipStreamSynchronize(m.stream));
          m.comm->broadcast(host.data(), bytes, r, nullptr);
          HIP_CHECK(hipMemcpyAsync(panel, host.data(), bytes, hipMemcpyHostToDevice, m.stream));
        }
      }
      if (m.gram_split) {
        launch::split_rows_f16(panel, prow, m.dp, m.dp, pxs, pxsh, m.stream);
        launch::rbf_gemm_store_split(pxs, pxsh, m.xsq + s.offset, s.size, m.xs, m.xsh, m.xsq + m.off, m.nl, m.dp,
                                     m.gamma, m.lines + (size_t)s.offset * m.ldl, m.ldl, m.stream, false,
                                     m.gram_cold_tau);
      } else {
        launch::rbf_gemm_store(panel, m.xsq + s.offset, s.size, m.dp, m.x, m.xsq + m.off, m.nl, m.dp, m.dp, m.gamma,
                               m.lines + (size_t)s.offset * m.ldl, m.ldl, m.stream, false);
      }
    }
    if (m.world > 1 && m.comm->device_memory()) sync_collective(m.comm, m.stream, "Gram panel broadcast");
    else HIP_CHECK(hipStreamSynchronize(m.stream));
    (void)hipFree(panel);
    if (pxs) (void)hipFree(pxs);
    if (pxsh) (void)hipFree(pxsh);
  }
  // record "no pending pair" in buffer 1 + the initial keys (published to the
  // exchange when there is one, else all-reduced when collectives run)
  void seed_keys(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo) {
    const FusedRec r0 = seed_record(iter0, b_hi, b_lo);
    HIP_CHECK(hipMemcpyAsync(m.rf + 1, &r0, sizeof(r0), hipMemcpyHostToDevice, m.stream));
    uint64_t* p1 = m.pf + 2 * m.Gf;
    launch::smo_fused(m.args, 0, nullptr, p1, m.rf + 1, nullptr, m.stream);
    if (m.collectives() && !m.xch) m.allreduce_keys(p1, 2 * m.Gf);
  }
  void seed(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo, SolveResult& res) override {
    gram(m, res);
    seed_keys(m, iter0, b_hi, b_lo);
  }
  double gram_seconds() override { return gram_timer.seconds(); }
  Pending pending(GpuSolver::Impl& m) override {
    // blocks have even length: the last kernel wrote record 1 (the persistent
    // engine leaves "no pending pair" there)
    FusedRec r;
    HIP_CHECK(hipMemcpy(&r, m.rf + 1, sizeof(r), hipMemcpyDeviceToHost));
    return pending_of(r);
  }
};

struct PersistDense final : DenseBase {
  EngineKind kind() const override { return EngineKind::PersistDense; }
  int block(const SolverParams& p) const override { return std::max(1, p.persist_block); }
  void run_block(GpuSolver::Impl& m, int B) override { launch::smo_persist(m.args, m.rf + 1, B, m.stream); }
};

struct FusedDense final : DenseBase {
  EngineKind kind() const override { return EngineKind::FusedDense; }
  int block(const SolverParams& p) const override { return even_block(p); }
  void seed(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo, SolveResult& res) override {
    DenseBase::seed(m, iter0, b_hi, b_lo, res);
    maybe_graph(m, block(m.p));
  }
  void run_block(GpuSolver::Impl& m, int B) override { run_launches(m, B); }
};

// Per-round collectives of the working-set engines at world > 1 (or forced at
// world 1, which tests the RCCL + graph-capture path on one GPU; every rank
// runs the merge and the sub-problem redundantly on identical inputs):
// all-gather of the candidate lists, and one sum all-reduce that assembles the
// sub-Gram (+ the members' f) from the columns each rank owns.  Device
// communicators (RCCL) enqueue on the stream and are captured in the round
// graph; host communicators stage through host memory.
void ws_allgather_cand(GpuSolver::Impl& m) {
  if (!m.collectives() || m.wsa.xpeer) return;  // peer exchange: pushed by ws_select itself
  const size_t bytes = (size_t)m.wsa.G * 2 * kWsCand * sizeof(uint64_t);
  if (m.comm->device_memory()) {
    m.comm->allgather(m.wsa.cand_out, m.wsa.cand, bytes, m.stream);  // in place: cand_out = cand + rank * bytes
    return;
  }
  m.h_wscand.resize(bytes * m.world);
  uint8_t* mine = m.h_wscand.data() + (size_t)m.rank * bytes;
  HIP_CHECK(hipMemcpyAsync(mine, m.wsa.cand_out, bytes, hipMemcpyDeviceToHost, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  m.comm->allgather(mine, m.h_wscand.data(), bytes, nullptr);
  HIP_CHECK(hipMemcpyAsync(m.wsa.cand, m.h_wscand.data(), bytes * m.world, hipMemcpyHostToDevice, m.stream));
}

// multi-block rounds at world > 1: every rank's line-search partials
void ws_allgather_part(GpuSolver::Impl& m) {
  if (!m.collectives() || m.wsa.xpeer) return;  // peer exchange: pushed by pass 1, polled by pass 2
  const size_t bytes = (size_t)m.wsa.p1G * std::max(1, m.wsa.ks) * 2 * sizeof(double);
  uint8_t* all = (uint8_t*)m.wsa.part;
  if (m.comm->device_memory()) {
    m.comm->allgather(all + (size_t)m.rank * bytes, all, bytes, m.stream);
    return;
  }
  m.h_wspart.resize(bytes * m.world);
  uint8_t* mine = m.h_wspart.data() + (size_t)m.rank * bytes;
  HIP_CHECK(hipMemcpyAsync(mine, all + (size_t)m.rank * bytes, bytes, hipMemcpyDeviceToHost, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  m.comm->allgather(mine, m.h_wspart.data(), bytes, nullptr);
  HIP_CHECK(hipMemcpyAsync(all, m.h_wspart.data(), bytes * m.world, hipMemcpyHostToDevice, m.stream));
}

void ws_allreduce_sub(GpuSolver::Impl& m, const WsArgs& w) {
  if (!m.collectives() || w.xpeer) return;  // peer exchange: assembled by the gather kernel
  // the P sub-Grams + the members' f of every block ([3][P][kWsMax] aux: f first)
  const size_t count = (size_t)w.blocks * ((size_t)w.q_max * w.q_max + kWsMax);
  if (m.comm->device_memory()) {
    m.comm->allreduce_sum_f32(m.wssub, count, m.stream);
    return;
  }
  m.h_wssub.resize(count);
  HIP_CHECK(hipMemcpyAsync(m.h_wssub.data(), m.wssub, count * 4, hipMemcpyDeviceToHost, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  m.comm->allreduce_sum_f32(m.h_wssub.data(), count, nullptr);
  HIP_CHECK(hipMemcpyAsync(m.wssub, m.h_wssub.data(), count * 4, hipMemcpyHostToDevice, m.stream));
}

// partitioned X, cache mode: the packed miss rows (owner's row, zeros elsewhere)
void ws_allreduce_rows(GpuSolver::Impl& m, int64_t rows) {
  if (!m.collectives()) return;
  const size_t count = (size_t)rows * m.dp;
  if (m.comm->device_memory()) {
    m.comm->allreduce_sum_f32(m.wsxq, count, m.stream);
    return;
  }
  m.h_wsxq.resize(count);
  HIP_CHECK(hipMemcpyAsync(m.h_wsxq.data(), m.wsxq, count * 4, hipMemcpyDeviceToHost, m.stream));
  HIP_CHECK(hipStreamSynchronize(m.stream));
  m.comm->allreduce_sum_f32(m.h_wsxq.data(), count, nullptr);
  HIP_CHECK(hipMemcpyAsync(m.wsxq, m.h_wsxq.data(), count * 4, hipMemcpyHostToDevice, m.stream));
}

bool ws_graphs(GpuSolver::Impl& m) {
  // host communicators stage through host memory: no graph, unless the rounds
  // need no collective at all (peer exchange)
  return m.p.use_graph && (m.device_comm() || !m.ws_round_collectives()) && !m.p.sync_debug && !sync_debug_env();
}

// B rounds captured into one hipGraph (`round` enqueues one round on m.stream)
template <class Fn>
void capture_rounds(GpuSolver::Impl& m, int B, hipGraph_t* graph, hipGraphExec_t* exec, Fn round) {
  HIP_CHECK(hipStreamBeginCapture(m.stream, hipStreamCaptureModeRelaxed));
  try {
    for (int i = 0; i < B; ++i) round();
  } catch (...) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(m.stream, &g);
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    throw;
  }
  HIP_CHECK(hipStreamEndCapture(m.stream, graph));
  HIP_CHECK(hipGraphInstantiate(exec, *graph, nullptr, nullptr, 0));
}

// Working-set rounds (ws_*.hip) on the resident Gram (ws-dense) or on a
// kernel-row cache (ws-cache: the Gram does not fit HBM).  A round is
//   [merge (+ cache mode: line assignment, one MFMA GEMM for the set's missing
//   rows)] -> gather (sub-Gram rows) -> solve (LDS sub-problem) -> select (f
//   update + next candidates)
// and a block is B rounds (one hipGraph), so f is consistent with alpha at
// every block boundary (checkpoints need no pending pair) and the host polls
// the status one block behind like the SMO engines.  Seed: (ws-dense) the Gram
// GEMM, the control record (no working set yet) and the first candidates.
//
// Multi-block rounds (wsa.blocks = P > 1) are adaptive: the device halves the
// block count after every damped round (strongly coupled blocks) and drops to
// one after an independent-clip event; once it is 1, the host switches to the
// one-block round kernels (cheaper merge, one f-update pass) at the first block
// boundary whose completed rounds include the one that set it — a value every
// rank reads identically, so every rank switches at the same round.
template <class Base, bool kCache>
struct WsRounds : Base {
  bool single = false;  // multi-block engine now running one-block rounds
  int64_t prev_launched = 0;  // `launched` at the previous observe() (the switch boundary test)
  int block(const SolverParams& p) const override { return std::max(1, p.ws_block); }
  // the one-block view of a multi-block engine's buffers: sub-Gram at the start
  // of wssub, its f / alpha / y right after it (one contiguous sum all-reduce)
  static WsArgs one_block(const GpuSolver::Impl& m) {
    WsArgs w = m.wsa;
    w.blocks = 1;
    w.q_max = m.ws_q1;  // ws_size rows (the multi-block rounds may use smaller blocks)
    w.inner_max = m.p.ws_inner > 0 ? m.p.ws_inner : 4 * w.q_max;
    w.aux = m.wssub + (size_t)w.q_max * w.q_max;
    w.aux_stride = kWsMax;
    w.xsub_rows = w.q_max;  // peer exchange: the one-block layout of the sub-Gram rows (same region)
    // the one-block engine's set turnover (multi-block rounds replace the
    // whole union): ws_new_auto (device_state.hpp)
    w.n_new = ws_new_auto(m.p.ws_new, w.q_max, m.dp);
    w.direct_sub = 0;  // the one-block rounds merge inside ws_gather
    return w;
  }
  // cache mode: the kernel rows of the round's misses (<= blocks x q_max rows), one GEMM
  static void miss_rows(GpuSolver::Impl& m, const WsArgs& w) {
    const int64_t mmax = (int64_t)w.blocks * w.q_max;
    const float* B = m.x + (size_t)(m.off - m.args.x_row0) * m.dp;  // the owned rows
    if (m.gram_split) {
      const size_t ru = (size_t)launch::split_row_u4(m.dp) * 16;
      const void* Bs = (const uint8_t*)m.xs + (size_t)(m.off - m.args.x_row0) * ru;
      const int32_t* Bsh = m.xsh + (m.off - m.args.x_row0);
      if (m.replicated) {
        launch::rbf_rows_indexed_split(m.xs, m.xsh, m.xsq, m.wsctrl_miss_row(), m.wsctrl_n_miss(), mmax, Bs, Bsh,
                                       m.xsq + m.off, m.nl, m.dp, m.gamma, m.lines, m.wsctrl_miss_line(), m.ldl,
                                       m.stream);
      } else {
        launch::ws_pack_rows(m.x, m.off, m.nl, m.dp, m.xsq, m.wsctrl, (int)mmax, m.wsxq, m.wsxqsq, m.stream);
        ws_allreduce_rows(m, mmax);
        launch::split_rows_f16(m.wsxq, mmax, m.dp, m.dp, m.wsxs, m.wsxsh, m.stream);
        launch::rbf_rows_indexed_split(m.wsxs, m.wsxsh, m.wsxqsq, m.wsiota, m.wsctrl_n_miss(), mmax, Bs, Bsh,
                                       m.xsq + m.off, m.nl, m.dp, m.gamma, m.lines, m.wsctrl_miss_line(), m.ldl,
                                       m.stream);
      }
      return;
    }
    if (m.replicated) {
      launch::rbf_rows_indexed(m.x, m.xsq, m.wsctrl_miss_row(), m.wsctrl_n_miss(), mmax, B, m.xsq + m.off, m.nl,
                               m.dp, m.gamma, m.lines, m.wsctrl_miss_line(), m.ldl, m.stream);
    } else {
      launch::ws_pack_rows(m.x, m.off, m.nl, m.dp, m.xsq, m.wsctrl, (int)mmax, m.wsxq, m.wsxqsq, m.stream);
      ws_allreduce_rows(m, mmax);
      launch::rbf_rows_indexed(m.wsxq, m.wsxqsq, m.wsiota, m.wsctrl_n_miss(), mmax, B, m.xsq + m.off, m.nl, m.dp,
                               m.gamma, m.lines, m.wsctrl_miss_line(), m.ldl, m.stream);
    }
  }
  static void round(GpuSolver::Impl& m, const WsArgs& w) {
    if (kCache && m.ws_recompute && w.blocks == 1) {
      // no row cache: merge + sub-Gram from the split X rows, the solve, then
      // the selection pass with the changed rows' kernel rows recomputed inside
      // the f update (ws_recompute.hip)
      launch::ws_subgram_split(w, m.xs, m.xsh, m.xsq, m.dp, m.gamma, m.stream);
      launch::ws_solve(w, m.stream);
      launch::ws_fupdate_split(w, m.xs, m.xsh, m.xsq, m.dp, m.gamma, m.stream);
      return;
    }
    // peer exchange: the candidate lists every rank pushed at the end of the
    // previous round (or the seed), collected in-kernel by a few workgroups (the
    // merge then reads them as from the all-gather and never spins)
    if (w.xpeer) launch::ws_xcollect_cand(w, m.stream);
    if (w.blocks > 1) launch::ws_merge_multi(w, m.stream);
    else if (kCache) launch::ws_merge(w, m.stream);  // ws-dense one-block rounds merge inside ws_gather
    if (kCache) miss_rows(m, w);
    if (!w.direct_sub) launch::ws_gather(w, m.stream);  // else ws_solve loads its block itself
    ws_allreduce_sub(m, w);
    launch::ws_solve(w, m.stream);
    if (w.blocks > 1) {
      launch::ws_select_pass(w, 1, m.stream);
      if (w.xpeer) launch::ws_xcollect_part(w, m.stream);  // peer exchange: the partials pass 1 pushed
      else ws_allgather_part(m);
      launch::ws_select_pass(w, 2, m.stream);
    } else {
      launch::ws_select(w, m.stream);
    }
    ws_allgather_cand(m);
  }
  void seed_rounds(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo) {
    single = false;
    prev_launched = 0;
    if (m.wsa.blocks > 1) HIP_CHECK(hipMemsetAsync(m.wsa.dalpha, 0, (size_t)m.n * 4, m.stream));
    WsCtrl c;
    memset(&c, 0, sizeof(c));
    c.iter = iter0;
    c.done = kRunning;
    c.b_hi = b_hi;
    c.b_lo = b_lo;
    c.p_act = c.p_round = m.wsa.blocks;
    HIP_CHECK(hipMemcpyAsync(m.wsctrl, &c, sizeof(c), hipMemcpyHostToDevice, m.stream));
    launch::ws_select(m.wsa, m.stream);
    ws_allgather_cand(m);
    if (ws_graphs(m) && !m.gexec) capture_rounds(m, this->block(m.p), &m.graph, &m.gexec, [&] { round(m, m.wsa); });
  }
  bool shortens() const override { return true; }
  void observe(GpuSolver::Impl& m, const SmoStatus& st, int64_t launched) override {
    if (single || m.wsa.blocks <= 1 || st.ws_p1_round <= 0) return;
    // the switch to the one-block graph happens on kWsSwitchRounds boundaries
    // only, with what the host knew one such span earlier — the rounds the
    // 32-round graph blocks switched at, whatever the graph block size (short
    // blocks end a solve sooner after convergence without moving a trajectory)
    const int64_t B = this->block(m.p), next = launched;  // first round after the launch in flight
    const int64_t span = std::max<int64_t>(B, kWsSwitchRounds);
    // the last span boundary at or before `next`; it must lie inside the launch
    // in flight (a short tail's single-round launches can leave `launched` off
    // the boundaries: a modulo test would then never switch)
    const int64_t prev = prev_launched;
    prev_launched = next;
    const int64_t bnd = next / span * span;
    if (bnd <= prev) return;
    if (st.ws_p1_round > bnd - span) return;  // set by a later round: next boundary
    single = true;
    const WsArgs w = one_block(m);
    launch::ws_to_single(w, m.stream);
    if (ws_graphs(m) && !m.gexec1) capture_rounds(m, this->block(m.p), &m.graph1, &m.gexec1, [&] { round(m, w); });
  }
  void run_block(GpuSolver::Impl& m, int B) override {
    hipGraphExec_t g = single ? m.gexec1 : m.gexec;
    if (g && B == this->block(m.p)) {  // a shorter launch (rounds before a predicted convergence): plain launches
      HIP_CHECK(hipGraphLaunch(g, m.stream));
    } else {
      const WsArgs w = single ? one_block(m) : m.wsa;
      for (int i = 0; i < B; ++i) round(m, w);
    }
  }
  Pending pending(GpuSolver::Impl&) override { return {}; }  // alphas committed every round
};

struct WsDense final : WsRounds<DenseBase, false> {
  EngineKind kind() const override { return EngineKind::WsDense; }
  void seed(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo, SolveResult& res) override {
    gram(m, res);
    seed_rounds(m, iter0, b_hi, b_lo);
  }
};

// ws-cache: the X pass of a round computes all of its set's missing rows in one
// GEMM (up to blocks x q_max rows) instead of 2 (+16 speculative) rows per SMO
// iteration in the pair-at-a-time cache engines.
struct WsCache final : WsRounds<Engine, true> {
  EngineKind kind() const override { return EngineKind::WsCache; }
  void seed(GpuSolver::Impl& m, int64_t iter0, float b_hi, float b_lo, SolveResult&) override {
    split_x(m);
    seed_rounds(m, iter0, b_hi, b_lo);
  }
};

}  // namespace

std::unique_ptr<Engine> make_engine(EngineKind k) {
  switch (k) {
    case EngineKind::PersistDense: return std::make_unique<PersistDense>();
    case EngineKind::FusedDense: return std::make_unique<FusedDense>();
    case EngineKind::WsDense: return std::make_unique<WsDense>();
    case EngineKind::WsCache: return std::make_unique<WsCache>();
    default: return need_quarantine("the pair-at-a-time cache / chain engines").make_engine(k);
  }
}

namespace {
std::atomic<const QuarantineOps*> g_quarantine{nullptr};
}

void register_quarantine(const QuarantineOps* ops) { g_quarantine.store(ops); }

const QuarantineOps* quarantine() { return g_quarantine.load(); }

}  // namespace gpu

bool quarantine_loaded() { return gpu::quarantine() != nullptr; }

namespace gpu {

const QuarantineOps& need_quarantine(const char* what) {
  const QuarantineOps* q = g_quarantine.load();
  DPSVM_CHECK(q != nullptr, std::string(what) + " live in the quarantined pair-cache plugin, which is not loaded "
                                                "(engines=\"all\": dpsvm_amd._native.load_quarantine(), or the CLIs)");
  return *q;
}

}  // namespace gpu
}  // namespace dpsvm
