// The timed SMO loop of the device solver (reference: svmTrainMain.cpp:206-314),
// checkpoints, fault injection and invariant checks (§5.2-5.3).
#include <hip/hip_runtime.h>

#include <cmath>

#include <unistd.h>

#include "gpu_impl.hpp"
#include "../runtime/timer.hpp"
#include "../runtime/trace.hpp"

namespace dpsvm {

using gpu::dmalloc;

void gpu_local_decision(GpuSolver::Impl& m, const std::vector<float>& alpha, float* out_dev);  // gpu_predict.hip

// Checkpoint snapshot (stream drained by the caller): alpha is replicated,
// the f shards are all-gathered; rank 0 writes.
void GpuSolver::Impl::snapshot(const SmoStatus& st) {
  Checkpoint ck;
  ck.n = n;
  ck.d = d;
  ck.C = p.C;
  ck.gamma = gamma;
  ck.eps = p.eps;
  ck.clip = (int)p.clip;
  ck.iter = st.iter;
  ck.b_hi = st.b_hi;
  ck.b_lo = st.b_lo;
  ck.alpha.resize((size_t)n);
  HIP_CHECK(hipMemcpy(ck.alpha.data(), alpha, n * 4, hipMemcpyDeviceToHost));
  // the latest pair's alphas may still be pending in the last kernel's record
  // (exact; the host-mapped status refreshes only every kStatusEvery)
  const gpu::Pending q = engine->pending(*this);
  if (q.valid) {
    ck.iter = q.iter;
    ck.b_hi = q.b_hi;
    ck.b_lo = q.b_lo;
    if (q.i_hi >= 0) {
      ck.alpha[q.i_lo] = q.a_lo;
      ck.alpha[q.i_hi] = q.a_hi;
    }
  }
  ck.f = gather_f();
  // replicated solve: every rank holds everything, the caller's rank 0 writes
  if (rank == 0 && outer_rank == 0) write_checkpoint(p.checkpoint_path, ck);
}

// every rank: the whole gradient (the solve's f shards all-gathered)
std::vector<float> GpuSolver::Impl::gather_f() {
  std::vector<float> floc((size_t)ldl, 0.f), fall((size_t)ldl * world);
  HIP_CHECK(hipMemcpy(floc.data(), f, nl * 4, hipMemcpyDeviceToHost));
  if (world > 1) {
    if (comm->device_memory()) {
      size_t tb = 0;
      float* gb = dmalloc<float>((size_t)ldl * world, &tb);
      HIP_CHECK(hipMemcpy(gb + (size_t)rank * ldl, f, ldl * 4, hipMemcpyDeviceToDevice));
      comm->allgather(gb + (size_t)rank * ldl, gb, ldl * 4, stream);
      HIP_CHECK(hipMemcpyAsync(fall.data(), gb, fall.size() * 4, hipMemcpyDeviceToHost, stream));
      sync_collective(comm, stream, "gradient all-gather");
      (void)hipFree(gb);
    } else {
      comm->allgather(floc.data(), fall.data(), ldl * 4, nullptr);
    }
  } else {
    fall = floc;
  }
  std::vector<float> out((size_t)n, 0.f);
  for (int r = 0; r < world; ++r) {
    Shard s = shard_of(n, r, world);
    std::copy(fall.begin() + (size_t)r * ldl, fall.begin() + (size_t)r * ldl + s.size, out.begin() + s.offset);
  }
  return out;
}

std::vector<float> GpuSolver::gradient_all() {
  HIP_CHECK(hipSetDevice(impl_->device));
  return impl_->gather_f();
}

SolveResult GpuSolver::solve(const Checkpoint* resume, const ProgressFn& progress) {
  auto& m = *impl_;
  HIP_CHECK(hipSetDevice(m.device));
  SolveResult res;
  res.world = m.world;
  res.cache_lines = m.L;
  auto ts0 = Clock::now();

  if (!m.lines) {  // released (release_cache): the same L lines again, empty
    m.lines = gpu::dmalloc<float>((size_t)m.L * m.ldl, &m.bytes);
    m.info.bytes_device = m.bytes;
    m.args.lines = m.lines;
    m.wsa.gram = m.lines;
  }
  // ---- state init (alpha = 0, f = -y, empty cache) or resume ----
  int64_t iter0 = 0;
  float b_hi0 = 0.f, b_lo0 = 0.f;
  HIP_CHECK(hipMemsetAsync(m.alpha, 0, m.n * 4, m.stream));
  if (resume) {
    check_resume(*resume, m.n, m.d, m.p, m.gamma);
    HIP_CHECK(hipMemcpyAsync(m.alpha, resume->alpha.data(), m.n * 4, hipMemcpyHostToDevice, m.stream));
    iter0 = resume->iter;
    b_hi0 = resume->b_hi;
    b_lo0 = resume->b_lo;
  }
  if (resume && (int64_t)resume->f.size() == m.n) {
    HIP_CHECK(hipMemcpyAsync(m.f, resume->f.data() + m.off, m.nl * 4, hipMemcpyHostToDevice, m.stream));
  } else if (resume) {
    // f_j = sum_i alpha_i y_i K(i, j) - y_j via the predict GEMM (b = 0)
    gpu_local_decision(m, resume->alpha, m.f);
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
  }
  m.engine->prepare(m);
  m.init_ctrl(iter0, b_hi0, b_lo0);
  if (m.xch) HIP_CHECK(hipMemsetAsync(m.xbuf, 0, (size_t)m.xregion * 8, m.stream));  // tags restart at iter0 + 1
  HIP_CHECK(hipStreamSynchronize(m.stream));
  if (m.world > 1) m.comm->barrier();
  res.t_setup = secs_since(ts0);

  // ================= timed region: the SMO loop (svmTrainMain.cpp:206-314) =================
  trace::Range loop_range("dpsvm/solve");
  const int64_t fault_iter = trace::fault_nan_iter();
  const int64_t exit_iter = trace::fault_exit_iter(m.outer_rank);
  const int64_t throw_iter = trace::fault_throw_iter(m.outer_rank);
  bool fault_done = false;
  auto t0 = Clock::now();
  m.engine->seed(m, iter0, b_hi0, b_lo0, res);
  const int B = m.engine->block(m.p);
  int64_t blocks = 0;
  const int64_t max_blocks = (m.p.max_iter - iter0) / B + 3;
  int64_t last_ck = iter0, last_log = iter0;
  SmoStatus st{};
  // watchdog at world > 1: the first blocks (the seed's Gram GEMM, graph
  // instantiation) get kWatchdogFirstS; later ones 50x the
  // slowest block seen, at least kWatchdogFloorS — a peer that died mid-solve
  // (a collective that never completes) fails this rank within seconds
  // (only when the user left watchdog_s at 0 = auto: an explicit bound is used as given)
  constexpr double kWatchdogFirstS = 120.0, kWatchdogFloorS = 20.0;
  struct WdReset {  // wd_limit must not outlive this solve (exceptions included)
    double& v;
    ~WdReset() { v = 0.0; }
  } wd_reset{m.wd_limit};
  auto t_prev = Clock::now();
  double blk_max = 0.0;
  int n_timed = 0;
  // one-at-a-time rounds near convergence (engines that take short launches):
  // the host reads each launch's status one launch behind, so a converged
  // round leaves the launch in flight to exit at once — ~12 such rounds
  // (~25 us each) with 8-round graphs on the headline.  When the gap of the
  // last completed launch times its per-launch decay predicts the stop test
  // to pass within the launch in flight, the following launches are single
  // rounds.  The status is identical on every rank, so is the decision.
  static const bool tail_env = [] {  // A/B: DPSVM_SHORT_TAIL=0 keeps full launches to the end
    const char* e = std::getenv("DPSVM_SHORT_TAIL");
    return !(e && atoi(e) == 0);
  }();
  const bool can_short = tail_env && m.engine->shortens() && B > 1;
  bool near = false;
  int near_left = 0;
  double prev_gap = -1.0;
  int64_t launched = 0;
  while (true) {
    const int Bk = near ? 1 : B;
    m.engine->run_block(m, Bk);
    launched += Bk;
    HIP_CHECK(hipEventRecord(m.ev[blocks & 1], m.stream));
    if (blocks > 0) {
      if (m.world > 1 && !(m.p.watchdog_s > 0.0))
        m.wd_limit = n_timed >= 2 ? std::min(kWatchdogDefaultS, std::max(kWatchdogFloorS, 50.0 * blk_max))
                                  : kWatchdogFirstS;
      m.wait_event(m.ev[(blocks - 1) & 1]);
      {
        const auto now = Clock::now();
        const double dt = std::chrono::duration<double>(now - t_prev).count();
        t_prev = now;
        if (blocks >= 2) {  // block 0's completion includes the seed
          blk_max = std::max(blk_max, dt);
          ++n_timed;
        }
      }
      st = m.read_status();
      if (progress && m.p.log_every > 0 && st.iter / m.p.log_every != last_log / m.p.log_every) {
        last_log = st.iter;
        progress(Progress{st.iter, st.b_hi, st.b_lo, secs_since(t0), st.hits, st.misses});
      }
      if (st.done != kRunning) break;
      if (can_short) {
        // on when the gap times its last decay is within 2 x the stop gap
        // (2 eps), for at most kShortRun single-round launches — a noisy drop on
        // a slowly converging problem costs that many, not the rest of the
        // solve in single rounds — then re-armed by the same test
        // a multiple of the launch size, so launches stay on the engines' span boundaries
        const int kShortRun = (32 + B - 1) / B * B;
        const double gap = (double)st.b_lo - (double)st.b_hi, eps = (double)m.p.eps;
        if (near_left > 0) {
          --near_left;
        } else if (prev_gap > 0.0 && gap > 0.0 && gap < prev_gap && gap * (gap / prev_gap) <= 4.0 * eps) {
          near_left = kShortRun;
        }
        near = near_left > 0;
        prev_gap = gap;
      }
      m.engine->observe(m, st, launched);  // launches 0 .. blocks - 1 completed, launch `blocks` in flight
      if (exit_iter >= 0 && st.iter >= exit_iter) {
        // DPSVM_FAULT=exit@K:R: this rank's process dies mid-solve
        fprintf(stderr, "[dpsvm] fault injection: rank %d exits at iteration %lld\n", m.outer_rank,
                (long long)st.iter);
        fflush(stderr);
        _exit(3);
      }
      if (throw_iter >= 0 && st.iter >= throw_iter) {
        // DPSVM_FAULT=throw@K:R: this rank's solve fails, its thread lives on;
        // drain its own stream first (nothing of this rank stays in flight)
        (void)hipStreamSynchronize(m.stream);
        fail("fault injection: rank " + std::to_string(m.outer_rank) + " throws at iteration " +
             std::to_string(st.iter));
      }
      if (fault_iter >= 0 && !fault_done && st.iter >= fault_iter) {
        // DPSVM_FAULT=nan@K: poison f[0]; lands between two enqueued blocks
        static const float qnan = std::nanf("");
        HIP_CHECK(hipMemcpyAsync(m.f, &qnan, 4, hipMemcpyHostToDevice, m.stream));
        fault_done = true;
      }
      if (m.p.checkpoint_every > 0 && !m.p.checkpoint_path.empty() && st.iter - last_ck >= m.p.checkpoint_every) {
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
    DPSVM_CHECK(launched <= (max_blocks + 2) * (int64_t)B, "SMO loop did not terminate (internal error)");
  }
  m.wait_event(m.ev[blocks & 1]);  // the overshoot block (early-exit kernels)
  HIP_CHECK(hipStreamSynchronize(m.stream));
  res.t_solve = secs_since(t0);
  res.t_gram = m.engine->gram_seconds();
  if (m.gram_cold_tau > 0.f) launch::gram_adapt_last(&res.gram_tiles, &res.gram_hot_tiles);
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
        fail("DPSVM_VERIFY: alpha[" + std::to_string(i) + "] = " + std::to_string(ah[i]) + " outside [0, C]");
    std::vector<float> fd((size_t)m.nl), fr((size_t)m.nl);
    HIP_CHECK(hipMemcpy(fd.data(), m.f, m.nl * 4, hipMemcpyDeviceToHost));
    size_t tb = 0;
    float* dref = dmalloc<float>((size_t)m.nl, &tb);
    gpu_local_decision(m, ah, dref);
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
    if (!(err <= tol)) fail("DPSVM_VERIFY: f inconsistent with alpha (max relative error " + std::to_string(err) + ")");
  }
  if ((m.outer_world > 1 || m.p.force_collectives) && (m.p.verify_ranks || trace::verify_enabled())) {
    // cross-rank consistency (on by default at world > 1): every rank must hold
    // bit-identical alphas; one 16-byte all-reduce per solve
    std::vector<float> ah((size_t)m.n);
    HIP_CHECK(hipMemcpy(ah.data(), m.alpha, m.n * 4, hipMemcpyDeviceToHost));
    const uint64_t h = trace::hash_floats(ah.data(), ah.size());
    uint64_t hk[2] = {h, ~h};
    Communicator* c = m.outer;
    if (c->device_memory()) {
      size_t tb = 0;
      uint64_t* dk = dmalloc<uint64_t>(2, &tb);
      HIP_CHECK(hipMemcpy(dk, hk, 16, hipMemcpyHostToDevice));
      c->allreduce_min_u64(dk, 2, m.stream);
      HIP_CHECK(hipMemcpyAsync(hk, dk, 16, hipMemcpyDeviceToHost, m.stream));
      sync_collective(c, m.stream, "alpha digest all-reduce");
      (void)hipFree(dk);
    } else {
      c->allreduce_min_u64(hk, 2, nullptr);
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
  res.outer = st.outer;
  if (m.working_set() && m.wsa.blocks > 1) {
    res.ws_blocks = m.wsa.blocks;
    res.ws_blocks_end = st.ws_p;
    res.ws_p1_round = st.ws_p1_round;
    res.ws_damped = st.ws_damped;
  }
  res.world = m.outer_world;
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

}  // namespace dpsvm
