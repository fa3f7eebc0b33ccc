// CPU modified-SMO solver: the no-GPU path (reference seq.cpp, C10) and the
// oracle the device solver is tested against.
//
// Same semantics as the reference MPI/GPU driver (svmTrainMain.cpp:235-310):
//   select  : b_hi = min_{I_up} f, b_lo = max_{I_low} f        (svmTrain.cu:41-95,400-483)
//   eta     : K(hi,hi)+K(lo,lo)-2K(hi,lo) from the explicit difference (svmTrain.cu:696-714)
//   update  : Catanzaro form + clip (svmTrainMain.cpp:285-299) -> common.hpp pair_update()
//   f update: f_j += dA_hi y_hi K(hi,j) + dA_lo y_lo K(lo,j)      (svmTrain.cu:98-137)
//   stop    : do { ... } while (b_lo > b_hi + 2 eps && ++iter < max_iter)
// Differences from the reference: deterministic lowest-index
// tie-break (Q15), eta floor (Q4), distance clamp at 0 (Q5), f32 indices never
// round-trip through float (Q2), kernel rows cached (seq.cpp recomputes every j).
//
// Sharding: X is replicated, f and cached kernel-row segments are per rank;
// the only collective per iteration is an element-wise MIN of two u64 keys.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <list>
#include <unordered_map>

#include "dpsvm/common.hpp"
#include "dpsvm/solver.hpp"
#include "../runtime/thread_pool.hpp"
#include <unistd.h>

#include "../runtime/timer.hpp"
#include "../runtime/trace.hpp"

namespace dpsvm {
namespace {

inline float dot_f32(const float* a, const float* b, int d) {
  // 4 partial sums (vectorisable); order fixed per row -> shard-invariant
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = 0;
  for (; k + 4 <= d; k += 4) {
    s0 += a[k] * b[k];
    s1 += a[k + 1] * b[k + 1];
    s2 += a[k + 2] * b[k + 2];
    s3 += a[k + 3] * b[k + 3];
  }
  for (; k < d; ++k) s0 += a[k] * b[k];
  return (s0 + s1) + (s2 + s3);
}

// LRU cache of kernel-row segments (local rows of one global row).
// Reference cache.cu:49-105 (std::map + std::list with O(L) lookup, Q11);
// here O(1) via unordered_map -> list iterator.
class RowCache {
 public:
  RowCache(int64_t lines, int64_t line_len) : cap_(std::max<int64_t>(2, lines)), len_(line_len) {}
  // returns {line pointer, hit}
  std::pair<float*, bool> get(int64_t key) {
    auto it = map_.find(key);
    if (it != map_.end()) {
      lru_.splice(lru_.begin(), lru_, it->second);
      return {it->second->data.data(), true};
    }
    if ((int64_t)map_.size() >= cap_) {
      auto& victim = lru_.back();
      map_.erase(victim.key);
      victim.key = key;
      lru_.splice(lru_.begin(), lru_, std::prev(lru_.end()));
    } else {
      lru_.push_front(Line{key, std::vector<float>((size_t)len_)});
    }
    map_[key] = lru_.begin();
    return {lru_.begin()->data.data(), false};
  }
  int64_t capacity() const { return cap_; }

 private:
  struct Line {
    int64_t key;
    std::vector<float> data;
  };
  int64_t cap_, len_;
  std::list<Line> lru_;
  std::unordered_map<int64_t, std::list<Line>::iterator> map_;
};

}  // namespace

SolveResult solve_cpu(const Dataset& ds, const SolverParams& p, Communicator* comm,
                      const Checkpoint* resume, const ProgressFn& progress) {
  auto t_setup0 = Clock::now();
  const int64_t n = ds.n;
  const int d = ds.d;
  DPSVM_CHECK(n >= 2 && d >= 1, "need at least 2 samples and 1 feature");
  DPSVM_CHECK(p.C > 0.f, "C must be > 0");
  const int rank = comm ? comm->rank() : 0;
  const int world = comm ? comm->size() : 1;
  DPSVM_CHECK(!comm || !comm->device_memory(), "CPU solver needs a host-memory communicator");
  const Shard sh = shard_of(n, rank, world);
  const int64_t nl = sh.size, off = sh.offset;
  const float gamma = resolve_gamma(p.gamma, d);
  const float C = p.C;
  const float* X = ds.x.data();
  const float* Y = ds.y.data();

  // flush-to-zero on every solver thread (restored for the caller on return):
  // adult-shape 48.5k iterations 199 s -> see profiles/r1_cpu_ftz.txt
  struct FpGuard {
    unsigned old;
    ~FpGuard() { set_fp_control(old); }
  } fp_guard{flush_denormals()};
  ThreadPool pool(default_threads(), /*ftz=*/true);

  // |x_i|^2 (reference: n separate thrust::inner_product launches, Q12)
  std::vector<float> xsq((size_t)n);
  pool.run(n, [&](int, int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) xsq[i] = dot_f32(X + (size_t)i * d, X + (size_t)i * d, d);
  }, 1024);

  std::vector<float> alpha((size_t)n, 0.f);
  std::vector<float> f((size_t)nl);
  for (int64_t j = 0; j < nl; ++j) f[j] = -Y[off + j];  // f = -y (svmTrain.cu:380)
  // f_j = sum_i alpha_i y_i K(i, j) - y_j from scratch (resume without f, DPSVM_VERIFY)
  auto recompute_f = [&](std::vector<float>& out) {
    pool.run(nl, [&](int, int64_t b, int64_t e) {
      for (int64_t j = b; j < e; ++j) {
        const float* xj = X + (size_t)(off + j) * d;
        float s = 0.f;
        for (int64_t i = 0; i < n; ++i) {
          if (alpha[i] == 0.f) continue;
          float d2 = xsq[i] + xsq[off + j] - 2.f * dot_f32(X + (size_t)i * d, xj, d);
          s += alpha[i] * Y[i] * std::exp(-gamma * std::max(d2, 0.f));
        }
        out[j] = s - Y[off + j];
      }
    }, 64);
  };
  int64_t iter0 = 0;
  float b_hi = 0.f, b_lo = 0.f;
  if (resume) {
    check_resume(*resume, n, d, p, gamma);
    alpha = resume->alpha;
    iter0 = resume->iter;
    b_hi = resume->b_hi;
    b_lo = resume->b_lo;
    if ((int64_t)resume->f.size() == n) {
      for (int64_t j = 0; j < nl; ++j) f[j] = resume->f[off + j];
    } else {
      recompute_f(f);
    }
  }

  // cache sizing: explicit lines / MiB, else up to a quarter of the machine's
  // RAM per process (all n rows when they fit: each kernel row computed once;
  // adult-shape needs 4.2 GB — with 1 GiB the LRU thrashed, ~2 misses/iteration)
  int64_t lines = p.cache_lines;
  if (lines <= 0) {
    double mb = p.cache_mb;
    if (mb <= 0) {
      const double phys = (double)sysconf(_SC_PHYS_PAGES) * (double)sysconf(_SC_PAGESIZE);
      mb = phys > 0 ? 0.25 * phys / (1024.0 * 1024.0) / std::max(1, world) : 1024.0;
    }
    lines = (int64_t)(mb * 1024.0 * 1024.0 / (4.0 * std::max<int64_t>(nl, 1)));
  }
  lines = std::max<int64_t>(2, std::min<int64_t>(lines, n));
  RowCache cache(lines, nl);

  SolveResult res;
  res.world = world;
  res.cache_lines = cache.capacity();
  res.t_setup = secs_since(t_setup0);

  auto compute_row = [&](int64_t gi, float* out) {
    const float* xi = X + (size_t)gi * d;
    const float si = xsq[gi];
    pool.run(nl, [&](int, int64_t b, int64_t e) {
      for (int64_t j = b; j < e; ++j) {
        float d2 = xsq[off + j] + si - 2.f * dot_f32(X + (size_t)(off + j) * d, xi, d);
        out[j] = std::exp(-gamma * std::max(d2, 0.f));
      }
    }, 512);
  };

  const int T = pool.size();
  std::vector<uint64_t> th_hi(T), th_lo(T);
  const int64_t fault_iter = trace::fault_nan_iter();
  const int64_t exit_iter = trace::fault_exit_iter(rank);
  const int64_t throw_iter = trace::fault_throw_iter(rank);
  trace::Range loop_range("dpsvm/smo_loop_cpu");
  auto t0 = Clock::now();
  int64_t iter = iter0;
  int status = 0;
  // per-thread selection keys of rows [b, e) (I-set classification + argmin /
  // argmax, svmTrain.cu:41-95), optionally after the f update of the same rows:
  // one pass and one pool dispatch per iteration
  auto select_rows = [&](int t, int64_t b, int64_t e) {
    uint64_t kh = kKeyNone, kl = kKeyNone;
    for (int64_t j = b; j < e; ++j) {
      const int64_t g = off + j;
      const float a = alpha[g], yj = Y[g], fj = f[j];
      if (in_up(a, yj, C)) kh = std::min(kh, make_key(fj, (uint32_t)g));
      if (in_low(a, yj, C)) kl = std::min(kl, make_key(-fj, (uint32_t)g));
    }
    th_hi[t] = kh;
    th_lo[t] = kl;
  };
  bool keys_ready = false;  // th_hi / th_lo hold this iteration's keys
  while (true) {
    // ---- local selection (unless the previous f update pass produced it) ----
    if (!keys_ready) {
      std::fill(th_hi.begin(), th_hi.end(), kKeyNone);
      std::fill(th_lo.begin(), th_lo.end(), kKeyNone);
      pool.run(nl, select_rows);
    }
    keys_ready = false;
    uint64_t keys[2] = {*std::min_element(th_hi.begin(), th_hi.end()),
                        *std::min_element(th_lo.begin(), th_lo.end())};
    if (world > 1) comm->allreduce_min_u64(keys, 2, nullptr);
    if (keys[0] == kKeyNone || keys[1] == kKeyNone) {
      status = 3;  // no violating pair can be formed
      break;
    }
    const int64_t i_hi = key_index(keys[0]), i_lo = key_index(keys[1]);
    b_hi = key_value(keys[0]);
    b_lo = -key_value(keys[1]);
    if (!std::isfinite(b_hi) || !std::isfinite(b_lo)) {
      status = 4;
      break;
    }
    // ---- eta from the explicit difference (reference host rbf_kernel) ----
    const float* xh = X + (size_t)i_hi * d;
    const float* xl = X + (size_t)i_lo * d;
    float dist2 = 0.f;
    for (int k = 0; k < d; ++k) {
      float t = xh[k] - xl[k];
      dist2 += t * t;
    }
    const float k_hl = std::exp(-gamma * dist2);
    const float a_hi_old = alpha[i_hi], a_lo_old = alpha[i_lo];
    PairUpdate u = pair_update(a_hi_old, a_lo_old, Y[i_hi], Y[i_lo], b_hi, b_lo, k_hl, C, p.tau,
                               (int)p.clip, i_hi == i_lo);
    alpha[i_lo] = u.a_lo_new;
    alpha[i_hi] = u.a_hi_new;  // hi written last: wins if i_hi == i_lo
    // ---- f update over local rows ----
    float* khi = nullptr;
    float* klo = nullptr;
    if (u.c_hi != 0.f) {
      auto [ptr, hit] = cache.get(i_hi);
      if (hit) ++res.cache_hits; else { ++res.cache_misses; ++res.rows_computed; compute_row(i_hi, ptr); }
      khi = ptr;
    }
    if (u.c_lo != 0.f) {
      auto [ptr, hit] = cache.get(i_lo);
      if (hit) ++res.cache_hits; else { ++res.cache_misses; ++res.rows_computed; compute_row(i_lo, ptr); }
      klo = ptr;  // capacity >= 2 and the hi line is MRU -> never the victim here
    }
    if (khi || klo) {
      // f update fused with the next iteration's selection over the same rows
      const float ch = u.c_hi, cl = u.c_lo;
      std::fill(th_hi.begin(), th_hi.end(), kKeyNone);
      std::fill(th_lo.begin(), th_lo.end(), kKeyNone);
      pool.run(nl, [&](int t, int64_t b, int64_t e) {
        for (int64_t j = b; j < e; ++j) {
          float delta;
          if (khi && klo) delta = (ch * khi[j]) + (cl * klo[j]);
          else if (khi) delta = ch * khi[j];
          else delta = cl * klo[j];
          f[j] += delta;
        }
        select_rows(t, b, e);
      });
      keys_ready = true;
    }
    ++iter;
    if (exit_iter >= 0 && iter >= exit_iter) {  // DPSVM_FAULT=exit@K:R: this rank's process dies
      fprintf(stderr, "[dpsvm] fault injection: rank %d exits at iteration %lld\n", rank, (long long)iter);
      fflush(stderr);
      _exit(3);
    }
    if (throw_iter >= 0 && iter >= throw_iter)  // DPSVM_FAULT=throw@K:R: this rank's solve fails
      fail("fault injection: rank " + std::to_string(rank) + " throws at iteration " + std::to_string(iter));
    if (fault_iter >= 0 && iter == fault_iter && nl > 0) {  // DPSVM_FAULT
      f[0] = std::nanf("");
      keys_ready = false;
    }
    const bool open = gap_open(b_hi, b_lo, p.eps);
    if (progress && p.log_every > 0 && iter % p.log_every == 0)
      progress(Progress{iter, b_hi, b_lo, secs_since(t0), res.cache_hits, res.cache_misses});
    if (!open) { status = 1; break; }
    const bool ck_on = p.checkpoint_every > 0 && !p.checkpoint_path.empty();
    if (ck_on && (iter % p.checkpoint_every == 0 || iter >= p.max_iter)) {
      Checkpoint ck;
      ck.n = n; ck.d = d; ck.C = C; ck.gamma = gamma; ck.eps = p.eps; ck.clip = (int)p.clip;
      ck.iter = iter; ck.b_hi = b_hi; ck.b_lo = b_lo; ck.alpha = alpha;
      if (world == 1) {
        ck.f = f;
        write_checkpoint(p.checkpoint_path, ck);
      } else {
        // gather f shards: sum of zero-padded copies (exact: one contributor per slot)
        std::vector<double> fg((size_t)n, 0.0);
        for (int64_t j = 0; j < nl; ++j) fg[off + j] = f[j];
        comm->allreduce_sum_f64(fg.data(), (size_t)n, nullptr);
        ck.f.assign(fg.begin(), fg.end());
        if (rank == 0) write_checkpoint(p.checkpoint_path, ck);
      }
    }
    if (iter >= p.max_iter) { status = 2; break; }
  }
  res.t_solve = secs_since(t0);
  if (trace::verify_enabled()) {
    // invariants: alpha in [0, C]; incremental f == f recomputed from alpha
    for (int64_t i = 0; i < n; ++i)
      if (!(alpha[i] >= 0.f && alpha[i] <= C))
        fail("DPSVM_VERIFY: alpha[" + std::to_string(i) + "] outside [0, C]");
    std::vector<float> fr((size_t)nl);
    recompute_f(fr);
    double err = 0.0;
    for (int64_t j = 0; j < nl; ++j) {
      const double e = std::fabs((double)f[j] - fr[j]) / (1.0 + std::fabs((double)fr[j]));
      err = std::isfinite(e) ? std::max(err, e) : INFINITY;
    }
    res.verify_f_err = err;
    const char* te = std::getenv("DPSVM_VERIFY_FTOL");
    if (!(err <= (te ? atof(te) : 1e-3)))
      fail("DPSVM_VERIFY: f inconsistent with alpha (max relative error " + std::to_string(err) + ")");
  }
  if (world > 1 && (p.verify_ranks || trace::verify_enabled())) {
    // cross-rank consistency: every rank must hold bit-identical alphas
    const uint64_t h = trace::hash_floats(alpha.data(), alpha.size());
    uint64_t hk[2] = {h, ~h};
    comm->allreduce_min_u64(hk, 2, nullptr);
    if (hk[0] != h || ~hk[1] != h) fail("DPSVM_VERIFY: ranks hold different alphas (diverged)");
  }
  res.iters = iter;
  res.status = status;
  res.b_hi = b_hi;
  res.b_lo = b_lo;
  res.b = (b_lo + b_hi) / 2.0f;  // svmTrainMain.cpp:329
  res.alpha = std::move(alpha);
  return res;
}

// ---------------------------------------------------------------------------
// CPU predictor (reference seq_test.cpp:187-210 ignores b; here b is applied as
// in the GPU accuracy path svmTrain.cu:646-658).
// ---------------------------------------------------------------------------
std::vector<float> decision_cpu(const Model& m, const float* x, int64_t n, int d, int threads) {
  DPSVM_CHECK(d == m.d || m.nsv() == 0, "feature count mismatch between model and data");
  std::vector<float> svsq((size_t)m.nsv());
  for (int64_t s = 0; s < m.nsv(); ++s) svsq[s] = dot_f32(&m.x[(size_t)s * d], &m.x[(size_t)s * d], d);
  std::vector<float> coef((size_t)m.nsv());
  for (int64_t s = 0; s < m.nsv(); ++s) coef[s] = m.alpha[s] * m.y[s];
  std::vector<float> dec((size_t)n);
  parallel_for(n, threads, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      const float* xi = x + (size_t)i * d;
      const float si = dot_f32(xi, xi, d);
      double acc = 0.0;
      for (int64_t s = 0; s < m.nsv(); ++s) {
        float d2 = svsq[s] + si - 2.f * dot_f32(&m.x[(size_t)s * d], xi, d);
        acc += (double)coef[s] * std::exp(-m.gamma * std::max(d2, 0.f));
      }
      dec[i] = (float)acc - m.b;
    }
  });
  return dec;
}

double accuracy_from_decision(const std::vector<float>& dec, const float* y, int64_t n) {
  if (n <= 0) return 0.0;
  int64_t ok = 0;
  for (int64_t i = 0; i < n; ++i) {
    float pred = dec[i] < 0.f ? -1.f : 1.f;
    ok += (pred == (y[i] > 0 ? 1.f : -1.f));
  }
  return (double)ok / (double)n;
}

}  // namespace dpsvm
