// Native unit tests (run by tests/test_native_unit.py; `--gpu` adds the
// device-side cases).  The reference had no tests at all.
#include <cmath>
#include <cstdio>
#include <functional>
#include <iostream>
#include <thread>
#include <unistd.h>

#include "dpsvm/comm.hpp"
#include "dpsvm/common.hpp"
#include "dpsvm/io.hpp"
#include "dpsvm/solver.hpp"

using namespace dpsvm;

static int g_fail = 0, g_pass = 0;
#define EXPECT(cond)                                                        \
  do {                                                                      \
    if (!(cond)) {                                                          \
      ++g_fail;                                                             \
      fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);     \
    } else {                                                                \
      ++g_pass;                                                             \
    }                                                                       \
  } while (0)

static void test_keys() {
  // ordering of f with lowest-index tie-break
  float vals[] = {-3.5f, -1.f, -0.f, 0.f, 1e-30f, 2.f, 1e9f, -1e9f};
  for (float a : vals)
    for (float b : vals) {
      uint64_t ka = make_key(a, 7), kb = make_key(b, 3);
      if (a < b) EXPECT(ka < kb);
      if (a > b) EXPECT(ka > kb);
      if (a == b) EXPECT(kb < ka);  // same value -> lower index wins
      EXPECT(key_value(ka) == a);
      EXPECT(key_index(ka) == 7u);
    }
}

static void test_shards() {
  for (int64_t n : {1, 2, 10, 60000, 60001})
    for (int w : {1, 2, 3, 7, 8, 10}) {
      int64_t tot = 0, prev_end = 0, mx = 0, mn = n + 1;
      for (int r = 0; r < w; ++r) {
        Shard s = shard_of(n, r, w);
        EXPECT(s.offset == prev_end);
        prev_end = s.offset + s.size;
        tot += s.size;
        mx = std::max(mx, s.size);
        mn = std::min(mn, s.size);
      }
      EXPECT(tot == n);
      EXPECT(mx - mn <= 1);
    }
}

static void test_geometry() {
  // headline (60k rows): 512 rows x 118 workgroups on 1 GPU, 15 per rank on 8
  {
    const Geometry g1 = make_geometry(60000, dense_rows_min(60000, 1));
    EXPECT(g1.rows == 512 && g1.groups == 118);
    const int64_t nl8 = (60000 + 7) / 8;
    const Geometry g8 = make_geometry(nl8, dense_rows_min(nl8, 8));
    EXPECT(g8.rows == 512 && g8.groups == 15);
  }
  for (int64_t n : {2, 1000, 60000, 200000, 581012, 786432, 2000000})
    for (int w : {1, 2, 4, 8}) {
      const int64_t nl = (n + w - 1) / w;
      const Geometry d = make_geometry(nl, dense_rows_min(nl, w));
      EXPECT(d.rows % 256 == 0 && d.rows * d.groups >= nl);
      if (nl <= 256 * 3072) {  // the persistent dense engine's range
        EXPECT(d.groups <= 256);
        EXPECT(d.rows <= 3072);
        if (nl * w <= 256 * 3072) EXPECT(w * d.groups <= 256);  // one poll batch
      }
      const Geometry c = make_geometry(nl, 0);  // cache mode: ~one workgroup per CU
      EXPECT(c.rows % 256 == 0 && c.rows * c.groups >= nl && c.groups <= 256);
    }
}

static void test_io() {
  char tmpl[] = "/tmp/dpsvm_unitXXXXXX";
  char* dir = mkdtemp(tmpl);
  EXPECT(dir != nullptr);
  std::string base = dir;
  Dataset ds = make_synthetic(Synth::Blobs, 257, 5, 3);
  write_csv(base + "/a.csv", ds);
  Dataset rd = read_csv(base + "/a.csv", 0, 0);
  EXPECT(rd.n == 257 && rd.d == 5);
  bool same = true;
  for (size_t i = 0; i < ds.x.size(); ++i) same &= ds.x[i] == rd.x[i];
  for (size_t i = 0; i < ds.y.size(); ++i) same &= ds.y[i] == rd.y[i];
  EXPECT(same);
  Dataset part = read_csv_rows(base + "/a.csv", 100, 50, 5);
  EXPECT(part.n == 50 && part.x[0] == ds.x[100 * 5] && part.y[49] == ds.y[149]);
  // model round trip (both formats)
  std::vector<float> alpha(ds.n, 0.f);
  for (int64_t i = 0; i < ds.n; i += 3) alpha[i] = 0.5f + i;
  Model m = make_model(ds, alpha, -0.25f, 0.7f);
  write_model(base + "/m.txt", m);
  Model r = read_model(base + "/m.txt");
  EXPECT(r.has_b && r.b == -0.25f && r.gamma == 0.7f && r.nsv() == m.nsv() && r.d == 5);
  EXPECT(r.x == m.x && r.alpha == m.alpha && r.y == m.y);
  write_model(base + "/l.txt", m, 9, true);
  Model l = read_model(base + "/l.txt");
  EXPECT(!l.has_b && l.b == 0.f && l.nsv() == m.nsv() && l.x == m.x);
  // checkpoint round trip
  Checkpoint ck;
  ck.n = ds.n; ck.d = 5; ck.C = 2; ck.gamma = 0.5f; ck.eps = 1e-3f; ck.iter = 17;
  ck.b_hi = -1; ck.b_lo = 1; ck.alpha = alpha; ck.f = alpha;
  write_checkpoint(base + "/c.ck", ck);
  Checkpoint c2 = read_checkpoint(base + "/c.ck");
  EXPECT(c2.n == ck.n && c2.iter == 17 && c2.alpha == ck.alpha && c2.f == ck.f && c2.C == 2.f);
  // libsvm
  FILE* fp = fopen((base + "/s.txt").c_str(), "w");
  fprintf(fp, "+1 1:1 3:1\n-1 2:0.5 4:1\n");
  fclose(fp);
  Dataset sv = read_libsvm(base + "/s.txt", 4);
  EXPECT(sv.n == 2 && sv.x[0] == 1.f && sv.x[2] == 1.f && sv.x[5] == 0.5f && sv.x[7] == 1.f && sv.y[1] == -1.f);
  std::string cmd = "rm -rf " + base;
  EXPECT(system(cmd.c_str()) == 0);
}

static SolverParams small_params() {
  SolverParams p;
  p.C = 2.f;
  p.gamma = 0.5f;
  p.eps = 1e-3f;
  p.max_iter = 100000;
  return p;
}

static void test_cpu_solver_ranks() {
  Dataset ds = make_synthetic(Synth::Blobs, 600, 4, 11, 0, -1, 1.5f);
  SolverParams p = small_params();
  SolveResult r1 = solve_cpu(ds, p);
  EXPECT(r1.status == 1);
  EXPECT(r1.iters > 10);
  // KKT sanity: alphas within the box
  bool box = true;
  for (float a : r1.alpha) box &= (a >= 0.f && a <= p.C);
  EXPECT(box);
  for (int world : {2, 3}) {
    ThreadCommGroup g(world);
    std::vector<SolveResult> rs(world);
    std::vector<std::thread> ts;
    for (int r = 0; r < world; ++r)
      ts.emplace_back([&, r] {
        auto c = g.comm(r);
        rs[r] = solve_cpu(ds, p, c.get());
      });
    for (auto& t : ts) t.join();
    // identical decisions on every rank and identical to one rank
    for (int r = 0; r < world; ++r) {
      EXPECT(rs[r].iters == r1.iters);
      EXPECT(rs[r].alpha == r1.alpha);
      EXPECT(rs[r].b == r1.b);
    }
  }
  // clip=box keeps sum(alpha*y) == 0
  p.clip = ClipMode::Box;
  SolveResult rb = solve_cpu(ds, p);
  double s = 0;
  for (int64_t i = 0; i < ds.n; ++i) s += rb.alpha[i] * ds.y[i];
  EXPECT(std::fabs(s) < 1e-2);
  EXPECT(rb.status == 1);
  // accuracy on separable-ish blobs
  Model m = make_model(ds, r1.alpha, r1.b, p.gamma);
  auto dec = decision_cpu(m, ds.x.data(), ds.n, ds.d);
  EXPECT(accuracy_from_decision(dec, ds.y.data(), ds.n) > 0.8);
}

static void test_cpu_checkpoint_resume() {
  Dataset ds = make_synthetic(Synth::Blobs, 400, 3, 5, 0, -1, 1.0f);
  SolverParams p = small_params();
  SolveResult full = solve_cpu(ds, p);
  char path[] = "/tmp/dpsvm_ckXXXXXX";
  int fd = mkstemp(path);
  close(fd);
  SolverParams pc = p;
  pc.max_iter = full.iters / 2;
  pc.checkpoint_every = full.iters / 4;
  pc.checkpoint_path = path;
  solve_cpu(ds, pc);
  Checkpoint ck = read_checkpoint(path);
  EXPECT(ck.iter > 0 && ck.iter <= pc.max_iter);
  SolveResult res = solve_cpu(ds, p, nullptr, &ck);
  EXPECT(res.iters == full.iters);
  EXPECT(res.alpha == full.alpha);
  // resume without f: f recomputed from alpha (fp order differs -> close, not equal)
  ck.f.clear();
  SolveResult res2 = solve_cpu(ds, p, nullptr, &ck);
  EXPECT(res2.status == 1);
  EXPECT(std::fabs(res2.b - full.b) < 1e-2);
  unlink(path);
}

static void test_gpu() {
  if (device_count() == 0) {
    printf("  (no GPU: device tests skipped)\n");
    return;
  }
  Dataset ds = make_synthetic(Synth::Blobs, 3000, 20, 9, 0, -1, 1.0f);
  SolverParams p = small_params();
  p.gamma = 0.05f;
  SolveResult rc = solve_cpu(ds, p);
  for (int mode = 0; mode < 3; ++mode) {
    SolverParams pg = p;
    pg.engines = 1;                       // the pair-at-a-time cache / partitioned engines (quarantined)
    if (mode == 1) pg.cache_lines = 64;   // LRU + speculation
    if (mode == 2) pg.x_mode = 2;         // partitioned records, LRU
    GpuSolver s(pg, nullptr, 0);
    s.setup(ds.x.data(), ds.n, ds.n, ds.d, ds.y.data());
    SolveResult rg = s.solve();
    EXPECT(rg.status == 1);
    int64_t nsv_c = 0, nsv_g = 0;
    for (int64_t i = 0; i < ds.n; ++i) { nsv_c += rc.alpha[i] > 0; nsv_g += rg.alpha[i] > 0; }
    printf("  gpu mode %d: iters %lld (cpu %lld)  nsv %lld (cpu %lld)  b %g (cpu %g)\n", mode,
           (long long)rg.iters, (long long)rc.iters, (long long)nsv_g, (long long)nsv_c, rg.b, rc.b);
    EXPECT(std::llabs(nsv_g - nsv_c) <= std::max<int64_t>(3, nsv_c / 50));
    EXPECT(std::fabs(rg.b - rc.b) < 2e-2);
    double acc = s.train_accuracy(rg);
    Model m = make_model(ds, rc.alpha, rc.b, p.gamma);
    double accc = accuracy_from_decision(decision_cpu(m, ds.x.data(), ds.n, ds.d), ds.y.data(), ds.n);
    EXPECT(std::fabs(acc - accc) < 0.02);
  }
}

int main(int argc, char** argv) {
  bool gpu = argc > 1 && std::string(argv[1]) == "--gpu";
  std::vector<std::pair<const char*, std::function<void()>>> tests = {
      {"keys", test_keys},
      {"shards", test_shards},
      {"io", test_io},
      {"cpu_solver_ranks", test_cpu_solver_ranks},
      {"cpu_checkpoint_resume", test_cpu_checkpoint_resume},
  };
  if (gpu) tests.push_back({"gpu", test_gpu});
  for (auto& [name, fn] : tests) {
    int before = g_fail;
    try {
      fn();
    } catch (const std::exception& e) {
      ++g_fail;
      fprintf(stderr, "  EXCEPTION in %s: %s\n", name, e.what());
    }
    printf("%-28s %s\n", name, g_fail == before ? "ok" : "FAILED");
  }
  printf("%d checks passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
