// Kernel-level test entry points of the working-set engine (ws_*.hip): each
// runs ONE kernel (or the two f-update passes) on crafted device state and
// returns the state it leaves, so tests/test_kernels_gpu.py can check the
// merge (sort, stop test, union, block assignment), the LDS pair loop and the
// line-search f update against float64 numpy models of the same rules —
// independently of the end-to-end solves (tests/test_ws_gpu.py), where one
// kernel's bug could hide behind another's.
//
// Reference rules: the I-set classification and selection functors
// (svmTrain.cu:41-95, 400-467), the pair update and clipping
// (svmTrainMain.cpp:282-299), the f update (svmTrain.cu:98-137).
#include <hip/hip_runtime.h>

#include <cstring>

#include "gpu_impl.hpp"

namespace dpsvm {
namespace kernels {

namespace {

template <class T>
T* upload(const std::vector<T>& h, size_t count, hipStream_t s, size_t* tb) {
  T* d = gpu::dmalloc<T>(std::max<size_t>(count, 1), tb);
  HIP_CHECK(hipMemsetAsync(d, 0, std::max<size_t>(count, 1) * sizeof(T), s));
  if (!h.empty()) HIP_CHECK(hipMemcpyAsync(d, h.data(), std::min(h.size(), count) * sizeof(T), hipMemcpyHostToDevice, s));
  return d;
}

template <class T>
std::vector<T> download(const T* d, size_t count, hipStream_t s) {
  std::vector<T> h(count);
  if (count) HIP_CHECK(hipMemcpyAsync(h.data(), d, count * sizeof(T), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return h;
}

struct Stream {
  hipStream_t s = nullptr;
  std::vector<void*> bufs;
  Stream() { HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
  ~Stream() {
    (void)hipStreamSynchronize(s);
    for (void* p : bufs) (void)hipFree(p);
    (void)hipStreamDestroy(s);
  }
  template <class T>
  T* up(const std::vector<T>& h, size_t count) {
    size_t tb = 0;
    T* d = upload(h, count, s, &tb);
    bufs.push_back(d);
    return d;
  }
};

std::unique_ptr<WsCtrl> blank_ctrl() {
  auto c = std::make_unique<WsCtrl>();
  memset(c.get(), 0, sizeof(WsCtrl));
  c->done = kRunning;
  return c;
}

}  // namespace

WsMergeProbe ws_merge_multi_probe(const std::vector<uint64_t>& cand, int G, int blocks, int p_act, int q_max,
                                  int n_new, float eps, const std::vector<int32_t>& prev_union, int64_t iter,
                                  int64_t max_iter) {
  DPSVM_CHECK(G >= 1 && G <= kWsMaxGroups && (int64_t)cand.size() == (int64_t)G * 2 * kWsCand,
              "ws_merge_multi_probe: cand must be [G][2][kWsCand = 16] with G <= 256");
  DPSVM_CHECK(blocks >= 2 && blocks <= kWsMaxBlocks && q_max >= 2 && q_max <= kWsMax && q_max % 2 == 0,
              "ws_merge_multi_probe: 2 <= blocks <= 128, blocks x q_max <= 6144, even q_max <= 192");
  DPSVM_CHECK((int64_t)prev_union.size() <= (int64_t)blocks * q_max, "ws_merge_multi_probe: previous union too long");
  Stream st;
  auto c = blank_ctrl();
  c->outer = 1;  // this round builds parity 1; the previous union sits in parity 0
  c->iter = iter;
  c->uq[0] = (int32_t)prev_union.size();
  for (size_t i = 0; i < prev_union.size(); ++i) c->uidx[0][i] = prev_union[i];
  c->p_act = p_act;
  for (int i = 0; i < kWsMaxAll; ++i) c->idx[1][i] = -1;
  std::vector<WsCtrl> hc(1);
  memcpy(&hc[0], c.get(), sizeof(WsCtrl));
  WsCtrl* dc = st.up(hc, 1);
  WsArgs a{};
  a.cand = a.cand_out = st.up(cand, cand.size());
  a.G = a.G_all = G;
  a.world = 1;
  a.blocks = blocks;
  a.q_max = q_max;
  a.n_new = n_new;
  a.eps = eps;
  a.max_iter = max_iter;
  a.ctrl = dc;
  a.sorted = st.up(std::vector<uint64_t>(), (size_t)2 * kWsMaxGroups * kWsCand);
  launch::ws_merge_multi(a, st.s);
  const WsCtrl o = download(dc, 1, st.s)[0];
  WsMergeProbe r;
  r.done = o.done;
  r.b_hi = o.b_hi;
  r.b_lo = o.b_lo;
  r.p_round = o.p_round;
  if (o.done != kRunning) return r;
  r.uidx.assign(o.uidx[1], o.uidx[1] + o.uq[1]);
  r.qb.assign(o.qb[1], o.qb[1] + blocks);
  r.idx.assign((size_t)blocks * q_max, -1);
  for (int p = 0; p < blocks; ++p)
    for (int la = 0; la < o.qb[1][p]; ++la) r.idx[(size_t)p * q_max + la] = o.idx[1][p * q_max + la];
  return r;
}

WsSolveProbe ws_solve_probe(const std::vector<float>& K, const std::vector<float>& f, const std::vector<float>& alpha,
                            const std::vector<float>& y, const std::vector<int32_t>& qb, int q_max, int blocks,
                            int p_round, float C, int clip, float eps, float rel, float eps_floor, float tau,
                            float b_hi, float b_lo, int inner_max, int64_t iter0, int64_t max_iter, int wss) {
  DPSVM_CHECK(blocks >= 1 && blocks <= kWsMaxBlocks && (int)qb.size() == blocks && q_max >= 2 && q_max <= kWsMax,
              "ws_solve_probe: 1 <= blocks <= 128, qb per block, q_max <= 192");
  const size_t nq = (size_t)blocks * q_max;
  DPSVM_CHECK(K.size() == nq * q_max && f.size() == nq && alpha.size() == nq && y.size() == nq,
              "ws_solve_probe: K [P][q_max][q_max], f / alpha / y [P][q_max]");
  for (int p = 0; p < blocks; ++p) DPSVM_CHECK(qb[p] >= 0 && qb[p] <= q_max, "ws_solve_probe: qb[p] <= q_max");
  DPSVM_CHECK(blocks > 1 || p_round == 1, "ws_solve_probe: one block means p_round 1");
  Stream st;
  const int stride = blocks * kWsMax;
  std::vector<float> sub(nq * q_max + 3 * (size_t)stride, 0.f);
  std::copy(K.begin(), K.end(), sub.begin());
  float* aux = sub.data() + nq * q_max;
  for (int p = 0; p < blocks; ++p)
    for (int a = 0; a < qb[p]; ++a) {
      const size_t g = (size_t)p * q_max + a;
      aux[p * kWsMax + a] = f[g];
      aux[stride + p * kWsMax + a] = alpha[g];
      aux[2 * stride + p * kWsMax + a] = y[g];
    }
  auto c = blank_ctrl();
  c->iter = iter0;
  c->b_hi = b_hi;
  c->b_lo = b_lo;
  c->q[0] = qb[0];
  c->p_round = p_round;
  c->p_act = p_round;
  for (int p = 0; p < blocks; ++p) {
    c->qb[0][p] = qb[p];
    for (int a = 0; a < q_max; ++a) c->idx[0][p * q_max + a] = c->line[0][p * q_max + a] = p * q_max + a;
  }
  std::vector<WsCtrl> hc(1);
  memcpy(&hc[0], c.get(), sizeof(WsCtrl));
  WsCtrl* dc = st.up(hc, 1);
  float* dsub = st.up(sub, sub.size());
  WsArgs a{};
  a.subg = dsub;
  a.aux = dsub + nq * q_max;
  a.aux_stride = stride;
  a.alpha = st.up(alpha, nq);
  a.dalpha = st.up(std::vector<float>(nq, 0.f), nq);
  a.blocks = blocks;
  a.q_max = q_max;
  a.inner_max = inner_max;
  a.rel_local = rel;
  a.eps_floor = eps_floor;
  a.C = C;
  a.eps = eps;
  a.tau = tau;
  a.clip = clip;
  a.max_iter = max_iter;
  a.wss = wss;
  a.clip_fallback = 1;
  a.t_halve = 0.9f;
  a.world = 1;
  a.ctrl = dc;
  launch::ws_solve(a, st.s);
  const WsCtrl o = download(dc, 1, st.s)[0];
  WsSolveProbe r;
  r.alpha = download(a.alpha, nq, st.s);
  r.iter = o.iter;
  r.outer = o.outer;
  r.done = o.done;
  r.p_act = o.p_act;
  r.p1_round = o.p1_round;
  if (blocks == 1) {
    r.steps = {(int32_t)(o.iter - iter0)};
    r.nab = {o.n_apply};
    r.apply_idx.assign(o.apply_idx, o.apply_idx + o.n_apply);
    r.apply_coef.assign(o.apply_coef, o.apply_coef + o.n_apply);
  } else {
    for (int p = 0; p < blocks; ++p) {
      r.steps.push_back(o.inb[p]);
      r.nab.push_back(o.nab[p]);
      r.apply_idx.insert(r.apply_idx.end(), o.apply_idx + p * q_max, o.apply_idx + p * q_max + o.nab[p]);
      r.apply_coef.insert(r.apply_coef.end(), o.apply_coef + p * q_max, o.apply_coef + p * q_max + o.nab[p]);
    }
  }
  return r;
}

WsSelectProbe ws_select_probe(const std::vector<float>& gram, int64_t L, int64_t ldg, const std::vector<float>& f,
                              const std::vector<float>& alpha, const std::vector<float>& y,
                              const std::vector<float>& dalpha, const std::vector<int32_t>& apply_line,
                              const std::vector<float>& apply_coef, const std::vector<int32_t>& nab, int blocks,
                              int p_round, int p_act, int q_max, float C, int64_t outer, int ks, int reps,
                              bool wide) {
  const int64_t n = (int64_t)f.size();
  DPSVM_CHECK(n >= 1 && (int64_t)alpha.size() == n && (int64_t)y.size() == n && (int64_t)dalpha.size() == n,
              "ws_select_probe: f / alpha / y / dalpha of n rows");
  DPSVM_CHECK(ldg >= n && (int64_t)gram.size() == L * ldg, "ws_select_probe: gram [L][ldg >= n]");
  DPSVM_CHECK(blocks >= 1 && blocks <= kWsMaxBlocks && (int)nab.size() == blocks && q_max >= 2 && q_max <= kWsMax,
              "ws_select_probe: nab per block, q_max <= 192");
  DPSVM_CHECK(apply_line.size() == apply_coef.size(), "ws_select_probe: apply lines / coefficients");
  int64_t tot = 0;
  for (int p = 0; p < blocks; ++p) {
    DPSVM_CHECK(nab[p] >= 0 && nab[p] <= q_max, "ws_select_probe: nab[p] <= q_max");
    tot += nab[p];
  }
  DPSVM_CHECK(tot == (int64_t)apply_line.size(), "ws_select_probe: sum(nab) apply rows");
  for (int32_t l : apply_line) DPSVM_CHECK(l >= 0 && l < L, "ws_select_probe: apply line out of range");
  int32_t G = 0, rpt = 0;
  launch::ws_geometry(n, 1, &G, &rpt);
  DPSVM_CHECK(rpt <= kWsMaxRPT, "ws_select_probe: too many rows");
  Stream st;
  auto c = blank_ctrl();
  c->outer = outer;
  c->n_apply = (int32_t)tot;
  c->p_round = p_round;
  c->p_act = p_act;
  int64_t at = 0;
  for (int p = 0; p < blocks; ++p) {
    c->nab[p] = nab[p];
    const int base = blocks == 1 ? 0 : p * q_max;
    for (int k = 0; k < nab[p]; ++k, ++at) {
      c->apply_line[base + k] = apply_line[at];
      c->apply_coef[base + k] = apply_coef[at];
      c->apply_idx[base + k] = apply_line[at];
    }
  }
  std::vector<WsCtrl> hc(1);
  memcpy(&hc[0], c.get(), sizeof(WsCtrl));
  WsArgs a{};
  a.ctrl = st.up(hc, 1);
  a.gram = st.up(gram, gram.size());
  a.ldg = ldg;
  a.f = st.up(f, (size_t)n);
  a.alpha = st.up(alpha, (size_t)n);
  a.y = st.up(y, (size_t)n);
  a.dalpha = st.up(dalpha, (size_t)n);
  a.ks = std::max(1, ks);
  a.p1G = G;
  if (wide && blocks > 1) {  // the wide pass 1 (ws_pass1_v4_kernel)
    a.p1v4 = 1;
    a.p1G = launch::ws_pass1_v4_groups(n);
  }
  a.dfs = st.up(std::vector<float>(), (size_t)n * a.ks);
  a.part = st.up(std::vector<double>(), (size_t)2 * a.p1G * a.ks);
  a.cand = a.cand_out = st.up(std::vector<uint64_t>(), (size_t)G * 2 * kWsCand);
  a.n = a.nl = n;
  a.off = 0;
  a.G = a.G_all = G;
  a.rpt = rpt;
  a.world = 1;
  a.rank = 0;
  a.q_max = q_max;
  a.C = C;
  a.blocks = blocks;
  a.t_halve = 0.9f;
  a.clip_fallback = 1;
  WsSelectProbe r;
  if (blocks > 1 && reps > 0) {
    // timing (bench/pass1_probe.py): pass 1 only reads the state, so it can repeat
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    for (int i = 0; i < reps; ++i) {
      HIP_CHECK(hipEventRecord(e0, st.s));
      launch::ws_select_pass(a, 1, st.s);
      HIP_CHECK(hipEventRecord(e1, st.s));
      HIP_CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      r.pass1_us.push_back(1e3 * ms);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  launch::ws_select(a, st.s);  // blocks > 1: pass 1 then pass 2
  const WsCtrl o = download(a.ctrl, 1, st.s)[0];
  r.G = G;
  r.rpt = rpt;
  r.f = download(a.f, (size_t)n, st.s);
  r.alpha = download(a.alpha, (size_t)n, st.s);
  r.dalpha = download(a.dalpha, (size_t)n, st.s);
  r.dfs = download(a.dfs, (size_t)n, st.s);  // slice 0 (all of it at ks = 1)
  r.part = download(a.part, (size_t)2 * a.p1G * a.ks, st.s);
  r.p1G = a.p1G;
  r.cand = download(a.cand_out, (size_t)G * 2 * kWsCand, st.s);
  r.t = o.t_last;
  r.p_act = o.p_act;
  r.n_damped = o.n_damped;
  r.p1_round = o.p1_round;
  r.nonfinite = o.nonfinite;
  return r;
}

}  // namespace kernels
}  // namespace dpsvm
