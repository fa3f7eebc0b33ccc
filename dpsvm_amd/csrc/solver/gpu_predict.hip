// SV compaction, distributed training accuracy, decision values, the stand-
// alone GpuPredictor (svmTest GPU path) and the kernel-level test entry points.
// Reference: test_setup / aggregate_sv / get_train_accuracy (svmTrain.cu:569-665:
// rank 0 alone, n x (Sgemv + transform_reduce)) and seq_test.cpp:187-210.
#include <hip/hip_runtime.h>

#include "gpu_impl.hpp"

namespace dpsvm {

using gpu::dmalloc;
using gpu::round_up;

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
        sync_collective(m.comm, m.stream, "SV count all-reduce");
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
          sync_collective(m.comm, m.stream, "SV all-gather");
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
void gpu_local_decision(GpuSolver::Impl& m, const std::vector<float>& alpha, float* out_dev) {
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
      sync_collective(m.comm, m.stream, "accuracy all-reduce");
      (void)hipFree(dt);
    } else {
      m.comm->allreduce_sum_f64(&tot, 1, nullptr);
    }
  }
  return tot / (double)m.n;
}

std::vector<float> GpuSolver::gradient() const {
  const auto& m = *impl_;
  HIP_CHECK(hipSetDevice(m.device));
  std::vector<float> f((size_t)m.nl);
  if (m.nl > 0) HIP_CHECK(hipMemcpy(f.data(), m.f, (size_t)m.nl * 4, hipMemcpyDeviceToHost));
  return f;
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
  int precision = 0;  // launch::rbf_predict's: 0 auto, 1 f32, 2 split
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

GpuPredictor::GpuPredictor(const Model& mdl, int device, int precision) : impl_(new Impl) {
  auto& m = *impl_;
  DPSVM_CHECK(precision >= 0 && precision <= 2, "GpuPredictor: precision must be 0 (auto), 1 (f32) or 2 (split)");
  m.device = device;
  m.precision = precision;
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
                        nullptr, nullptr, m.stream, m.precision);
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
                      nullptr, nullptr, s, m.precision);
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

void stream_read(const void* x, int64_t bytes, float* out, int blocks, void* stream) {
  launch::stream_read(x, bytes, out, blocks, (hipStream_t)stream);
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
  gpu::need_quarantine("k_rbf_rows (smo_rows)").smo_rows(a, s);
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
  gpu::need_quarantine("k_select_partials (smo_step)").smo_step(a, s);
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

namespace {
// split rows (rbf_gemm_split.hip) of `rows` fp32 rows of x, in a fresh buffer
struct SplitRows {
  void* planes = nullptr;
  int32_t* shift = nullptr;
  SplitRows(const float* x, int64_t rows, int ld, hipStream_t s) {
    const int64_t pr = launch::split_pad_rows(rows);
    const size_t bytes = (size_t)pr * launch::split_row_u4(ld) * 16;
    size_t tb = 0;
    planes = dmalloc<uint8_t>(bytes, &tb);
    shift = dmalloc<int32_t>((size_t)pr, &tb);
    HIP_CHECK(hipMemsetAsync(planes, 0, bytes, s));
    HIP_CHECK(hipMemsetAsync(shift, 0, (size_t)pr * 4, s));
    launch::split_rows_f16(x, rows, ld, ld, planes, shift, s);
  }
  ~SplitRows() {
    (void)hipFree(planes);
    (void)hipFree(shift);
  }
};
}  // namespace

void rbf_gram_split(const float* a, const float* asq, int64_t m, const float* b, const float* bsq, int64_t n, int ld,
                    float gamma, float* out, int64_t out_ld, bool symmetric, void* stream, float cold_tau) {
  hipStream_t s = (hipStream_t)stream;
  SplitRows sa(a, m, ld, s);
  if (symmetric) {
    launch::rbf_gemm_store_split(sa.planes, sa.shift, asq, m, sa.planes, sa.shift, asq, n, ld, gamma, out, out_ld, s,
                                 true, cold_tau);
    HIP_CHECK(hipStreamSynchronize(s));
    return;
  }
  SplitRows sb(b, n, ld, s);
  launch::rbf_gemm_store_split(sa.planes, sa.shift, asq, m, sb.planes, sb.shift, bsq, n, ld, gamma, out, out_ld, s,
                               false, cold_tau);
  HIP_CHECK(hipStreamSynchronize(s));
}

std::pair<int64_t, int64_t> gram_adapt_last() {
  int64_t t = -1, h = -1;
  launch::gram_adapt_last(&t, &h);
  return {t, h};
}

void rbf_rows_indexed(const float* x, const float* xsq, int64_t n, int ld, const int* rows, int m, float gamma,
                      float* out, int64_t out_ld, const int* out_rows, void* stream, bool split) {
  DPSVM_CHECK(ld % 16 == 0 && m >= 0 && m <= 4096, "rbf_rows_indexed: ld multiple of 16, m <= 4096");
  hipStream_t s = (hipStream_t)stream;
  size_t tb = 0;
  int32_t* md = dmalloc<int32_t>(1, &tb);
  HIP_CHECK(hipMemcpyAsync(md, &m, 4, hipMemcpyHostToDevice, s));
  if (split) {
    SplitRows sx(x, n, ld, s);
    launch::rbf_rows_indexed_split(sx.planes, sx.shift, xsq, rows, md, m, sx.planes, sx.shift, xsq, n, ld, gamma, out,
                                   out_rows, out_ld, s);
    HIP_CHECK(hipStreamSynchronize(s));
  } else {
    launch::rbf_rows_indexed(x, xsq, rows, md, m, x, xsq, n, ld, gamma, out, out_rows, out_ld, s);
    HIP_CHECK(hipStreamSynchronize(s));
  }
  (void)hipFree(md);
}

std::vector<float> rbf_rows_indexed_split_bench(const float* x, const float* xsq, int64_t n, int ld, const int* rows,
                                                int m, float gamma, float* out, int64_t out_ld, const int* out_rows,
                                                int reps, void* stream) {
  DPSVM_CHECK(ld % 16 == 0 && m >= 0 && m <= 4096 && reps > 0, "rbf_rows_indexed_split_bench: arguments");
  hipStream_t s = (hipStream_t)stream;
  size_t tb = 0;
  int32_t* md = dmalloc<int32_t>(1, &tb);
  HIP_CHECK(hipMemcpyAsync(md, &m, 4, hipMemcpyHostToDevice, s));
  SplitRows sx(x, n, ld, s);
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < reps; ++r) {
    HIP_CHECK(hipEventRecord(e0, s));
    launch::rbf_rows_indexed_split(sx.planes, sx.shift, xsq, rows, md, m, sx.planes, sx.shift, xsq, n, ld, gamma, out,
                                   out_rows, out_ld, s);
    HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipEventSynchronize(e1));
    float t = 0.f;
    HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(md);
  return ms;
}

void xpass_rows(const float* x, const float* xsq, int64_t n, int ld, const int* keys, int nq, float gamma,
                float* out, int64_t out_ld, int rows_per_group, void* stream) {
  DPSVM_CHECK(ld % 16 == 0 && rows_per_group > 0 && rows_per_group % kFusedThreads == 0,
              "xpass_rows: ld multiple of 16, rows_per_group multiple of 256");
  const int64_t G = (n + rows_per_group - 1) / rows_per_group;
  DPSVM_CHECK(out_ld >= G * rows_per_group, "xpass_rows: out rows must cover every workgroup's tiles");
  SmoArgs a{};
  a.x = x;
  a.xsq = xsq;
  a.lines = out;
  a.ldl = out_ld;
  a.n = n;
  a.nl = n;
  a.off = 0;
  a.x_row0 = 0;
  a.dp = ld;
  a.d = ld;
  a.gamma = gamma;
  a.fused_rows = rows_per_group;
  a.fused_G = (int32_t)G;
  hipStream_t s = (hipStream_t)stream;
  gpu::need_quarantine("k_xpass_rows (xpass)").xpass_rows(a, keys, nq, s);
  HIP_CHECK(hipStreamSynchronize(s));
}

void fused_select(const float* f, const float* alpha, const float* y, int64_t n, float C, int rows_per_group,
                  uint64_t* keys_out, void* stream) {
  DPSVM_CHECK(rows_per_group > 0 && rows_per_group % kFusedThreads == 0, "fused_select: rows multiple of 256");
  SmoArgs a{};
  a.f = const_cast<float*>(f);
  a.alpha = const_cast<float*>(alpha);
  a.y = y;
  a.nl = n;
  a.n = n;
  a.off = 0;
  a.C = C;
  a.fused_rows = rows_per_group;
  a.fused_G = (int32_t)((n + rows_per_group - 1) / rows_per_group);
  a.xworld = 0;  // keys to memory, no exchange
  hipStream_t s = (hipStream_t)stream;
  launch::smo_fused(a, 0, nullptr, keys_out, nullptr, nullptr, s);
  HIP_CHECK(hipStreamSynchronize(s));
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
