// Host-memory communicators: LocalComm (world of one) and ThreadComm (ranks as
// threads of one process).  ThreadComm is the in-process stand-in for the
// reference's `mpirun -np P` on one host (Makefile:88-89): it lets
// the full P-rank algorithm run, and be tested, with a single GPU or none.
#include <condition_variable>
#include <cstring>
#include <mutex>

#include "dpsvm/comm.hpp"
#include "dpsvm/common.hpp"

namespace dpsvm {
namespace {

class LocalComm final : public Communicator {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  bool device_memory() const override { return false; }
  std::string name() const override { return "local"; }
  void allreduce_min_u64(uint64_t*, size_t, hipStream_t) override {}
  void allreduce_sum_f64(double*, size_t, hipStream_t) override {}
  void allreduce_sum_f32(float*, size_t, hipStream_t) override {}
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t) override {
    if (send != recv) memmove(recv, send, bytes);
  }
  void broadcast(void*, size_t, int, hipStream_t) override {}
  void barrier() override {}
};

}  // namespace

std::unique_ptr<Communicator> make_local_comm() { return std::make_unique<LocalComm>(); }

struct ThreadCommGroup::Impl {
  explicit Impl(int w) : world(w), ptrs((size_t)w, nullptr) {}
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<const void*> ptrs;
  bool aborted = false;

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) fail("ThreadComm aborted");
    uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
      if (aborted) fail("ThreadComm aborted");
    }
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

namespace {

class ThreadComm final : public Communicator {
 public:
  ThreadComm(std::shared_ptr<ThreadCommGroup::Impl> g, int r) : g_(std::move(g)), rank_(r) {}
  int rank() const override { return rank_; }
  int size() const override { return g_->world; }
  bool device_memory() const override { return false; }
  std::string name() const override { return "thread"; }

  template <class T, class Op>
  void allreduce(T* buf, size_t count, Op op) {
    g_->ptrs[rank_] = buf;
    g_->barrier();
    std::vector<T> tmp(buf, buf + count);
    for (int r = 0; r < g_->world; ++r) {
      if (r == rank_) continue;
      const T* o = (const T*)g_->ptrs[r];
      for (size_t i = 0; i < count; ++i) tmp[i] = op(tmp[i], o[i]);
    }
    g_->barrier();
    memcpy(buf, tmp.data(), count * sizeof(T));
    g_->barrier();
  }
  void allreduce_min_u64(uint64_t* buf, size_t count, hipStream_t) override {
    allreduce(buf, count, [](uint64_t a, uint64_t b) { return a < b ? a : b; });
  }
  void allreduce_sum_f64(double* buf, size_t count, hipStream_t) override {
    // deterministic: sum in rank order regardless of the calling rank
    g_->ptrs[rank_] = buf;
    g_->barrier();
    std::vector<double> tmp(count, 0.0);
    for (int r = 0; r < g_->world; ++r) {
      const double* o = (const double*)g_->ptrs[r];
      for (size_t i = 0; i < count; ++i) tmp[i] += o[i];
    }
    g_->barrier();
    memcpy(buf, tmp.data(), count * sizeof(double));
    g_->barrier();
  }
  void allreduce_sum_f32(float* buf, size_t count, hipStream_t) override {
    g_->ptrs[rank_] = buf;
    g_->barrier();
    std::vector<float> tmp(count, 0.f);
    for (int r = 0; r < g_->world; ++r) {
      const float* o = (const float*)g_->ptrs[r];
      for (size_t i = 0; i < count; ++i) tmp[i] += o[i];
    }
    g_->barrier();
    memcpy(buf, tmp.data(), count * sizeof(float));
    g_->barrier();
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t) override {
    g_->ptrs[rank_] = send;
    g_->barrier();
    std::vector<char> tmp(bytes * g_->world);
    for (int r = 0; r < g_->world; ++r) memcpy(tmp.data() + r * bytes, g_->ptrs[r], bytes);
    g_->barrier();
    memcpy(recv, tmp.data(), tmp.size());
    g_->barrier();
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t) override {
    g_->ptrs[rank_] = buf;
    g_->barrier();
    std::vector<char> tmp((const char*)g_->ptrs[root], (const char*)g_->ptrs[root] + bytes);
    g_->barrier();
    if (rank_ != root) memcpy(buf, tmp.data(), bytes);
    g_->barrier();
  }
  void barrier() override { g_->barrier(); }
  void abort() override { g_->abort(); }

 private:
  std::shared_ptr<ThreadCommGroup::Impl> g_;
  int rank_;
};

}  // namespace

ThreadCommGroup::ThreadCommGroup(int world) : impl_(std::make_shared<Impl>(world)) {
  DPSVM_CHECK(world >= 1, "ThreadCommGroup world must be >= 1");
}
ThreadCommGroup::~ThreadCommGroup() = default;
std::unique_ptr<Communicator> ThreadCommGroup::comm(int rank) {
  DPSVM_CHECK(rank >= 0 && rank < impl_->world, "ThreadCommGroup rank out of range");
  return std::make_unique<ThreadComm>(impl_, rank);
}

}  // namespace dpsvm
