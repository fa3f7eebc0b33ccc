// RCCL communicator (xGMI within a node).  Replaces the reference's OpenMPI
// C++ bindings over TCP (svmTrainMain.cpp:144-362, Makefile:74): device
// buffers, stream-ordered collectives (capturable into hipGraphs), local rank
// bound to its own GPU (the reference never calls cudaSetDevice).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

#include "dpsvm/comm.hpp"
#include "dpsvm/common.hpp"
#include "../runtime/hip_check.hpp"

namespace dpsvm {
namespace {

#define RCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess)                                                                \
      ::dpsvm::fail(std::string("RCCL error: ") + ncclGetErrorString(_r) + " at " #expr " [" \
                    __FILE__ ":" + std::to_string(__LINE__) + "]");                       \
  } while (0)

class RcclComm final : public Communicator {
 public:
  RcclComm(ncclComm_t c, int rank, int world, int device)
      : comm_(c), rank_(rank), world_(world), device_(device) {
    HIP_CHECK(hipSetDevice(device_));
    HIP_CHECK(hipMalloc(&scratch_, 64));
    HIP_CHECK(hipStreamCreateWithFlags(&bstream_, hipStreamNonBlocking));
  }
  ~RcclComm() override {
    (void)hipSetDevice(device_);
    if (scratch_) (void)hipFree(scratch_);
    if (bstream_) (void)hipStreamDestroy(bstream_);
    std::lock_guard<std::mutex> lk(mu_);
    if (comm_) ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  bool device_memory() const override { return true; }
  std::string name() const override { return "rccl"; }

  // Every collective runs under mu_ with the handle checked inside the lock,
  // so an abort can never free the communicator between the check and the
  // enqueue; ncclCommAbort itself only ever runs on the thread that issues the
  // collectives (abort() / a pending request seen by live() or async_error()).
  void allreduce_min_u64(uint64_t* buf, size_t count, hipStream_t s) override {
    std::lock_guard<std::mutex> lk(mu_);
    RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclUint64, ncclMin, live(), s));
  }
  void allreduce_sum_f64(double* buf, size_t count, hipStream_t s) override {
    std::lock_guard<std::mutex> lk(mu_);
    RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, live(), s));
  }
  void allreduce_sum_f32(float* buf, size_t count, hipStream_t s) override {
    std::lock_guard<std::mutex> lk(mu_);
    RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, live(), s));
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    std::lock_guard<std::mutex> lk(mu_);
    RCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, live(), s));
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
    std::lock_guard<std::mutex> lk(mu_);
    RCCL_CHECK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, live(), s));
  }
  void barrier() override {
    HIP_CHECK(hipSetDevice(device_));
    {
      std::lock_guard<std::mutex> lk(mu_);
      RCCL_CHECK(ncclAllReduce(scratch_, scratch_, 1, ncclInt32, ncclSum, live(), bstream_));
    }
    // bounded by the same abort path as the solver's waits: a peer that died
    // before the barrier makes this rank fail once someone requests the abort
    while (true) {
      hipError_t q = hipStreamQuery(bstream_);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) HIP_CHECK(q);
      std::string err = async_error();
      if (!err.empty()) ::dpsvm::fail("RCCL barrier failed on rank " + std::to_string(rank_) + ": " + err);
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  std::string async_error() override {
    std::lock_guard<std::mutex> lk(mu_);
    if (abort_req_.load() && comm_) abort_locked();
    if (!comm_) return "communicator aborted";
    ncclResult_t e = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &e) != ncclSuccess) return "ncclCommGetAsyncError failed";
    return e == ncclSuccess ? std::string() : std::string(ncclGetErrorString(e));
  }
  // Owning thread: ncclCommAbort raises the communicator's abort flag, which
  // its in-flight kernels poll, so a collective blocked on a dead peer ends now
  // (the solver's wait loop then fails) instead of when the watchdog fires.
  // Every later call fails with "communicator aborted"; a hipGraph holding
  // this communicator's nodes must not be launched again (the solver checks
  // async_error() before every block).
  void abort() override {
    abort_req_.store(true);
    std::lock_guard<std::mutex> lk(mu_);
    if (comm_) abort_locked();
  }
  // Other threads: only the request (ncclCommAbort racing the owner's
  // enqueue would free the handle under it).
  void request_abort() override { abort_req_.store(true); }

 private:
  void abort_locked() {
    (void)hipSetDevice(device_);
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
  // with mu_ held
  ncclComm_t live() {
    if (abort_req_.load() && comm_) abort_locked();
    if (!comm_) ::dpsvm::fail("RCCL communicator aborted (rank " + std::to_string(rank_) + ")");
    return comm_;
  }
  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
  void* scratch_ = nullptr;
  hipStream_t bstream_ = nullptr;
  std::atomic<bool> abort_req_{false};
  std::mutex mu_;
};

}  // namespace

void sync_collective(Communicator* c, hipStream_t stream, const char* what, double limit_s) {
  const double limit = limit_s > 0.0 ? limit_s : kWatchdogDefaultS;
  const auto t0 = std::chrono::steady_clock::now();
  const bool multi = c != nullptr && c->size() > 1;
  for (int spins = 0;; ++spins) {
    const hipError_t q = hipStreamQuery(stream);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) HIP_CHECK(q);
    if (multi) {
      const std::string err = c->async_error();
      if (!err.empty()) {
        c->abort();
        ::dpsvm::fail(std::string(what) + ": collective failed on rank " + std::to_string(c->rank()) + ": " + err);
      }
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      if (multi) c->abort();
      ::dpsvm::fail(std::string(what) + ": collective did not finish within " + std::to_string(limit) + " s");
    }
    if (spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::vector<uint8_t>((uint8_t*)id.internal, (uint8_t*)id.internal + NCCL_UNIQUE_ID_BYTES);
}

std::unique_ptr<Communicator> make_rccl_comm(const std::vector<uint8_t>& uid, int rank, int world,
                                             int device) {
  DPSVM_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "RCCL unique id must be 128 bytes");
  ncclUniqueId id;
  memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  HIP_CHECK(hipSetDevice(device));
  ncclComm_t c;
  RCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
  return std::make_unique<RcclComm>(c, rank, world, device);
}

std::vector<std::unique_ptr<Communicator>> make_rccl_comms_all(const std::vector<int>& devices) {
  int n = (int)devices.size();
  std::vector<ncclComm_t> cs((size_t)n);
  RCCL_CHECK(ncclCommInitAll(cs.data(), n, devices.data()));
  std::vector<std::unique_ptr<Communicator>> out;
  for (int r = 0; r < n; ++r) out.push_back(std::make_unique<RcclComm>(cs[r], r, n, devices[r]));
  return out;
}

}  // namespace dpsvm
