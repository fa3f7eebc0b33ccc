// RCCL communicator (xGMI within a node).  Replaces the reference's OpenMPI
// C++ bindings over TCP (svmTrainMain.cpp:144-362, Makefile:74): device
// buffers, stream-ordered collectives (capturable into hipGraphs), local rank
// bound to its own GPU (the reference never calls cudaSetDevice).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

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
    if (comm_) {
      if (aborted_) ncclCommAbort(comm_);
      else ncclCommDestroy(comm_);
    }
  }
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  bool device_memory() const override { return true; }
  std::string name() const override { return "rccl"; }

  void allreduce_min_u64(uint64_t* buf, size_t count, hipStream_t s) override {
    RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclUint64, ncclMin, comm_, s));
  }
  void allreduce_sum_f64(double* buf, size_t count, hipStream_t s) override {
    RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, comm_, s));
  }
  void allreduce_sum_f32(float* buf, size_t count, hipStream_t s) override {
    RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm_, s));
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    RCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
    RCCL_CHECK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, s));
  }
  void barrier() override {
    HIP_CHECK(hipSetDevice(device_));
    RCCL_CHECK(ncclAllReduce(scratch_, scratch_, 1, ncclInt32, ncclSum, comm_, bstream_));
    HIP_CHECK(hipStreamSynchronize(bstream_));
  }
  std::string async_error() override {
    ncclResult_t e = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &e) != ncclSuccess) return "ncclCommGetAsyncError failed";
    return e == ncclSuccess ? std::string() : std::string(ncclGetErrorString(e));
  }
  void abort() override { aborted_ = true; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
  void* scratch_ = nullptr;
  hipStream_t bstream_ = nullptr;
  bool aborted_ = false;
};

}  // namespace

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
