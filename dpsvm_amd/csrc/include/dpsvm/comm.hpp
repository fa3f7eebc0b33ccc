// Communicator abstraction for the data-parallel SMO solver.
//
// The reference's only hot-loop collective is a 16-byte-per-rank host MPI
// Allgather (svmTrainMain.cpp:244) plus 4 setup barriers (183,191,198,233).
// Here the per-iteration exchange is an element-wise MIN all-reduce of packed
// u64 selection keys (exact, deterministic) or, with partitioned X, an
// all-gather of per-rank candidate records that carry the candidate rows.
//
// Backends:
//   LocalComm    - world of one (no-ops)
//   ThreadComm   - N ranks as threads of one process (host rendezvous); used by
//                  the CLI's simulated ranks and the C++/pytest multi-rank tests
//   RcclComm     - RCCL over xGMI, device buffers, stream-ordered, graph-capturable
//   CallbackComm - (python bindings) host callbacks into torch.distributed/gloo
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

typedef struct ihipStream_t* hipStream_t;

namespace dpsvm {

class Communicator {
 public:
  virtual ~Communicator() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // true: collectives take DEVICE pointers and are enqueued on `stream`
  // false: collectives take HOST pointers and complete before returning
  virtual bool device_memory() const = 0;
  virtual std::string name() const = 0;

  virtual void allreduce_min_u64(uint64_t* buf, size_t count, hipStream_t stream) = 0;
  virtual void allreduce_sum_f64(double* buf, size_t count, hipStream_t stream) = 0;
  virtual void allreduce_sum_f32(float* buf, size_t count, hipStream_t stream) = 0;
  // recv must hold size()*bytes; rank r's block lands at recv + r*bytes
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t stream) = 0;
  virtual void broadcast(void* buf, size_t bytes, int root, hipStream_t stream) = 0;
  virtual void barrier() = 0;
  // RCCL: poll async errors (watchdog); others: no-op.  Called by the thread
  // that issues this communicator's collectives; it also carries out an abort
  // requested by another thread (request_abort), so a peer's failure ends a
  // collective blocked on it.
  virtual std::string async_error() { return {}; }
  // abort NOW, from the thread that issues this communicator's collectives
  virtual void abort() {}
  // any thread (e.g. a failed rank thread for its peers): ask for an abort;
  // the owning thread performs it at its next collective or async_error()
  // poll.  Host communicators abort at once (their abort is thread-safe).
  virtual void request_abort() { abort(); }
};

std::unique_ptr<Communicator> make_local_comm();

// Wait for `stream` after a device communicator's collective, bounded: polls
// the stream, the communicator's async error (which also carries out an abort
// another rank thread requested: a collective blocked on a failed peer ends
// instead of hanging the waiting rank forever) and a time limit (seconds;
// <= 0: the watchdog default).  Fails (dpsvm::fail) with `what` on error.
void sync_collective(Communicator* c, hipStream_t stream, const char* what, double limit_s = 0.0);

// ThreadComm: create a group once, then hand comm(r) to thread r.
class ThreadCommGroup {
 public:
  explicit ThreadCommGroup(int world);
  ~ThreadCommGroup();
  std::unique_ptr<Communicator> comm(int rank);
  struct Impl;

 private:
  std::shared_ptr<Impl> impl_;
};

// RCCL
std::vector<uint8_t> rccl_unique_id();  // 128 bytes
std::unique_ptr<Communicator> make_rccl_comm(const std::vector<uint8_t>& uid, int rank, int world,
                                             int device);
// single-process, one comm per device (ncclCommInitAll)
std::vector<std::unique_ptr<Communicator>> make_rccl_comms_all(const std::vector<int>& devices);

}  // namespace dpsvm
