// Tracing, fault injection and cross-rank verification hooks.
//
//   DPSVM_ROCTX=1        ROCTx ranges around setup / Gram / SMO loop / accuracy
//                        (visible in rocprofv3 --marker-trace); libroctx64 is
//                        dlopen'ed so no link dependency exists when unused.
//   DPSVM_FAULT=nan@K    poison f at the first block boundary at/after SMO
//                        iteration K (exercises the non-finite abort path).
//   DPSVM_FAULT=exit@K:R rank R's process dies (_exit(3)) at the first block
//                        boundary at/after iteration K: the surviving ranks
//                        must fail (bounded exchange polls, collective errors,
//                        watchdog) instead of hanging, and the last checkpoint
//                        resumes the run (any rank count).
//   DPSVM_FAULT=throw@K:R rank R's solve throws (its thread / process stays
//                        alive) at the first block boundary at/after iteration
//                        K: in-process ranks (svmTrain --ranks / -p) must
//                        abort their peers' communicators and report rank R's
//                        error as the root cause.
//   DPSVM_FAULT=throwphase@P:R  rank R throws right after shrinking phase P
//                        (gpu_shrink.cpp): its peers are then blocked in the
//                        phase boundary's collectives, which must end through
//                        the abort (bounded waits, sync_collective).
//   DPSVM_VERIFY=1       after solve: alpha in [0, C], f recomputed from alpha,
//                        and the cross-rank alpha digest (the digest alone runs
//                        by default at world > 1: SolverParams::verify_ranks).
#pragma once

#include <dlfcn.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

namespace dpsvm {
namespace trace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    const char* e = std::getenv("DPSVM_ROCTX");
    if (!e || e[0] != '1') return;
    void* h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW);
    if (!h) return;
    push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
    pop = (int (*)())dlsym(h, "roctxRangePop");
    if (!push || !pop) push = nullptr, pop = nullptr;
  }
  static Roctx& get() {
    static Roctx r;
    return r;
  }
};

class Range {
 public:
  explicit Range(const char* name) : on_(Roctx::get().push != nullptr) {
    if (on_) Roctx::get().push(name);
  }
  ~Range() {
    if (on_) Roctx::get().pop();
  }

 private:
  bool on_;
};

// DPSVM_FAULT=nan@K -> K, else -1
inline int64_t fault_nan_iter() {
  const char* e = std::getenv("DPSVM_FAULT");
  if (!e || strncmp(e, "nan@", 4) != 0) return -1;
  return atoll(e + 4);
}

// DPSVM_FAULT=exit@K:R -> K when this is rank R, else -1
inline int64_t fault_rank_iter(const char* kind, int rank) {
  const char* e = std::getenv("DPSVM_FAULT");
  const size_t k = strlen(kind);
  if (!e || strncmp(e, kind, k) != 0) return -1;
  const char* c = strchr(e + k, ':');
  if (!c || atoi(c + 1) != rank) return -1;
  return atoll(e + k);
}
inline int64_t fault_exit_iter(int rank) { return fault_rank_iter("exit@", rank); }
// DPSVM_FAULT=throw@K:R -> K when this is rank R, else -1
inline int64_t fault_throw_iter(int rank) { return fault_rank_iter("throw@", rank); }
// DPSVM_FAULT=throwphase@P:R -> P when this is rank R, else -1
inline int64_t fault_throw_phase(int rank) { return fault_rank_iter("throwphase@", rank); }

inline bool verify_enabled() {
  const char* e = std::getenv("DPSVM_VERIFY");
  return e && e[0] == '1';
}

// order-sensitive 64-bit hash of float bit patterns (FNV-1a over words)
inline uint64_t hash_floats(const float* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) {
    uint32_t u;
    memcpy(&u, p + i, 4);
    h ^= u;
    h *= 1099511628211ull;
  }
  return h;
}

}  // namespace trace
}  // namespace dpsvm
