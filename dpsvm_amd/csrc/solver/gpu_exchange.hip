// Cross-rank plumbing of the device solver: small collectives that work on
// device (RCCL) and host (threads, gloo) communicators, the in-kernel peer
// exchange setup (receive buffers, IPC / peer mappings, self test) and the
// residency census of the persistent engines.
//
// Reference: one 16-byte MPI Allgather per iteration (svmTrainMain.cpp:244)
// and four setup barriers (svmTrainMain.cpp:183,191,198,233).
#include <hip/hip_runtime.h>

#include <unistd.h>

#include "gpu_impl.hpp"

namespace dpsvm {

using gpu::dmalloc;

void GpuSolver::Impl::allreduce_keys(uint64_t* buf, int64_t count) {
  if (comm->device_memory()) {
    comm->allreduce_min_u64(buf, (size_t)count, stream);  // in the iteration stream (waits: wait_event)
  } else {
    if ((int64_t)h_partials.size() < count) h_partials.resize((size_t)count);
    HIP_CHECK(hipMemcpyAsync(h_partials.data(), buf, 8 * count, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    comm->allreduce_min_u64(h_partials.data(), (size_t)count, nullptr);
    HIP_CHECK(hipMemcpyAsync(buf, h_partials.data(), 8 * count, hipMemcpyHostToDevice, stream));
  }
}

void GpuSolver::Impl::allgather_bytes(const void* send, void* recv, size_t nbytes) {
  if (world == 1) {
    memcpy(recv, send, nbytes);
    return;
  }
  if (comm->device_memory()) {
    size_t tb = 0;
    uint8_t* d = dmalloc<uint8_t>(nbytes * (world + 1), &tb);
    HIP_CHECK(hipMemcpy(d + nbytes * world, send, nbytes, hipMemcpyHostToDevice));
    comm->allgather(d + nbytes * world, d, nbytes, stream);
    HIP_CHECK(hipMemcpyAsync(recv, d, nbytes * world, hipMemcpyDeviceToHost, stream));
    sync_collective(comm, stream, "setup all-gather");
    (void)hipFree(d);
  } else {
    comm->allgather(send, recv, nbytes, nullptr);
  }
}

bool GpuSolver::Impl::all_agree(bool mine, Communicator* c, int w) {
  if (w == 1) return mine;
  uint64_t v = mine ? 1ull : 0ull;  // MIN over ranks: 1 only if every rank holds 1
  if (c->device_memory()) {
    size_t tb = 0;
    uint64_t* d = dmalloc<uint64_t>(1, &tb);
    HIP_CHECK(hipMemcpy(d, &v, 8, hipMemcpyHostToDevice));
    c->allreduce_min_u64(d, 1, stream);
    HIP_CHECK(hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, stream));
    sync_collective(c, stream, "setup agreement");
    (void)hipFree(d);
  } else {
    c->allreduce_min_u64(&v, 1, nullptr);
  }
  return v == 1ull;
}

// Peer exchange setup (collective over the communicator): receive buffers,
// pointer / IPC-handle all-gather, mapping, and an in-kernel ping that every
// rank must pass.  Returns false (everywhere) if any rank failed.
//
// Receive buffers that peers on OTHER devices write over xGMI must be uncached
// device memory: coarse-grained memory is only coherent within one device, so a
// poll could keep reading a stale line of this device's L2.  When that
// allocation fails at world > 1 the exchange is refused (every rank falls back
// to the communicator's all-reduce) unless coarse memory was asked for
// explicitly (xch_mem = 2, A/B runs on one device).
bool GpuSolver::Impl::setup_exchange(int64_t region_words) {
  struct alignas(16) XInfo {
    int64_t pid, device, ok;
    uint64_t ptr;
    hipIpcMemHandle_t handle;
  };
  XInfo me{};
  me.pid = (int64_t)getpid();
  me.device = device;
  me.ok = 1;
  const int64_t ping_words = 64;
  xstride = std::max<int64_t>(kXchGranules, p.xch_stride);
  xregion = region_words > 0 ? region_words : (int64_t)2 * world * Gf * xstride;
  try {
    DPSVM_CHECK(world <= 64, "peer exchange supports at most 64 ranks");
    launch::preload_fused_kernels(stream);
    launch::preload_persist_kernel(stream);
    if (const gpu::QuarantineOps* qo = gpu::quarantine()) qo->preload(stream);  // pair-cache plugin loaded
    const size_t xbytes = (size_t)(xregion + ping_words) * 8;
    const bool want_uc = p.xch_mem == 1 || (p.xch_mem == 0 && world > 1);
    bool got_uc = false;
    if (want_uc) {
      got_uc = hipExtMallocWithFlags((void**)&xbuf, xbytes, hipDeviceMallocUncached) == hipSuccess;
      if (!got_uc) {
        (void)hipGetLastError();
        xbuf = nullptr;
        if (world > 1) {
          xch_diag = "rank " + std::to_string(rank) + ": uncached receive buffer unavailable";
          fail(xch_diag + " (coarse memory is not coherent across devices; set xch_mem=coarse to force it)");
        }
      }
    }
    if (!got_uc) HIP_CHECK(hipMalloc((void**)&xbuf, xbytes));
    xch_mem = got_uc ? "uncached" : "coarse";
    HIP_CHECK(hipMemset(xbuf, 0, xbytes));
    HIP_CHECK(hipDeviceSynchronize());
    me.ptr = (uint64_t)xbuf;
    if (world > 1) HIP_CHECK(hipIpcGetMemHandle(&me.handle, xbuf));
  } catch (const std::exception& e) {
    if (p.verbose) fprintf(stderr, "[dpsvm] peer exchange unavailable on rank %d: %s\n", rank, e.what());
    me.ok = 0;
  }
  std::vector<XInfo> all((size_t)world);
  allgather_bytes(&me, all.data(), sizeof(XInfo));
  bool ok = true;
  for (const auto& r : all) ok &= r.ok != 0;
  for (int r = 0; r < world; ++r) {
    // rank threads of one process on one device: their streams may share a
    // hardware queue, so one spinning kernel can block the other's forever
    if (r != rank && all[r].pid == me.pid && all[r].device == me.device) {
      ok = false;
      xch_diag = "ranks " + std::to_string(rank) + " and " + std::to_string(r) + " share a device in one process";
    }
  }
  std::vector<uint64_t*> ptrs((size_t)world, nullptr);
  if (ok) {
    try {
      for (int r = 0; r < world; ++r) {
        if (r == rank) {
          ptrs[r] = xbuf;
        } else if (all[r].pid == me.pid) {  // rank thread of this process: direct pointer
          ptrs[r] = (uint64_t*)all[r].ptr;
          if (all[r].device != device) {
            const hipError_t e = hipDeviceEnablePeerAccess((int)all[r].device, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
            (void)hipGetLastError();
          }
        } else {  // other process: dmabuf IPC mapping (xGMI peer memory)
          void* q = nullptr;
          HIP_CHECK(hipIpcOpenMemHandle(&q, all[r].handle, hipIpcMemLazyEnablePeerAccess));
          xopened.push_back(q);
          ptrs[r] = (uint64_t*)q;
        }
      }
      size_t tb = 0;
      xpeer_d = dmalloc<uint64_t*>((size_t)world, &tb);
      HIP_CHECK(hipMemcpy(xpeer_d, ptrs.data(), world * sizeof(uint64_t*), hipMemcpyHostToDevice));
    } catch (const std::exception& e) {
      if (p.verbose) fprintf(stderr, "[dpsvm] peer mapping failed on rank %d: %s\n", rank, e.what());
      ok = false;
    }
  }
  // in-kernel self test (a rank that failed above does not ping: the others time out)
  size_t tb = 0;
  int32_t* okd = dmalloc<int32_t>(2, &tb);
  HIP_CHECK(hipMemsetAsync(okd, 0, 8, stream));  // stream-ordered before the ping (non-blocking stream)
  if (world > 1) comm->barrier();
  if (ok) launch::xch_ping(xpeer_d, rank, world, xregion, 1u, (int64_t)5e8 /* 5 s */, okd, stream);
  int32_t okh = 0;
  HIP_CHECK(hipMemcpyAsync(&okh, okd, 4, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  (void)hipFree(okd);
  if (xch_diag.empty())
    xch_diag = "rank " + std::to_string(rank) + ": mapped=" + std::to_string((int)ok) + " ping=" + std::to_string(okh);
  const bool all_ok = all_agree(ok && okh == 1, comm, world);
  if (!all_ok) {
    for (void* q : xopened) (void)hipIpcCloseMemHandle(q);
    xopened.clear();
    if (xbuf) (void)hipFree(xbuf);
    if (xpeer_d) (void)hipFree(xpeer_d);
    xbuf = nullptr;
    xpeer_d = nullptr;
    xch_mem = "none";
  }
  if (world > 1) comm->barrier();
  return all_ok;
}

// A persistent engine spins on its own workgroups' (and peers') publications,
// so every workgroup of its grid must be resident at once.  Checked twice:
// the occupancy API (resident blocks per CU x CUs >= grid) and a census run of
// the engine's own kernel with its own grid and resources (census_arrive):
// a partitioned device or CUs held elsewhere fail here, bounded, and every rank
// falls back to the one-launch-per-iteration engine together.
bool GpuSolver::Impl::census(EngineKind k) {
  const bool dense_k = k == EngineKind::PersistDense;
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  const int per_cu = dense_k ? launch::smo_persist_blocks_per_cu(args)
                             : gpu::need_quarantine("the persistent-cache census").persist_lru_blocks_per_cu(args);
  info.cus = cus;
  info.blocks_per_cu = per_cu;
  const int groups = p.census_groups > 0 ? p.census_groups : (int)Gf;
  // the API can answer one block per CU too many at some SGPR counts
  // (MI355X_MICROARCH.md, Residency): require one block of margin per CU
  // (a census_groups test grid skips this check: the census itself must catch it)
  bool ok = p.census_groups > 0 ||
            (per_cu >= 1 && (groups <= cus || (int64_t)(std::min(per_cu, 8) - 1) * cus >= groups));
  if (ok) {
    size_t tb = 0;
    int32_t* words = dmalloc<int32_t>(2, &tb);
    HIP_CHECK(hipMemsetAsync(words, 0, 8, stream));  // stream-ordered before the census kernel
    SmoArgs a = args;
    a.census = words;
    // 2 s (s_memrealtime: 100 MHz): a resident grid arrives within microseconds,
    // but ranks sharing a device (rehearsals) can have their queue time-sliced out
    a.census_ticks = (int64_t)(2.0 * 1e8);
    if (dense_k) launch::smo_persist_census(a, groups, stream);
    else gpu::need_quarantine("the persistent-cache census").persist_lru_census(a, groups, stream);
    int32_t h[2] = {0, 0};
    HIP_CHECK(hipMemcpyAsync(h, words, 8, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    (void)hipFree(words);
    ok = h[1] == 0 && h[0] == groups;
    if (!ok)
      info.engine_note = std::string(engine_name(k)) + ": census " + std::to_string(h[0]) + "/" +
                         std::to_string(groups) + " workgroups co-resident";
  } else {
    info.engine_note = std::string(engine_name(k)) + ": " + std::to_string(groups) + " workgroups > " +
                       std::to_string(per_cu) + " per CU x " + std::to_string(cus) + " CUs";
  }
  const bool agreed = all_agree(ok, comm, world);
  if (ok && !agreed) info.engine_note = std::string(engine_name(k)) + ": census failed on another rank";
  info.census = agreed ? "ok" : "failed";
  return agreed;
}

}  // namespace dpsvm
