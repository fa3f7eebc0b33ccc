"""Multi-process data parallelism: one process per GPU, torch.distributed
bootstrap, RCCL over xGMI for the SMO collectives.

Reference: OpenMPI ranks over TCP, `mpirun -np P --hostfile hf` (Makefile:74),
contiguous row shards (svmTrainMain.cpp:367-384), one 16-byte host Allgather
per iteration (svmTrainMain.cpp:244).

Here:
  * ranks come from torchrun / torch.distributed.run env (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT);
  * each rank binds GPU LOCAL_RANK (the reference never calls cudaSetDevice);
  * the per-iteration collective runs inside the native solver on a native
    RCCL communicator (device buffers, stream-ordered, captured into the
    iteration hipGraph); its 128-byte unique id is broadcast through the
    torch.distributed store/process group;
  * on CPU (tests, no GPU) the same native solver runs with a callback
    communicator backed by torch.distributed/gloo.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .._native import gpu_available, load


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: str = "cpu"          # "cuda:<local_rank>" or "cpu"
    backend: str = "none"        # torch.distributed backend in use
    initialized_here: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(device: str = "auto", timeout_s: int = 1800) -> DistContext:
    """Initialise torch.distributed from the torchrun environment (idempotent).

    GPU: backend "cpu:gloo,cuda:nccl" — RCCL for device tensors, gloo for the
    small host-side bootstrap objects.  CPU: "gloo".
    """
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DPSVM_FORCE_DEVICE"):
        # testing aid: several ranks share one GPU (e.g. a 1-GPU box rehearsing N > 1)
        local_rank = int(os.environ["DPSVM_FORCE_DEVICE"])
    use_gpu = (device == "cuda") or (device == "auto" and gpu_available())
    ctx = DistContext(rank=rank, world=world, local_rank=local_rank,
                      device=f"cuda:{local_rank}" if use_gpu else "cpu")
    if use_gpu:
        torch.cuda.set_device(local_rank)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # lazy NCCL(RCCL) init (no device_id): ranks rehearsing on a shared GPU
        # (DPSVM_FORCE_DEVICE) only ever touch the gloo side
        shared_gpu = bool(os.environ.get("DPSVM_FORCE_DEVICE"))
        backend = "cpu:gloo,cuda:nccl" if (use_gpu and not shared_gpu) else "gloo"
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
        ctx.backend = backend
        ctx.initialized_here = True
    elif dist.is_initialized():
        ctx.backend = str(dist.get_backend())
    return ctx


def shutdown(ctx: DistContext) -> None:
    import torch.distributed as dist

    if ctx.initialized_here and dist.is_initialized():
        dist.destroy_process_group()


def _host_group():
    """A gloo group for host-side callbacks (the default group may be NCCL-only)."""
    import torch.distributed as dist

    be = str(dist.get_backend())
    if "gloo" in be:
        return None
    global _GLOO
    try:
        return _GLOO
    except NameError:
        _GLOO = dist.new_group(backend="gloo")
        return _GLOO


_U64_FLIP = np.uint64(1 << 63)


def gloo_comm(ctx: DistContext):
    """Native communicator whose collectives call torch.distributed (gloo) on
    host buffers.  Used by the CPU solver and by GPU tests with several ranks
    sharing one device (RCCL refuses duplicate GPUs)."""
    import torch
    import torch.distributed as dist

    C = load()
    if ctx.world == 1:
        return C.local_comm()
    grp = _host_group()

    def ar_min_u64(a: np.ndarray) -> None:
        # order-preserving u64 -> i64 map (flip the top bit), MIN, map back
        t = torch.from_numpy((a ^ _U64_FLIP).view(np.int64).copy())
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=grp)
        a[:] = t.numpy().view(np.uint64) ^ _U64_FLIP

    def ar_sum_f64(a: np.ndarray) -> None:
        t = torch.from_numpy(a)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=grp)

    def ar_sum_f32(a: np.ndarray) -> None:
        t = torch.from_numpy(a)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=grp)

    def allgather(send: np.ndarray, recv: np.ndarray) -> None:
        n = send.shape[0]
        outs = [torch.from_numpy(recv[r * n:(r + 1) * n]) for r in range(ctx.world)]
        dist.all_gather(outs, torch.from_numpy(send), group=grp)

    def broadcast(a: np.ndarray, root: int) -> None:
        dist.broadcast(torch.from_numpy(a), src=root, group=grp)

    def barrier() -> None:
        dist.barrier(group=grp)

    return C.callback_comm(ctx.rank, ctx.world, ar_min_u64, ar_sum_f64, ar_sum_f32, allgather, broadcast,
                           barrier)


def agree(ok: bool) -> bool:
    """True on every rank iff ``ok`` is true on every rank (host group MIN)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=_host_group())
    return bool(t.item())


class CommUnavailable(RuntimeError):
    """Raised on EVERY rank when a communicator could not be built on some rank."""


def rccl_comm(ctx: DistContext):
    """Native RCCL communicator on this rank's GPU (xGMI), bootstrapped by
    broadcasting ncclGetUniqueId's 128 bytes through torch.distributed.

    Every step BEFORE the blocking ncclCommInitRank that can fail on one rank
    only — the unique id on rank 0, this rank's device (present and bindable)
    — is followed by an agreement over the host (gloo) group, so a rank that
    cannot even start the bootstrap makes every rank raise CommUnavailable
    together instead of leaving the others blocked inside ncclCommInitRank.
    ncclCommInitRank itself is a collective: a rank that fails INSIDE it (after
    its peers entered) is only bounded by RCCL's bootstrap timeout; its own
    error is then agreed like the others."""
    import torch.distributed as dist

    C = load()
    if ctx.world == 1:
        # a real one-rank RCCL communicator (exercises the collective + graph
        # capture path on a single GPU; the solver needs force_collectives)
        return C.rccl_comm(C.rccl_unique_id(), 0, 1, ctx.local_rank)
    uid, err = None, ""
    if ctx.rank == 0:
        try:
            uid = C.rccl_unique_id()
        except Exception as e:  # noqa: BLE001
            err = str(e)
    obj = [uid]
    dist.broadcast_object_list(obj, src=0, group=_host_group())
    if not agree(obj[0] is not None):
        raise CommUnavailable(f"ncclGetUniqueId failed on rank 0 {err}".strip())
    dev_err = ""
    try:
        import torch

        n_dev = C.device_count()
        if ctx.local_rank >= n_dev:
            raise RuntimeError(f"local rank {ctx.local_rank} but {n_dev} visible devices")
        torch.cuda.set_device(ctx.local_rank)
    except Exception as e:  # noqa: BLE001
        dev_err = str(e) or type(e).__name__
    if not agree(not dev_err):
        raise CommUnavailable(f"device binding failed on some rank {dev_err}".strip())
    comm, err = None, ""
    try:
        comm = C.rccl_comm(obj[0], ctx.rank, ctx.world, ctx.local_rank)
    except Exception as e:  # noqa: BLE001
        err = str(e)
    if not agree(comm is not None):
        del comm
        raise CommUnavailable(f"ncclCommInitRank failed on some rank {err}".strip())
    return comm


def make_comm(ctx: DistContext, kind: str = "auto"):
    """kind: auto (rccl on GPU, gloo on CPU; RCCL failing on any rank falls back
    to gloo on every rank) | rccl | gloo | local."""
    if kind == "local" or (ctx.world == 1 and kind in ("auto", "gloo")):
        return load().local_comm()
    if kind == "auto":
        if not ctx.device.startswith("cuda"):
            return gloo_comm(ctx)
        try:
            return rccl_comm(ctx)
        except CommUnavailable:
            return gloo_comm(ctx)
    return rccl_comm(ctx) if kind == "rccl" else gloo_comm(ctx)


def train_distributed(X, y, ctx: DistContext, comm=None, **svc_kwargs):
    """Train an SVC with every rank of ``ctx`` participating.

    X/y: the full training set on every rank (X replicated on device when it
    fits, as in the reference; pass x_mode="partitioned" to keep only the
    rank's rows on the GPU).  Returns the fitted SVC (identical on all ranks).
    """
    from ..models.svc import SVC

    if comm is None:
        comm = make_comm(ctx)
    device = svc_kwargs.pop("device", ctx.device)
    clf = SVC(device=device, **svc_kwargs)
    clf.fit(X, y, comm=comm)
    clf.comm_ = comm
    return clf
