"""Data parallelism (row sharding of the SMO state across GPUs).

See :mod:`dpsvm_amd.parallel.dist`.  The native layer additionally offers
in-process communicators: ``native().ThreadCommGroup(world)`` (ranks as
threads; the CLI's ``--ranks``) and ``native().local_comm()``.
"""
from .dist import (CommUnavailable, DistContext, agree, gloo_comm, init_distributed, make_comm,  # noqa: F401
                   rccl_comm, shutdown, train_distributed)

__all__ = ["CommUnavailable", "DistContext", "agree", "init_distributed", "make_comm", "gloo_comm", "rccl_comm",
           "shutdown", "train_distributed"]
