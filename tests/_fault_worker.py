"""One rank of the GPU rank-death test (tests/test_failure_gpu.py): a sharded
working-set solve over gloo + the in-kernel peer exchange, ranks sharing
device 0.  DPSVM_FAULT=exit@K:1 in the environment kills rank 1 mid-solve; the
surviving rank must report an error by itself (exchange poll timeout), not hang.
Prints one line "rank R: finished|error: ..." and exits 0 / 1."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from dpsvm_amd import SVC
    from dpsvm_amd.parallel import init_distributed, make_comm
    from dpsvm_amd.utils.datasets import synthetic

    ctx = init_distributed(device="cuda", timeout_s=40)
    comm = make_comm(ctx, kind="gloo")
    X, y = synthetic("mnist", n=12000, seed=3)
    try:
        SVC(device="cuda", C=10.0, gamma=0.25, solver="ws", dp="shard", xch_timeout_s=15.0,
            watchdog_s=30.0).fit(X, y, comm=comm)
        print(f"rank {ctx.rank}: finished", flush=True)
        return 0
    except Exception as e:  # noqa: BLE001
        print(f"rank {ctx.rank}: error: {str(e)[:300]}", flush=True)
        return 1


if __name__ == "__main__":
    sys.exit(main())
