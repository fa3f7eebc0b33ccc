"""Worker for the peer-exchange multi-process GPU tests (two, four or eight ranks,
launched by torch.distributed.run): train with the in-kernel peer exchange, write the
result digest to <out>.rank<r>.json."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out: str, engine: str, n: int, extra_json: str = "{}") -> int:
    import torch  # noqa: F401
    from dpsvm_amd import SVC
    from dpsvm_amd.parallel import init_distributed, make_comm, shutdown
    from dpsvm_amd.utils.datasets import synthetic

    ctx = init_distributed(device="cuda")
    comm = make_comm(ctx, "gloo")
    knobs = json.loads(extra_json)
    data = knobs.pop("_data", "covtype")  # "mnist": the uncoupled headline shape (C 10, gamma 0.25)
    X, y = synthetic(data, n=n, seed=2)
    hp = dict(C=10.0, gamma=0.25) if data == "mnist" else dict(C=4.0, gamma=0.5)
    extra = {"cache_lines": 256, "engines": "all"} if engine == "persistent-cache" else {}
    if engine.startswith("ws"):  # working-set rounds, rows sharded (candidates + sub-Gram rows in-kernel)
        extra = {"solver": "ws", "dp": "shard"}
        if engine == "ws-cache":
            extra.update(force_cache=True, cache_lines=1500)
    else:
        extra.update(persist="off" if engine == "fused" else "on", persist_block=257)
    extra.update(knobs)  # SVCConfig knobs (geometry, poll batch, ...)
    clf = SVC(eps=1e-3, device=ctx.device, exchange="peer", xch_timeout_s=30.0, **hp,
              **extra).fit(X, y, comm=comm)
    rec = {"exchange": clf.setup_info_["exchange"], "iteration": clf.setup_info_["iteration"],
           "exchange_mem": clf.setup_info_["exchange_mem"],
           "iters": int(clf.n_iter_), "rounds": int(getattr(clf, "n_rounds_", 0) or 0), "b": float(clf.b_),
           "alpha_sha": hashlib.sha256(clf.alpha_.tobytes()).hexdigest(),
           "ws_blocks": int(clf.stats_.get("ws_blocks", 1) or 1), "engine_note": clf.setup_info_.get("engine_note", ""),
           "ws_exchange": clf.setup_info_.get("ws_exchange", "none"),
           "ws_p1_round": int(clf.stats_.get("ws_p1_round", 0) or 0)}
    with open(f"{out}.rank{ctx.rank}.json", "w") as f:
        json.dump(rec, f)
    del comm
    shutdown(ctx)
    return 0


if __name__ == "__main__":
    try:
        sys.exit(main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 6000,
                      sys.argv[4] if len(sys.argv) > 4 else "{}"))
    except Exception as e:  # the test reads this instead of torchrun's summary
        import traceback

        with open(f"{sys.argv[1]}.rank{os.environ.get('RANK', '0')}.err", "w") as f:
            f.write(f"{type(e).__name__}: {e}\n{traceback.format_exc()}")
        raise
