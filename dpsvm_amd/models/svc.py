"""SVC: the estimator-level API over the native MI355X solver.

Reference capability map (farshid83/dpsvm):
  fit()                -> svmTrainMain.cpp:142-365 (GPU/MPI trainer) or seq.cpp (CPU)
  decision_function()  -> svmTrain.cu:633-665 (training accuracy) / seq_test.cpp:187-210
  save() / load_model()-> svmTrainMain.cpp:386-416 model writer, seq_test.cpp:212-249 reader
Labels: the reference requires +1/-1 (svmTrain.cu:58,73); any two distinct
labels are accepted here and mapped (classes_[1] -> +1), like scikit-learn.
"""
from __future__ import annotations

import dataclasses
import math
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Optional

import numpy as np

from .._native import gpu_available, load, load_quarantine


def _as_f32_2d(X) -> np.ndarray:
    try:
        import torch

        if isinstance(X, torch.Tensor):
            X = X.detach().to("cpu", dtype=torch.float32).numpy()
    except ImportError:
        pass
    X = np.ascontiguousarray(np.asarray(X, dtype=np.float32))
    if X.ndim != 2:
        raise ValueError(f"X must be 2-D (n_samples, n_features), got shape {X.shape}")
    return X


def _as_1d(y) -> np.ndarray:
    try:
        import torch

        if isinstance(y, torch.Tensor):
            y = y.detach().cpu().numpy()
    except ImportError:
        pass
    return np.asarray(y).reshape(-1)


_CLIP = {"independent": 0, "box": 1}
_XMODE = {"auto": 0, "replicated": 1, "partitioned": 2}
_EXCHANGE = {"auto": 0, "allreduce": 1, "peer": 2}
_PERSIST = {"auto": 0, "off": 1, "on": 2}
_CACHE_ENGINE = {"fused": 0, "chain": 1}
_XCH_MEM = {"auto": 0, "uncached": 1, "coarse": 2}
_DP = {"auto": 0, "shard": 1, "replicate": 2}
_SOLVER = {"auto": 0, "smo": 1, "ws": 2}


def _pick(table: dict, value: str, name: str) -> int:
    if value not in table:
        raise ValueError(f"{name} must be one of {list(table)}, got {value!r}")
    return table[value]


@dataclass
class SVCConfig:
    """Solver configuration (mirrors the svmTrain flags)."""

    C: float = 1.0                  # -c (reference default 1)
    gamma: Optional[float] = None   # -g; None -> 1/d (reference: integer 1/d, Q1)
    eps: float = 1e-3               # -e
    max_iter: int = 150000          # -n
    clip: str = "independent"       # reference clipping; "box" = LIBSVM joint box
    tau: float = 1e-12              # eta floor (Q4)
    cache_lines: int = 0            # -s (0 = auto: fill HBM; dense Gram when it fits)
    cache_mb: float = 0.0
    cache_frac: float = 0.80
    host_cache_lines: int = 0       # pinned host tier lines (LRU mode; 0 = off)
    spec_rows: int = 14             # speculative rows per X pass (LRU mode)
    graph_block: int = 64           # SMO iterations per hipGraph
    use_graph: bool = True
    x_mode: str = "auto"            # auto | replicated | partitioned
    log_every: int = 0
    checkpoint_path: Optional[str] = None
    checkpoint_every: int = 0
    device: str = "auto"            # auto | cpu | cuda | cuda:N
    verbose: bool = False
    force_collectives: bool = False  # run the per-iteration collective even with one rank (tests)
    exchange: str = "auto"          # per-iteration key exchange (dense mode): auto | allreduce | peer
    persist: str = "auto"           # engine: auto | off (one launch per iteration) | on (persistent, dense or cache mode)
    persist_block: int = 2048       # SMO iterations per persistent launch
    # engine / geometry selection (all recorded in setup_info_ and the run summaries)
    dp: str = "auto"                # world > 1: auto | shard (rows split) | replicate (every rank solves it all)
    force_cache: bool = False       # kernel-row cache mode even when the Gram fits
    cache_engine: str = "fused"     # cache mode, one launch per iteration: fused | chain
    # production (ws-dense, ws-cache, persistent-dense, fused-dense) | all: also the quarantined
    # pair-at-a-time engines for a non-resident Gram / partitioned X (persistent-cache, fused-cache, chain;
    # host_cache_lines and cache_engine=chain need it) — tests and A/B probes (device_state.hpp kQuarantineTable)
    engines: str = "production"
    cache_groups: int = 256         # cache mode workgroups per rank
    rows_per_group: int = 0         # rows per workgroup of the fused/persistent engines (0 auto; multiple of 256)
    xch_poll_batch: int = 0         # peer exchange: publications per lane per poll round (0 auto)
    xch_sleep: int = 1
    xch_stride: int = 4
    xch_mem: str = "auto"           # auto | uncached | coarse
    xch_timeout_s: float = 120.0    # give-up bound of one in-kernel poll (then the solve fails)
    watchdog_s: float = 0.0  # 0: auto (1800 s; adaptive to the block time at world > 1)
    census_groups: int = 0          # residency census grid (tests)
    verify_ranks: bool = True       # cross-rank alpha digest after each solve (world > 1)
    # solver: auto (ws from 50k rows, else smo) | smo (pair-at-a-time engines, the reference's trajectory) |
    # ws (working-set rounds: the reference's pair rule on a q-row sub-problem
    # in LDS, the same global stop test; ws_*.hip)
    solver: str = "auto"
    ws_size: int = 192              # working-set rows (<= 192)
    ws_new: int = 0                 # rows replaced per one-block round (0: auto, ws_size from 128 padded features, else 3/4)
    ws_rel: float = 0.3             # sub-problem tolerance relative to the global gap (< 1)
    # working-set engines: up to P sub-problems per round (1..128, P x ws_size <= 6144).  0 auto, from 50k rows:
    # uncoupled (numerically diagonal) ws-dense kernels 128 blocks of 48 rows (6144-row union; 64 x 48 = 3072
    # when ranks sharing one device would not leave room for the peer exchange's producers), coupled kernels
    # and ws-cache 32 blocks of 96 (3072-row union); below 50k rows 1.  Adaptive —
    # halved after every damped round (coupled blocks), then the one-block round kernels (ws_*.hip;
    # kWsMaxBlocks / kWsMaxAll in include/dpsvm/device_state.hpp)
    ws_blocks: int = 0
    ws_inner: int = 0               # pair steps per round at most (0: 4 * ws_size)
    ws_wss: int = 0                 # sub-problem pair choice: 0 auto (second order on coupled kernels), 1 first, 2 second
    ws_block: int = 8               # rounds per hipGraph block (or per persistent-round launch)
    # ws-cache rounds without the kernel-row cache (ws_recompute.hip: the round's kernel rows recomputed inside
    # the f update, the sub-Gram straight from X): auto (one GPU, one block, d <= 64) | on | off
    ws_recompute: str = "auto"
    # one GPU: LIBSVM-style shrinking as problem reduction (solve_shrinking: phases on the rows that can
    # still violate, the rest of the gradient updated by one predict GEMM per phase).  auto: on where it
    # pays — one GPU, working-set rounds, the whole Gram not resident (C.shrink_auto) | on | off
    shrink: str = "auto"
    ws_t_halve: float = 0.9         # multi-block: a round damped below this t halves the block count
    ws_clip_fallback: bool = True   # multi-block, independent clipping: one block per round after a clip
    eta: str = "x"                  # pair engines' K(hi, lo): x (from the X rows) | gram (resident Gram)
    # Gram / kernel-row GEMM arithmetic: auto (split for the working-set engines, f32 for the pair engines),
    # f32 (f32-input MFMA), split (fp16 MFMA over hi/lo split operands: fp32 accuracy, 3/16 of the MFMA time)
    gram: str = "auto"
    # adaptive resident split Gram (ws-dense, docs/DESIGN.md §13): one-product tiles where every element is
    # provably within gram_cold_tau of the three-product value, the rest recomputed — auto (on when a row
    # sample passes the bound) | on | off
    gram_adapt: str = "auto"
    gram_cold_tau: float = 2.0 ** -22

    def shrink_mode(self) -> str:
        s = self.shrink
        if s is True or s is False:
            return "on" if s else "off"
        if s not in ("auto", "on", "off"):
            raise ValueError(f"shrink must be auto, on or off (got {s!r})")
        return s

    def resolved_gamma(self, d: int) -> float:
        return float(self.gamma) if self.gamma is not None and self.gamma >= 0 else 1.0 / float(d)

    def to_native(self, d: int):
        C = load()
        if self.clip not in _CLIP:
            raise ValueError(f"clip must be one of {list(_CLIP)}")
        if self.x_mode not in _XMODE:
            raise ValueError(f"x_mode must be one of {list(_XMODE)}")
        if not self.C > 0:
            raise ValueError("C must be > 0")
        p = C.SolverParams()
        p.C = float(self.C)
        p.gamma = self.resolved_gamma(d)
        p.eps = float(self.eps)
        p.max_iter = int(self.max_iter)
        p.clip = C.ClipMode.box if self.clip == "box" else C.ClipMode.independent
        p.tau = float(self.tau)
        p.cache_lines = int(self.cache_lines)
        p.cache_mb = float(self.cache_mb)
        p.cache_frac = float(self.cache_frac)
        p.host_cache_lines = int(self.host_cache_lines)
        p.spec_rows = int(self.spec_rows)
        p.graph_block = int(self.graph_block)
        p.use_graph = bool(self.use_graph)
        p.x_mode = _XMODE[self.x_mode]
        p.log_every = int(self.log_every)
        p.verbose = bool(self.verbose)
        p.checkpoint_every = int(self.checkpoint_every)
        p.checkpoint_path = self.checkpoint_path or ""
        p.force_collectives = bool(self.force_collectives)
        if self.exchange not in _EXCHANGE:
            raise ValueError(f"exchange must be one of {list(_EXCHANGE)}")
        p.exchange = _EXCHANGE[self.exchange]
        if self.persist not in _PERSIST:
            raise ValueError(f"persist must be one of {list(_PERSIST)}")
        p.persist = _PERSIST[self.persist]
        p.persist_block = int(self.persist_block)
        p.dp_policy = _pick(_DP, self.dp, "dp")
        p.force_cache = bool(self.force_cache)
        p.cache_engine = _pick(_CACHE_ENGINE, self.cache_engine, "cache_engine")
        p.engines = _pick({"production": 0, "all": 1}, self.engines, "engines")
        p.cache_groups = int(self.cache_groups)
        if self.rows_per_group % 256:
            raise ValueError("rows_per_group must be a multiple of 256")
        p.rows_per_group = int(self.rows_per_group)
        p.xch_poll_batch = int(self.xch_poll_batch)
        p.xch_sleep = int(self.xch_sleep)
        p.xch_stride = int(self.xch_stride)
        p.xch_mem = _pick(_XCH_MEM, self.xch_mem, "xch_mem")
        p.xch_timeout_s = float(self.xch_timeout_s)
        p.watchdog_s = float(self.watchdog_s)
        p.census_groups = int(self.census_groups)
        p.verify_ranks = bool(self.verify_ranks)
        p.solver = _pick(_SOLVER, self.solver, "solver")
        p.ws_size = int(self.ws_size)
        p.ws_new = int(self.ws_new)
        p.ws_rel = float(self.ws_rel)
        p.ws_blocks = int(self.ws_blocks)
        p.ws_inner = int(self.ws_inner)
        p.ws_wss = int(self.ws_wss)
        p.ws_t_halve = float(self.ws_t_halve)
        p.ws_clip_fallback = int(bool(self.ws_clip_fallback))
        p.ws_block = int(self.ws_block)
        p.ws_recompute = _pick({"auto": 0, "on": 1, "off": 2}, self.ws_recompute, "ws_recompute")
        p.eta = _pick({"x": 0, "gram": 1}, self.eta, "eta")
        p.gram_precision = _pick({"auto": 0, "f32": 1, "split": 2}, self.gram, "gram")
        p.gram_adapt = _pick({"auto": 0, "on": 1, "off": 2}, self.gram_adapt, "gram_adapt")
        p.gram_cold_tau = float(self.gram_cold_tau)
        return p

    def device_kind(self) -> tuple[str, int]:
        dev = self.device
        if dev == "auto":
            return ("cuda", 0) if gpu_available() else ("cpu", 0)
        if dev == "cpu":
            return ("cpu", 0)
        if dev.startswith("cuda"):
            idx = int(dev.split(":")[1]) if ":" in dev else 0
            return ("cuda", idx)
        raise ValueError(f"unknown device {dev!r}")


class SVC:
    """Binary RBF C-SVM trained by modified SMO on MI355X (or the CPU).

    Attributes after fit: ``alpha_`` (dual variables, len n), ``b_`` (threshold:
    decision = sum alpha_i y_i K(x_i, x) - b), ``intercept_`` (= -b_),
    ``support_`` (indices with alpha > 0), ``support_vectors_``, ``dual_coef_``
    (alpha*y of the SVs), ``n_iter_``, ``status_``, ``fit_time_`` (SMO loop
    seconds, the reference's timed region), ``stats_`` (cache / pass counters).
    """

    def __init__(self, C: float = 1.0, gamma: Optional[float] = None, eps: float = 1e-3,
                 max_iter: int = 150000, device: str = "auto", **kwargs: Any):
        self.config = SVCConfig(C=C, gamma=gamma, eps=eps, max_iter=max_iter, device=device, **kwargs)
        self._model = None
        self._gpu_pred = None
        self.classes_ = np.array([-1.0, 1.0], dtype=np.float32)

    # ------------------------------------------------------------------ labels
    def _encode(self, y) -> np.ndarray:
        y = _as_1d(y)
        u = np.unique(y)
        if len(u) > 2:
            raise ValueError(f"binary classifier: got {len(u)} classes")
        if len(u) == 2 and set(u.tolist()) <= {-1, 1}:
            self.classes_ = np.array([-1.0, 1.0], dtype=np.float32)
            return np.where(y > 0, 1.0, -1.0).astype(np.float32)
        if len(u) == 1:
            self.classes_ = np.array([u[0], u[0]])
            return np.ones(len(y), dtype=np.float32) * (1.0 if (u[0] > 0 if np.isreal(u[0]) else True) else -1.0)
        self.classes_ = u
        return np.where(y == u[1], 1.0, -1.0).astype(np.float32)

    def _decode(self, s: np.ndarray) -> np.ndarray:
        if np.array_equal(self.classes_, np.array([-1.0, 1.0], dtype=np.float32)):
            return s.astype(np.float32)
        return np.where(s > 0, self.classes_[-1], self.classes_[0])

    def _use_shrink(self, p, n: int, d: int, dev: int, comm=None) -> bool:
        """collective at world > 1 (every rank calls; agreed)"""
        mode = self.config.shrink_mode()
        return mode == "on" or (mode == "auto" and bool(load().shrink_auto(p, n, d, dev, comm)))

    # ------------------------------------------------------------------ fit
    def fit(self, X, y, comm=None, resume=None, progress: Optional[Callable] = None,
            rank_rows: Optional[int] = None) -> "SVC":
        """Train.  ``comm``: a native communicator (see dpsvm_amd.parallel) for
        multi-rank training; ``resume``: checkpoint path or native Checkpoint."""
        C = load()
        if self.config.engines == "all" or self.config.host_cache_lines or self.config.cache_engine == "chain":
            load_quarantine()  # the quarantined pair-at-a-time cache engines (plugin)
        X = _as_f32_2d(X)
        ys = self._encode(y)
        n, d = X.shape[0], X.shape[1]
        if rank_rows is None and ys.shape[0] != n:
            raise ValueError("len(y) != X.shape[0]")
        cfg = self.config
        p = cfg.to_native(d)
        if cfg.log_every and progress is None:
            def progress(it, bh, bl, el, hits, misses):  # noqa: E306
                print(f"iter {it}  b_hi {bh:.6g}  b_lo {bl:.6g}  gap {bl - bh:.3g}  "
                      f"{it / max(el, 1e-9):.0f} it/s  hits {hits} misses {misses}", flush=True)
        ck = None
        if resume is not None:
            ck = C.read_checkpoint(resume) if isinstance(resume, str) else resume
        kind, dev = cfg.device_kind()
        self.device_ = f"{kind}:{dev}" if kind == "cuda" else "cpu"
        t0 = time.perf_counter()
        if kind == "cuda" and rank_rows is None and self._use_shrink(p, n, d, dev, comm):
            shr = C.ShrinkingSolver(p, comm, dev)
            self.setup_info_ = shr.setup(X, ys)  # the whole-problem phases' solver; iteration "ws+shrinking"
            alpha, info = shr.solve(ck, progress)
            self.setup_info_["engine_note"] = f"{info['shrink_phases']} shrinking phases: {info['phase_log']}"
            self._solver = None
        elif kind == "cuda":
            solver = C.GpuSolver(p, comm, dev)
            self.setup_info_ = solver.setup(X, ys.shape[0], ys)
            alpha, info = solver.solve(ck, progress)
            self._solver = solver
        else:
            if rank_rows is not None:
                raise ValueError("partitioned X needs the GPU solver")
            alpha, info = C.solve_cpu(X, ys, p, comm, ck, progress)
            self._solver = None
        self.wall_time_ = time.perf_counter() - t0
        self.alpha_ = alpha
        self.b_ = float(info["b"])
        self.intercept_ = -self.b_
        self.n_iter_ = int(info["iters"])
        self.n_rounds_ = int(info.get("outer", 0))
        self.status_ = int(info["status"])
        self.converged_ = bool(info["converged"])
        self.fit_time_ = float(info["t_solve"])
        self.setup_time_ = float(info["t_setup"])
        self.stats_ = dict(info)
        if self.status_ == 2 and self.n_rounds_ > 0:
            import warnings

            warnings.warn(f"stopped at max_iter with gap {info['b_lo'] - info['b_hi']:.3g} > 2 eps: an unconverged "
                          "working-set model differs from the reference's pair-at-a-time iterate at the same cap; "
                          "raise max_iter to converge, or solver='smo' for the reference's trajectory (engines='all' "
                          "when the Gram is not resident)", RuntimeWarning, stacklevel=2)
        self.gamma_ = p.gamma
        self.n_features_in_ = d
        self._X_train, self._y_train = (X, ys) if rank_rows is None else (None, None)
        if rank_rows is None:
            self.support_ = np.nonzero(alpha > 0)[0]
            self.support_vectors_ = X[self.support_]
            self.dual_coef_ = (alpha[self.support_] * ys[self.support_]).astype(np.float32)
            self.n_support_ = int(len(self.support_))
        self._model = None
        self._gpu_pred = None
        return self

    # ------------------------------------------------------------------ model
    def to_model(self):
        C = load()
        if self._model is None:
            if self._X_train is None:
                raise RuntimeError("to_model() needs the full training set on this rank")
            self._model = C.make_model(self._X_train, self._y_train, self.alpha_, self.b_, self.gamma_)
        return self._model

    def save(self, path: str, precision: int = 9, legacy: bool = False) -> None:
        """Write the reference text model (gamma, b, then alpha,y,x... per SV)."""
        load().write_model(path, self.to_model(), precision, legacy)

    # ------------------------------------------------------------------ predict
    def _predictor(self):
        if self._gpu_pred is None:
            kind, dev = self.config.device_kind()
            if kind == "cuda":
                self._gpu_pred = load().GpuPredictor(self.to_model(), dev)
        return self._gpu_pred

    def decision_function(self, X) -> np.ndarray:
        """sum_sv alpha y K(sv, x) - b  (svmTrain.cu:646-652)."""
        X = _as_f32_2d(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, model has {self.n_features_in_}")
        gp = self._predictor()
        if gp is not None:
            return gp.decision(X)
        return load().decision_cpu(self.to_model(), X, 0)

    def predict(self, X) -> np.ndarray:
        dec = self.decision_function(X)
        return self._decode(np.where(dec < 0, -1.0, 1.0))  # d >= 0 -> +1 (svmTrain.cu:654-657)

    def score(self, X, y) -> float:
        yy = _as_1d(y)
        return float(np.mean(self.predict(X) == yy))

    def train_accuracy(self) -> float:
        """Training accuracy computed on device (distributed across ranks)."""
        if getattr(self, "_solver", None) is not None:
            return float(self._solver.train_accuracy(self.alpha_, self.b_))
        return self.score(self._X_train, self._y_train)

    def get_params(self, deep: bool = True) -> dict:
        return dataclasses.asdict(self.config)


class LoadedModel:
    """A model read from a reference-format file (svmTest path)."""

    def __init__(self, model, device: str = "auto"):
        self.model = model
        self.device = device
        self._gpu = None

    @property
    def gamma(self) -> float:
        return self.model.gamma

    @property
    def b(self) -> float:
        return self.model.b

    @property
    def n_support(self) -> int:
        return self.model.nsv

    def decision_function(self, X) -> np.ndarray:
        X = _as_f32_2d(X)
        use_gpu = self.device.startswith("cuda") or (self.device == "auto" and gpu_available())
        if use_gpu:
            if self._gpu is None:
                dev = int(self.device.split(":")[1]) if ":" in self.device else 0
                self._gpu = load().GpuPredictor(self.model, dev)
            return self._gpu.decision(X)
        return load().decision_cpu(self.model, X, 0)

    def predict(self, X) -> np.ndarray:
        return np.where(self.decision_function(X) < 0, -1.0, 1.0).astype(np.float32)

    def score(self, X, y) -> float:
        return float(np.mean(self.predict(X) == np.where(_as_1d(y) > 0, 1.0, -1.0)))


def load_model(path: str, device: str = "auto", legacy: bool = False) -> LoadedModel:
    return LoadedModel(load().read_model(path, legacy), device)
