"""torch-facing wrappers of the individual HIP kernels (device tensors in,
device tensors out).  Used by the GPU numerics tests, which compare each
kernel with a plain PyTorch fp32 reference of the same op, and usable as
building blocks (e.g. an RBF Gram / decision op on torch tensors).

Every wrapper raises if the native extension is missing: there is no silent
PyTorch fallback on a GPU box.
"""
from __future__ import annotations

import torch

from .._native import load, load_quarantine

STEP_ROWS = 128


def _pad_rows_cols(x: torch.Tensor, row_mult: int = 128, col_mult: int = 16, extra_rows: int = 128):
    n, d = x.shape
    dp = (d + col_mult - 1) // col_mult * col_mult
    rows = (n + row_mult - 1) // row_mult * row_mult + extra_rows
    out = torch.zeros(rows, dp, device=x.device, dtype=torch.float32)
    out[:n, :d] = x.to(torch.float32)
    return out, dp


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def row_sqnorm(x: torch.Tensor) -> torch.Tensor:
    """|x_i|^2 per row (one wave per row)."""
    C = load()
    xp, dp = _pad_rows_cols(x)
    out = torch.zeros(xp.shape[0], device=x.device, dtype=torch.float32)
    C.k_row_sqnorm(xp.data_ptr(), x.shape[0], dp, dp, out.data_ptr(), _stream(x))
    return out[: x.shape[0]]


def rbf_gram(a: torch.Tensor, b: torch.Tensor | None = None, gamma: float = 1.0, split: bool = False,
             cold_tau: float = 0.0) -> torch.Tensor:
    """Gram block K[i, j] = exp(-gamma |a_i - b_j|^2) with the dense-mode MFMA
    GEMM (32x32x2 f32, fused exp; split=True: fp16 MFMA over hi/lo split
    operands, rbf_gemm_split.hip).  b=None: the symmetric Gram of a, computed
    as upper-triangle tiles plus their mirrored transposes.  cold_tau > 0
    (split only): the adaptive Gram — one-product values where they are
    provably within cold_tau of the three-product ones (docs/DESIGN.md §13);
    gram_adapt_last() then reports its tile counts."""
    C = load()
    sym = b is None
    ap, dp = _pad_rows_cols(a)
    bp = ap if sym else _pad_rows_cols(b)[0]
    asq = torch.zeros(ap.shape[0], device=a.device)
    C.k_row_sqnorm(ap.data_ptr(), ap.shape[0], dp, dp, asq.data_ptr(), _stream(a))
    if sym:
        bsq = asq
    else:
        bsq = torch.zeros(bp.shape[0], device=a.device)
        C.k_row_sqnorm(bp.data_ptr(), bp.shape[0], dp, dp, bsq.data_ptr(), _stream(a))
    m = a.shape[0]
    n = m if sym else b.shape[0]
    ld = (n + 127) // 128 * 128
    out = torch.full((m, ld), float("nan"), device=a.device)
    if split:
        C.k_rbf_gram_split(ap.data_ptr(), asq.data_ptr(), m, bp.data_ptr(), bsq.data_ptr(), n, dp, float(gamma),
                           out.data_ptr(), ld, sym, _stream(a), float(cold_tau))
    else:
        if cold_tau:
            raise ValueError("cold_tau needs split=True")
        C.k_rbf_gram(ap.data_ptr(), asq.data_ptr(), m, bp.data_ptr(), bsq.data_ptr(), n, dp, float(gamma),
                     out.data_ptr(), ld, sym, _stream(a))
    return out[:, :n]


def gram_adapt_last() -> tuple[int, int]:
    """(one-product tiles, hot tiles recomputed) of this thread's last adaptive
    split Gram, or (-1, -1) when it was not adaptive."""
    return tuple(load().k_gram_adapt_last())


def rbf_rows(x: torch.Tensor, w: torch.Tensor, gamma: float) -> torch.Tensor:
    """K[q, j] = exp(-gamma |x_j - w_q|^2) for up to 16 query rows w (the
    smo_rows MFMA 16x16x4 kernel; quarantined pair-cache plugin)."""
    C = load()
    load_quarantine()
    nq = w.shape[0]
    if not 1 <= nq <= 16:
        raise ValueError("1 <= len(w) <= 16")
    xp, dp = _pad_rows_cols(x)
    wp, _ = _pad_rows_cols(w)
    xsq = torch.zeros(xp.shape[0], device=x.device)
    wsq = torch.zeros(wp.shape[0], device=x.device)
    C.k_row_sqnorm(xp.data_ptr(), xp.shape[0], dp, dp, xsq.data_ptr(), _stream(x))
    C.k_row_sqnorm(wp.data_ptr(), wp.shape[0], dp, dp, wsq.data_ptr(), _stream(x))
    n = x.shape[0]
    ld = (n + STEP_ROWS - 1) // STEP_ROWS * STEP_ROWS
    out = torch.zeros(nq, ld, device=x.device)
    C.k_rbf_rows(xp.data_ptr(), xsq.data_ptr(), n, dp, wp.data_ptr(), wsq.data_ptr(), nq, float(gamma),
                 out.data_ptr(), ld, _stream(x))
    return out[:, :n]


def select_partials(f: torch.Tensor, alpha: torch.Tensor, y: torch.Tensor, C_: float, offset: int = 0):
    """Per-workgroup packed (b_hi, I_hi) / (-b_lo, I_lo) keys of smo_step
    (quarantined pair-cache plugin)."""
    C = load()
    load_quarantine()
    n = f.shape[0]
    g = (n + STEP_ROWS - 1) // STEP_ROWS
    part = torch.zeros(2 * g, device=f.device, dtype=torch.int64)
    a_full = alpha.contiguous().float()
    blocks = C.k_select_partials(f.contiguous().float().data_ptr(), a_full.data_ptr(),
                                 y.contiguous().float().data_ptr(), n, offset, float(C_), part.data_ptr(),
                                 _stream(f))
    return part.view(-1, 2)[:blocks]


def decode_key(k: int):
    """(value, index) of a packed selection key (python int, may be negative i64)."""
    C = load()
    k &= (1 << 64) - 1
    return C.key_value(k), C.key_index(k)


def rbf_decision(x: torch.Tensor, sv: torch.Tensor, coef: torch.Tensor, gamma: float, b: float) -> torch.Tensor:
    """dec_i = sum_s coef_s exp(-gamma |x_i - sv_s|^2) - b (MFMA 32x32x2 GEMM +
    fused exp + row reduce)."""
    C = load()
    xp, dp = _pad_rows_cols(x)
    svp, _ = _pad_rows_cols(sv)
    xsq = torch.zeros(xp.shape[0], device=x.device)
    svsq = torch.zeros(svp.shape[0], device=x.device)
    cf = torch.zeros(svp.shape[0], device=x.device)
    cf[: coef.shape[0]] = coef.float()
    C.k_row_sqnorm(xp.data_ptr(), xp.shape[0], dp, dp, xsq.data_ptr(), _stream(x))
    C.k_row_sqnorm(svp.data_ptr(), svp.shape[0], dp, dp, svsq.data_ptr(), _stream(x))
    dec = torch.zeros(xp.shape[0], device=x.device)
    C.k_predict(xp.data_ptr(), xsq.data_ptr(), x.shape[0], dp, svp.data_ptr(), svsq.data_ptr(), cf.data_ptr(),
                sv.shape[0], float(gamma), float(b), dec.data_ptr(), _stream(x))
    return dec[: x.shape[0]]


def compact_positive(alpha: torch.Tensor) -> torch.Tensor:
    """Indices i with alpha_i > 0, in index order (ballot + scan kernels)."""
    C = load()
    a = alpha.contiguous().float()
    idx = torch.empty(a.shape[0] + 1, device=a.device, dtype=torch.int32)
    cnt = C.k_compact(a.data_ptr(), a.shape[0], idx.data_ptr(), _stream(a))
    return idx[:cnt]


def xpass_rows(x: torch.Tensor, keys, gamma: float, rows_per_group: int = 256) -> torch.Tensor:
    """The cache engines' X pass (xpass.hpp, v_mfma_f32_16x16x4_f32): rows
    K(x_keys[q], x_j) for up to 16 query rows, every workgroup filling its own
    rows_per_group-row segment of each line; quarantined pair-cache plugin)."""
    C = load()
    load_quarantine()
    keys = [int(k) for k in keys]
    if not 1 <= len(keys) <= 16:
        raise ValueError("1..16 query rows per X pass")
    n = x.shape[0]
    groups = (n + rows_per_group - 1) // rows_per_group
    span = groups * rows_per_group
    xp, dp = _pad_rows_cols(x, row_mult=rows_per_group)
    xsq = torch.zeros(xp.shape[0], device=x.device)
    C.k_row_sqnorm(xp.data_ptr(), xp.shape[0], dp, dp, xsq.data_ptr(), _stream(x))
    kd = torch.tensor(keys, dtype=torch.int32, device=x.device)
    out = torch.full((len(keys), span), float("nan"), device=x.device)
    C.k_xpass_rows(xp.data_ptr(), xsq.data_ptr(), n, dp, kd.data_ptr(), len(keys), float(gamma), out.data_ptr(),
                   span, rows_per_group, _stream(x))
    return out[:, :n]


def rbf_rows_indexed(x: torch.Tensor, rows, gamma: float, out_lines=None, n_lines: int = 0,
                     split: bool = False) -> torch.Tensor:
    """The working-set cache engine's row GEMM (rbf_gemm EPI_ROWS: A rows by
    index, output rows to their lines, M read on the device): lines
    [n_lines][n] with line out_lines[i] = K(x_rows[i], x_j).  split=True: the
    fp16 split-operand kernel (rbf_gemm_split.hip)."""
    C = load()
    rows = [int(r) for r in rows]
    m = len(rows)
    n = x.shape[0]
    xp, dp = _pad_rows_cols(x, row_mult=512)  # the GEMM reads whole 512-column tiles
    xsq = torch.zeros(xp.shape[0], device=x.device)
    C.k_row_sqnorm(xp.data_ptr(), xp.shape[0], dp, dp, xsq.data_ptr(), _stream(x))
    out_lines = list(range(m)) if out_lines is None else [int(v) for v in out_lines]
    n_lines = max(n_lines, max(out_lines) + 1 if out_lines else 1)
    rd = torch.tensor(rows or [0], dtype=torch.int32, device=x.device)
    od = torch.tensor(out_lines or [0], dtype=torch.int32, device=x.device)
    ld = (n + 127) // 128 * 128
    out = torch.full((n_lines, ld), float("nan"), device=x.device)
    C.k_rbf_rows_indexed(xp.data_ptr(), xsq.data_ptr(), n, dp, rd.data_ptr(), m, float(gamma), out.data_ptr(), ld,
                         od.data_ptr(), _stream(x), bool(split))
    return out[:, :n]


KEY_NONE = (1 << 64) - 1
WS_CAND = 16  # candidates per side per selection workgroup (device_state.hpp kWsCand)


def ws_merge_multi(cand, blocks: int, q_max: int, n_new: int, eps: float, prev_union=(), p_act: int | None = None,
                   iteration: int = 0, max_iter: int = 1 << 40) -> dict:
    """One launch of the multi-block merge (ws_*.hip ws_merge_multi_kernel) on
    crafted candidate lists ``cand`` [G][2][WS_CAND] (u64 keys, up then low; KEY_NONE
    for empty slots) and a previous union (newest first).  Returns the new
    union, the [blocks][q_max] block layout (-1 unused), rows per block, the
    global b_hi / b_lo and the stop code (0 running, 1 converged)."""
    import numpy as np

    c = np.ascontiguousarray(np.asarray(cand, dtype=np.uint64).reshape(-1, 2, WS_CAND))
    prev = np.asarray(list(prev_union), dtype=np.int32)
    return load().k_ws_merge_multi(c.reshape(-1), c.shape[0], blocks, blocks if p_act is None else p_act, q_max,
                                   n_new, float(eps), prev, int(iteration), int(max_iter))


def ws_solve(K, f, alpha, y, qb, q_max: int, C_: float, clip: str = "independent", eps: float = 1e-3,
             rel: float = 0.3, eps_floor: float = 3e-4, tau: float = 1e-12, b_hi: float = 0.0, b_lo: float = 0.0,
             inner_max: int = 768, p_round: int | None = None, iteration: int = 0, max_iter: int = 1 << 40,
             wss: int = 1) -> dict:
    """One launch of the sub-problem solver (ws_solve_kernel): P = len(qb)
    blocks, block p with qb[p] rows, sub-Gram K[p] ([q_max][q_max]) and f /
    alpha / y [p][q_max]; b_hi / b_lo = the round's global selection (the local
    tolerance is max(eps_floor, rel (b_lo - b_hi) / 2)).  P > 1 runs the
    multi-block kernel (p_round active blocks share max_iter).  wss: 1 the
    reference's first-order pair choice, 2 second order (WSS2)."""
    import numpy as np

    P = len(qb)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float32)).reshape(-1)  # noqa: E731
    return load().k_ws_solve(f32(K), f32(f), f32(alpha), f32(y), np.asarray(qb, dtype=np.int32), q_max, P,
                             P if p_round is None else p_round, float(C_), 1 if clip == "box" else 0, float(eps),
                             float(rel), float(eps_floor), float(tau), float(b_hi), float(b_lo), int(inner_max),
                             int(iteration), int(max_iter), int(wss))


def ws_select(gram, f, alpha, y, dalpha, apply_lines, apply_coef, nab, C_: float, q_max: int = 192,
              p_round: int | None = None, p_act: int | None = None, outer: int = 1, ks: int = 0,
              wide: bool = False) -> dict:
    """The working-set f update + candidate selection (ws_select_kernel) on a
    dense gram [L][ldg >= n] (rows = lines).  len(nab) == 1: the one-pass
    kernel; more blocks: pass 1 (d_f, d'Qd / g'd partials) and pass 2 (line
    search t, f += t d_f, alpha = alpha_new - (1 - t) d_alpha, candidates).
    ks > 1: pass 1 split into ks list slices per selection group (dfs then
    holds slice 0, part [G][ks][2]).  wide: the wide pass 1 (1024-column
    groups, 16-B row loads; part [p1G][ks][2])."""
    import numpy as np

    g = np.ascontiguousarray(np.asarray(gram, dtype=np.float32))
    P = len(nab)
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float32)).reshape(-1)  # noqa: E731
    return load().k_ws_select(g.reshape(-1), g.shape[0], g.shape[1], f32(f), f32(alpha), f32(y), f32(dalpha),
                              np.asarray(apply_lines, dtype=np.int32), f32(apply_coef), np.asarray(nab, dtype=np.int32),
                              P, P if p_round is None else p_round, P if p_act is None else p_act, q_max, float(C_),
                              int(outer), ks=int(ks), wide=bool(wide))


def fused_select(f: torch.Tensor, alpha: torch.Tensor, y: torch.Tensor, C_: float, rows_per_group: int = 256):
    """Per-workgroup (up, low) selection keys of the fused / persistent engines
    (classification + wave-64 DPP minimum + LDS across waves): [groups, 2] u64
    (as int64 tensor; decode with decode_key)."""
    C = load()
    n = f.shape[0]
    groups = (n + rows_per_group - 1) // rows_per_group
    pad = groups * rows_per_group + 256

    def padded(t, fill):
        o = torch.full((pad,), fill, device=f.device, dtype=torch.float32)
        o[:n] = t.to(torch.float32)
        return o

    fp, ap, yp = padded(f, 0.0), padded(alpha, 0.0), padded(y, 1.0)
    out = torch.zeros(2 * groups + 2, dtype=torch.int64, device=f.device)
    C.k_fused_select(fp.data_ptr(), ap.data_ptr(), yp.data_ptr(), n, float(C_), rows_per_group, out.data_ptr(),
                     _stream(f))
    return out[: 2 * groups].view(groups, 2)


def split_rows(x: torch.Tensor, rows: int, dp: int, ldx: int | None = None):
    """The split GEMMs' operand preparation (split_rows_kernel): per row a
    power-of-two shift s (largest |x| into [2^14, 2^15)) and the fp16 planes
    h = fp16(x 2^s), l = fp16(x 2^s - h), laid out as ceil(dp / 32) blocks of
    32 h then 32 l values.  ``x``: a flat float32 CUDA tensor holding the rows at
    stride ``ldx`` >= dp, columns d .. dp - 1 zero (any stride / offset: the
    kernel's 16-B path needs ldx % 4 == 0 and an aligned base, else it reads
    element by element).  Returns
    (planes [rows, blocks, 2, 32] float16, shift [rows] int32)."""
    C = load()
    ldx = ldx or dp
    if ldx < dp or x.numel() < (rows - 1) * ldx + dp:
        raise ValueError("split_rows: need ldx >= dp and (rows - 1) * ldx + dp elements")
    nkb = (dp + 31) // 32
    planes = torch.zeros(rows * nkb * 64, device=x.device, dtype=torch.float16)
    shift = torch.zeros(rows, device=x.device, dtype=torch.int32)
    C.k_split_rows(x.data_ptr(), rows, dp, ldx, planes.data_ptr(), shift.data_ptr(), _stream(x))
    torch.cuda.synchronize(x.device)
    return planes.view(rows, nkb, 2, 32), shift
