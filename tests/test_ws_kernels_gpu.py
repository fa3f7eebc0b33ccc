"""Kernel-level tests of the working-set engine (ws_*.hip): each kernel runs
once on crafted state (dpsvm_amd.ops.kernels.ws_*) and is checked against a
numpy model of the same rule — the merge (sort, stop test, union with
first-position-wins deduplication, previous-union retention, block
assignment), the one-wave LDS pair loop (the reference's pair rule
svmTrainMain.cpp:255-299 in both clipping modes, eta floor), and the two-pass
f update with the line search (d_f, d'Qd, g'd, t, f, alpha, candidates).
The end-to-end solves (tests/test_ws_gpu.py) cannot tell which kernel a
compensating bug sits in; these can."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NONE = np.uint64((1 << 64) - 1)
KC = 16  # candidates per side per selection workgroup (device_state.hpp kWsCand)
KC1 = 4  # ... produced for (and read by) the one-block rounds (kWsCand1)


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dpsvm_amd.ops import kernels

    return kernels


# ---------------------------------------------------------------- key model (common.hpp)
def f32_order(f):
    u = np.asarray(f, dtype=np.float32).reshape(-1).view(np.uint32).copy()
    u[u == 0x80000000] = 0
    neg = (u & np.uint32(0x80000000)) != 0
    return np.where(neg, ~u, u | np.uint32(0x80000000)).astype(np.uint32)


def make_key(f, idx):
    return (f32_order(f).astype(np.uint64) << np.uint64(32)) | np.asarray(idx, dtype=np.uint64).reshape(-1)


def key_value(k):
    o = (np.asarray(k, dtype=np.uint64) >> np.uint64(32)).astype(np.uint32)
    u = np.where(o & np.uint32(0x80000000), o & np.uint32(0x7FFFFFFF), ~o).astype(np.uint32)
    return u.view(np.float32)


def in_up(a, y, C):
    a, y = np.asarray(a, np.float32), np.asarray(y, np.float32)
    return np.where(a == 0, y == 1, np.where(a == np.float32(C), y != 1, True))


def in_low(a, y, C):
    a, y = np.asarray(a, np.float32), np.asarray(y, np.float32)
    return np.where(a == 0, y != 1, np.where(a == np.float32(C), y == 1, True))


# ---------------------------------------------------------------- merge
def merge_model(cand, blocks, p_act, q_max, n_new, eps, prev):
    c = np.asarray(cand, dtype=np.uint64).reshape(-1, 2, KC)
    up, low = np.sort(c[:, 0, :].ravel()), np.sort(c[:, 1, :].ravel())
    b_hi, b_lo = key_value(up[0])[()], -key_value(low[0])[()]
    if up[0] == NONE or low[0] == NONE:
        return dict(done=3)
    if not (np.float32(b_lo) > np.float32(b_hi) + np.float32(2.0) * np.float32(eps)):
        return dict(done=1, b_hi=b_hi, b_lo=b_lo)
    P = max(1, min(p_act, blocks))
    qmax = P * q_max
    want = qmax if len(prev) == 0 else min(P * n_new, qmax)
    half = (want + 1) // 2
    chosen, seen = [], set()
    for r in range(half):
        for side in (up, low):
            k = side[r] if r < len(side) else NONE
            if k == NONE:
                continue
            row = int(k & np.uint64(0xFFFFFFFF))
            if row not in seen:
                seen.add(row)
                chosen.append(row)
    union = chosen[:want]
    if len(union) < qmax:
        cs = set(union)
        union += [int(r) for r in prev if int(r) not in cs][: qmax - len(union)]
    idx = -np.ones((blocks, q_max), dtype=np.int64)
    qb = np.zeros(blocks, dtype=np.int64)
    for u, row in enumerate(union):
        pi = u // 2
        b, la = pi % P, 2 * (pi // P) + (u & 1)
        idx[b, la] = row
        qb[b] = max(qb[b], la + 1)
    return dict(done=0, b_hi=b_hi, b_lo=b_lo, uidx=union, idx=idx, qb=qb, P=P)


def crafted_candidates(rng, G, n_rows, ties=True):
    """G lists of up to KC keys per side: rows are free (both sides), up-only or
    low-only; several rows share f values (ties break by index)."""
    rows = rng.choice(200000, size=n_rows, replace=False)
    f = rng.normal(size=n_rows).astype(np.float32)
    if ties:
        f[: n_rows // 10] = f[0]
    kind = rng.integers(0, 3, size=n_rows)  # 0 free, 1 up only, 2 low only
    owner = rng.integers(0, G, size=n_rows)
    cand = np.full((G, 2, KC), NONE, dtype=np.uint64)
    for g in range(G):
        sel = np.nonzero(owner == g)[0]
        ups = np.sort(make_key(f[sel][kind[sel] != 2], rows[sel][kind[sel] != 2]))[:KC]
        lows = np.sort(make_key(-f[sel][kind[sel] != 1], rows[sel][kind[sel] != 1]))[:KC]
        cand[g, 0, : len(ups)] = ups
        cand[g, 1, : len(lows)] = lows
    return cand, rows


@pytest.mark.parametrize("G,blocks,p_act,n_prev,n_new", [(256, 8, 8, 0, 192), (256, 8, 4, 300, 96),
                                                        (37, 8, 8, 1000, 192), (200, 4, 1, 150, 144),
                                                        (256, 2, 2, 64, 40), (256, 32, 32, 0, 96),
                                                        (256, 32, 16, 2500, 48), (240, 16, 16, 900, 96),
                                                        (256, 128, 128, 0, 48), (256, 128, 64, 4000, 24),
                                                        (235, 128, 128, 6000, 48)])
def test_ws_merge_multi_matches_model(K, G, blocks, p_act, n_prev, n_new):
    """128 x 48: the 6,144-row union (3,072 ranks a side over 4,096 keys, hash
    tables three-quarters full)."""
    rng = np.random.default_rng(G * 31 + blocks + p_act + n_prev)
    q_max = 192 if blocks == 8 else 48 if blocks > 64 else 96
    cand, rows = crafted_candidates(rng, G, 3000 if blocks <= 8 else 12000 if blocks <= 64 else 30000)
    # previous union: half of it rows the merge picks again (dropped from the
    # retained tail), half rows it does not
    prev = np.concatenate([rng.choice(rows, size=n_prev // 2, replace=False),
                           rng.choice(np.arange(300000, 400000), size=n_prev - n_prev // 2, replace=False)])
    prev = list(dict.fromkeys(int(v) for v in prev))[: blocks * q_max]
    got = K.ws_merge_multi(cand, blocks, q_max, n_new, 1e-3, prev, p_act=p_act)
    ref = merge_model(cand, blocks, p_act, q_max, n_new, 1e-3, prev)
    assert got["done"] == 0 == ref["done"]
    assert got["b_hi"] == ref["b_hi"] and got["b_lo"] == ref["b_lo"]
    assert got["p_round"] == ref["P"]
    assert got["uidx"] == ref["uidx"]
    assert len(set(got["uidx"])) == len(got["uidx"])  # no row twice
    assert list(got["qb"]) == list(ref["qb"])
    assert np.array_equal(np.asarray(got["idx"]).reshape(blocks, q_max), ref["idx"])
    # block 0 holds the global extremes (the maximal violating pair: progress)
    up0 = int(np.sort(cand[:, 0, :].ravel())[0] & np.uint64(0xFFFFFFFF))
    assert got["idx"][0] == up0


def test_ws_merge_multi_stop_test_and_empty_side(K):
    rng = np.random.default_rng(5)
    cand, _ = crafted_candidates(rng, 16, 200, ties=False)
    up_min = key_value(np.sort(cand[:, 0, :].ravel())[0])[()]
    # every low key at -(b_hi + eps): b_lo = b_hi + eps <= b_hi + 2 eps -> converged
    low = make_key(np.full(16 * KC, -(up_min + np.float32(1e-3)), dtype=np.float32),
                   np.arange(10**6, 10**6 + 16 * KC))
    c2 = cand.copy()
    c2[:, 1, :] = np.sort(low).reshape(16, KC)
    got = K.ws_merge_multi(c2, 8, 192, 192, 1e-3)
    assert got["done"] == 1 and got["b_hi"] == up_min
    c3 = cand.copy()
    c3[:, 1, :] = NONE  # I_low empty: no pair
    assert K.ws_merge_multi(c3, 8, 192, 192, 1e-3)["done"] == 3
    assert K.ws_merge_multi(cand, 8, 192, 192, 1e-3, iteration=50, max_iter=50)["done"] == 2


# ---------------------------------------------------------------- solve
def pair_step_model(a_hi, a_lo, y_hi, y_lo, bh, bl, khl, C, tau, box, same):
    f32 = np.float32
    eta = f32(2.0) - f32(2.0) * f32(khl)
    eta = eta if eta >= f32(tau) else f32(tau)
    s = f32(y_lo * y_hi)
    a_lo_new = f32(a_lo + f32(f32(y_lo * f32(bh - bl)) / eta))
    clipped = False
    if box and not same:
        if y_hi != y_lo:
            dl = f32(a_lo - a_hi)
            L, hL = (dl, f32(0)) if dl > 0 else (f32(0), f32(-1))
            H, hH = (f32(C + dl), f32(C)) if f32(C + dl) < C else (f32(C), f32(-1))
        else:
            sm = f32(a_lo + a_hi)
            L, hL = (f32(sm - C), f32(C)) if f32(sm - C) > 0 else (f32(0), f32(-1))
            H, hH = (sm, f32(0)) if sm < C else (f32(C), f32(-1))
        atL = a_lo_new <= L
        atH = (not atL) and a_lo_new >= H
        a_lo_new = L if atL else (H if atH else a_lo_new)
        snap = hL if atL else (hH if atH else f32(-1))
        a_hi_new = snap if snap >= 0 else f32(a_hi + f32(s * f32(a_lo - a_lo_new)))
        a_hi_new = f32(min(max(a_hi_new, 0), C))
    else:
        a_hi_new = f32(a_hi + f32(s * f32(a_lo - a_lo_new)))
        lo_raw, hi_raw = a_lo_new, a_hi_new
        a_lo_new = f32(min(max(a_lo_new, 0), C))
        a_hi_new = f32(min(max(a_hi_new, 0), C))
        clipped = lo_raw != a_lo_new or hi_raw != a_hi_new
    return a_hi_new, a_lo_new, f32(f32(a_hi_new - a_hi) * y_hi), f32(f32(a_lo_new - a_lo) * y_lo), clipped


def solve_model(Kq, f, a, y, C, box, eps_in, tau, cap, w2=False):
    """the ws_solve loop in float32 (IEEE division where the kernel uses a
    refined v_rcp: results agree to ~1 ulp per step).  w2: the low row by the
    second-order gain (f_lo - b_hi)^2 / eta(hi, lo) (WSS2)."""
    f32 = np.float32
    Kq = Kq.astype(np.float32)
    a = a.astype(np.float32).copy()
    y = y.astype(np.float32)
    fu = np.where(in_up(a, y, C), f, np.inf).astype(np.float32)
    fl = np.where(in_low(a, y, C), -f, np.inf).astype(np.float32)
    steps, clipped_any = 0, False
    while steps < cap:
        mu, ml = fu.min(), fl.min()
        bh, bl = mu, f32(-ml)
        if not (mu < np.inf and ml < np.inf and bl > f32(bh + f32(f32(2.0) * f32(eps_in)))):
            break
        ph, pl = int(np.argmin(fu)), int(np.argmin(fl))
        if w2:
            dv = (-fl - bh).astype(np.float32)
            eta = np.maximum(np.float32(2.0) - np.float32(2.0) * Kq[ph, :], np.float32(tau)).astype(np.float32)
            g = np.where(np.isfinite(fl) & (dv > 0), -(dv * dv) / eta, np.inf)
            pl = int(np.argmin(g))
            bl = f32(-fl[pl])
        a_hi_new, a_lo_new, c_hi, c_lo, cl = pair_step_model(a[ph], a[pl], y[ph], y[pl], bh, bl, Kq[ph, pl], C, tau,
                                                             box, ph == pl)
        clipped_any |= cl
        dl = (c_hi * Kq[ph, :]).astype(np.float32) + (c_lo * Kq[pl, :]).astype(np.float32)
        fu = (fu + dl).astype(np.float32)
        fl = (fl - dl).astype(np.float32)
        f_lo_new = f32(bl + f32(f32(c_hi * Kq[ph, pl]) + f32(c_lo * Kq[pl, pl])))
        f_hi_new = f32(bh + f32(f32(c_hi * Kq[ph, ph]) + f32(c_lo * Kq[pl, ph])))
        for pos, an, fp in ((pl, a_lo_new, f_lo_new), (ph, a_hi_new, f_hi_new)):  # hi placed last
            fu[pos] = fp if in_up(an, y[pos], C) else np.inf
            fl[pos] = -fp if in_low(an, y[pos], C) else np.inf
        a[pl] = a_lo_new
        a[ph] = a_hi_new
        steps += 1
    return a, steps, clipped_any


def sub_problem(rng, q, C, d=6, gamma=0.7, dup=False):
    X = rng.normal(size=(q, d)).astype(np.float32)
    if dup:
        X[1] = X[0]  # K(0, 1) = 1: eta = 0 -> the tau floor
    d2 = ((X[:, None, :].astype(np.float64) - X[None, :, :]) ** 2).sum(-1)
    Kq = np.exp(-gamma * d2).astype(np.float32)
    np.fill_diagonal(Kq, 1.0)
    y = np.where(rng.random(q) < 0.5, 1.0, -1.0).astype(np.float32)
    a = rng.uniform(0, C, size=q).astype(np.float32)
    a[rng.random(q) < 0.3] = 0.0
    a[rng.random(q) < 0.15] = np.float32(C)
    f = (Kq.astype(np.float64) @ (a * y) - y + rng.normal(scale=0.3, size=q)).astype(np.float32)
    return Kq, f, a, y


def padded_block(Kq, f, a, y, q_max):
    q = len(f)
    Kp = np.zeros((q_max, q_max), np.float32)
    Kp[:q, :q] = Kq
    pad = lambda v, fill: np.concatenate([v, np.full(q_max - q, fill, np.float32)])  # noqa: E731
    return Kp, pad(f, 0), pad(a, 0), pad(y, 1)


def extremes(f, a, y, C):
    up, lo = in_up(a, y, C), in_low(a, y, C)
    return np.float32(f[up].min()), np.float32(f[lo].max())


@pytest.mark.parametrize("clip", ["independent", "box"])
@pytest.mark.parametrize("q,q_max,dup", [(150, 192, False), (64, 192, True), (40, 40, False), (192, 192, False)])
def test_ws_solve_matches_pair_rule_model(K, clip, q, q_max, dup):
    rng = np.random.default_rng(q * 3 + q_max + (7 if dup else 0) + (1 if clip == "box" else 0))
    C = 2.0
    Kq, f, a, y = sub_problem(rng, q, C, dup=dup)
    bh, bl = extremes(f, a, y, C)
    eps, rel = 1e-3, 0.3
    eps_floor = np.float32(rel * eps)
    eps_in = max(eps_floor, np.float32(np.float32(rel * np.float32(0.5)) * np.float32(bl - bh)))
    Kp, fp, ap, yp = padded_block(Kq, f, a, y, q_max)
    box = clip == "box"
    # the first steps exactly (a step is ~1 ulp from the model's IEEE division)
    for cap in (1, 3, 8):
        got = K.ws_solve(Kp, fp, ap, yp, [q], q_max, C, clip=clip, eps=eps, rel=rel, eps_floor=eps_floor,
                         b_hi=bh, b_lo=bl, inner_max=cap)
        ref_a, ref_steps, _ = solve_model(Kq, f, a, y, C, box, eps_in, 1e-12, cap)
        assert got["steps"] == [ref_steps] and got["iter"] == ref_steps
        np.testing.assert_allclose(got["alpha"][:q], ref_a, rtol=2e-6, atol=2e-6 * C)
    # to the sub-problem's tolerance (ulp-level differences may steer the two
    # trajectories apart near ties: same stop rule, similar length)
    got = K.ws_solve(Kp, fp, ap, yp, [q], q_max, C, clip=clip, eps=eps, rel=rel, eps_floor=eps_floor,
                     b_hi=bh, b_lo=bl, inner_max=4 * q_max)
    _, ref_steps, _ = solve_model(Kq, f, a, y, C, box, eps_in, 1e-12, 4 * q_max)
    an = got["alpha"][:q]
    assert np.all((an >= 0) & (an <= C))
    assert abs(got["steps"][0] - ref_steps) <= max(3, ref_steps // 5)
    # the apply list: exactly the rows whose alpha changed, in position order, coef = d_alpha y
    ch = np.nonzero(an != a)[0]
    assert got["apply_idx"] == ch.tolist()
    np.testing.assert_array_equal(got["apply_coef"], ((an[ch] - a[ch]) * y[ch]).astype(np.float32))
    if box:  # the joint box keeps sum(alpha y)
        assert abs(float(np.sum((an.astype(np.float64) - a) * y))) < 1e-4 * C * q
    # the sub-problem's stop test holds on the exact (float64) sub-gradient
    fn = f + Kq.astype(np.float64) @ ((an.astype(np.float64) - a) * y)
    if got["steps"][0] < 4 * q_max:
        bh2, bl2 = extremes(fn, an, y, C)
        assert bl2 <= bh2 + 2 * eps_in + 1e-4


def test_ws_solve_multi_block_matches_single_blocks_and_shares_max_iter(K):
    rng = np.random.default_rng(17)
    C, q_max = 1.5, 96
    blocks = []
    for q in (96, 50, 70):
        blocks.append(sub_problem(rng, q, C))
    # the global selection: over all blocks
    fa = np.concatenate([b[1] for b in blocks])
    aa = np.concatenate([b[2] for b in blocks])
    ya = np.concatenate([b[3] for b in blocks])
    bh, bl = extremes(fa, aa, ya, C)
    kw = dict(clip="box", eps=1e-3, rel=0.3, eps_floor=3e-4, b_hi=bh, b_lo=bl, inner_max=400)
    pads = [padded_block(*b, q_max) for b in blocks]
    Kall = np.stack([p[0] for p in pads])
    cat = lambda i: np.concatenate([p[i] for p in pads])  # noqa: E731
    qb = [len(b[1]) for b in blocks]
    got = K.ws_solve(Kall, cat(1), cat(2), cat(3), qb, q_max, C, **kw)
    for p, (Kq, f, a, y) in enumerate(blocks):
        one = K.ws_solve(pads[p][0], pads[p][1], pads[p][2], pads[p][3], [len(f)], q_max, C, **kw)
        # the same arithmetic on the same block: bit-identical
        assert got["steps"][p] == one["steps"][0]
        np.testing.assert_array_equal(got["alpha"][p * q_max:p * q_max + len(f)], one["alpha"][:len(f)])
    assert got["iter"] == sum(got["steps"]) and got["outer"] == 1 and got["done"] == 0
    # only p_round = 2 of the 3 blocks active: block 2 takes no step
    two = K.ws_solve(Kall, cat(1), cat(2), cat(3), qb, q_max, C, p_round=2, **kw)
    assert two["steps"][2] == 0 and two["steps"][:2] == got["steps"][:2]
    # max_iter shared: 10 steps over 3 blocks -> 4 / 3 / 3
    capped = K.ws_solve(Kall, cat(1), cat(2), cat(3), qb, q_max, C, max_iter=10, **kw)
    assert capped["steps"] == [4, 3, 3] and capped["done"] == 2


def test_ws_solve_independent_clip_event_drops_to_one_block(K):
    rng = np.random.default_rng(23)
    C, q_max = 1.0, 64
    blocks = [sub_problem(rng, 64, C), sub_problem(rng, 64, C)]
    pads = [padded_block(*b, q_max) for b in blocks]
    cat = lambda i: np.concatenate([p[i] for p in pads])  # noqa: E731
    fa, aa, ya = cat(1), cat(2), cat(3)
    bh, bl = extremes(fa, aa, ya, C)
    got = K.ws_solve(np.stack([p[0] for p in pads]), fa, aa, ya, [64, 64], q_max, C, clip="independent",
                     b_hi=bh, b_lo=bl)
    # random states at the box edges clip immediately: sum(alpha y) broken -> one block from now on
    assert got["p_act"] == 1 and got["p1_round"] == 1
    box = K.ws_solve(np.stack([p[0] for p in pads]), fa, aa, ya, [64, 64], q_max, C, clip="box", b_hi=bh, b_lo=bl)
    assert box["p_act"] == 2 and box["p1_round"] == 0


# ---------------------------------------------------------------- select (f update + line search)
def rbf(X, gamma):
    d2 = ((X[:, None, :].astype(np.float64) - X[None, :, :]) ** 2).sum(-1)
    return np.exp(-gamma * d2)


def candidates_model(f, a, y, C, G, rpt, nc=KC):
    out = np.full((G, 2, nc), NONE, dtype=np.uint64)
    n = len(f)
    for b in range(G):
        lo, hi = b * rpt * 256, min(n, (b + 1) * rpt * 256)
        j = np.arange(lo, hi)
        if len(j) == 0:
            continue
        u = np.sort(make_key(f[j][in_up(a[j], y[j], C)], j[in_up(a[j], y[j], C)]))[:nc]
        l_ = np.sort(make_key(-f[j][in_low(a[j], y[j], C)], j[in_low(a[j], y[j], C)]))[:nc]
        out[b, 0, : len(u)] = u
        out[b, 1, : len(l_)] = l_
    return out


def select_state(rng, n, C, n_changed, gamma=0.3):
    X = rng.normal(size=(n, 5)).astype(np.float32)
    gram = rbf(X, gamma).astype(np.float32)
    y = np.where(rng.random(n) < 0.5, 1.0, -1.0).astype(np.float32)
    a_old = rng.uniform(0, C, n).astype(np.float32)
    a_old[rng.random(n) < 0.4] = 0.0
    ch = rng.choice(n, size=n_changed, replace=False)
    a_new = a_old.copy()
    a_new[ch] = np.clip(a_old[ch] + rng.normal(scale=0.3 * C, size=n_changed), 0, C).astype(np.float32)
    a_new[ch[: n_changed // 4]] = np.float32(C)  # steps that end on a bound
    dal = np.zeros(n, np.float32)
    dal[ch] = a_new[ch] - a_old[ch]
    f = rng.normal(size=n).astype(np.float32)
    return gram, f, a_new, y, dal, ch


def line_search_rule(q, g, P):
    if P <= 1:
        return np.float32(1.0)
    if not g > 0:
        return np.float32(0.0)
    if not q > g:
        return np.float32(1.0)
    t = np.float32(g / q)
    return np.float32(1.0) if t >= np.float32(0.9) else t


@pytest.mark.parametrize("target,P,p_act", [(0.5, 4, 4), (0.95, 4, 4), (-1.0, 2, 2), (0.3, 2, 2), (0.5, 1, 1),
                                            (0.4, 4, 1)])
def test_ws_select_two_pass_line_search_matches_model(K, target, P, p_act):
    """target = the line-search factor g'd / d'Qd the state is built for
    (negative: g'd < 0, no ascent)."""
    rng = np.random.default_rng(int(abs(target) * 100) + P)
    n, C, q_max = 3000, 2.0, 96
    gram, f, a_new, y, dal, ch = select_state(rng, n, C, min(P, 4) * 40)
    c = (dal.astype(np.float64) * y)
    d_f = gram.astype(np.float64).T @ c  # gram is symmetric: rows = lines
    q = float(np.sum(c[ch] * d_f[ch]))
    # steer g'd = -sum c_j f_j to target * q through one changed row's f
    j0 = ch[int(np.argmax(np.abs(c[ch])))]
    rest = ch[ch != j0]
    g_rest = -float(np.sum(c[rest] * f[rest]))
    f[j0] = np.float32((target * q - g_rest) / -c[j0])
    g = -float(np.sum(c[ch] * f.astype(np.float64)[ch]))
    nab = [len(ch) // P + (1 if p < len(ch) % P else 0) for p in range(P)] if P > 1 else [len(ch)]
    order = ch  # apply rows block by block (lines = rows: the resident Gram)
    if P == 1:
        nab = nab + [0]  # a one-block round through the two-pass kernels (the multi engine at p = 1)
    got = K.ws_select(gram, f, a_new, y, dal, order, c[order].astype(np.float32), nab, C, q_max=q_max,
                      p_round=P, p_act=p_act)
    G, rpt = got["G"], got["rpt"]
    np.testing.assert_allclose(got["dfs"], d_f, rtol=1e-4, atol=2e-5)
    part = np.asarray(got["part"]).reshape(G, 2)
    qk, gk = part[:, 0].sum(), part[:, 1].sum()
    # the partials: d'Qd over the kernel's own d_f, g'd over f (float64 sums)
    assert qk == pytest.approx(float(np.sum(c[ch] * got["dfs"].astype(np.float64)[ch])), rel=1e-9)
    assert gk == pytest.approx(g, rel=1e-6, abs=1e-9)
    t = line_search_rule(qk, gk, P)
    assert got["t"] == pytest.approx(float(t), rel=1e-6)
    t = np.float32(got["t"])
    want_f = (f + (got["dfs"] if t == 1 else t * got["dfs"])).astype(np.float32)
    np.testing.assert_array_equal(got["f"], want_f)
    if t < 1:
        want_a = a_new.copy()
        want_a[ch] = np.clip(a_new[ch] - np.float32(np.float32(1.0) - t) * dal[ch], 0, C).astype(np.float32)
    else:
        want_a = a_new  # full step: alphas on a bound stay exactly there
    # alpha_new - (1 - t) d_alpha may compile to one fused multiply-add: a few ulp
    np.testing.assert_allclose(got["alpha"], want_a, rtol=1e-6, atol=1e-7 * C)
    if t == 1:
        np.testing.assert_array_equal(got["alpha"], want_a)
    assert not np.any(got["dalpha"])
    # blocks: halved after a damped round (never below the clip fallback's 1)
    damped = t < 1
    assert got["n_damped"] == int(damped)
    assert got["p_act"] == (min(p_act, max(1, P // 2)) if damped else p_act)
    assert got["p1_round"] == (1 if damped and got["p_act"] == 1 else 0)
    cand = np.asarray(got["cand"], dtype=np.uint64).reshape(G, 2, KC)  # multi-block kernels: KC per side
    np.testing.assert_array_equal(cand, candidates_model(got["f"], got["alpha"], y, C, G, rpt))


@pytest.mark.parametrize("ks", [2, 5])
def test_ws_select_pass1_list_slices_match_model(K, ks):
    """Pass 1 split into ks slices of the changed-row list per selection group
    (ws_pass1_splits: a rank's shard of a sharded run has few groups): the
    partials still sum to d'Qd and g'd, pass 2 sums the slices' changes, and f
    after the round matches the model and the one-slice kernel."""
    rng = np.random.default_rng(40 + ks)
    n, C, q_max, P = 3000, 2.0, 96, 4
    gram, f, a_new, y, dal, ch = select_state(rng, n, C, 160)
    c = dal.astype(np.float64) * y
    d_f = gram.astype(np.float64).T @ c
    q = float(np.sum(c[ch] * d_f[ch]))
    g = -float(np.sum(c[ch] * f.astype(np.float64)[ch]))
    nab = [40] * P
    kw = dict(q_max=q_max)
    got = K.ws_select(gram, f, a_new, y, dal, ch, c[ch].astype(np.float32), nab, C, ks=ks, **kw)
    one = K.ws_select(gram, f, a_new, y, dal, ch, c[ch].astype(np.float32), nab, C, ks=1, **kw)
    part = np.asarray(got["part"]).reshape(got["G"] * ks, 2)
    assert part[:, 0].sum() == pytest.approx(q, rel=1e-4)
    assert part[:, 1].sum() == pytest.approx(g, rel=1e-6, abs=1e-9)
    assert got["t"] == pytest.approx(float(line_search_rule(part[:, 0].sum(), part[:, 1].sum(), P)), rel=1e-6)
    assert got["t"] == pytest.approx(one["t"], rel=1e-5)
    np.testing.assert_allclose(got["f"], f + np.float32(got["t"]) * d_f, rtol=1e-4, atol=3e-5)
    np.testing.assert_allclose(got["f"], one["f"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(got["alpha"], one["alpha"], rtol=1e-5, atol=1e-6 * C)


def test_ws_select_one_pass_matches_model(K):
    rng = np.random.default_rng(3)
    n, C = 70000, 1.0  # 2 rows per selection thread
    X = rng.normal(size=(n, 4)).astype(np.float32)
    lines = rng.choice(n, size=150, replace=False)
    Xl = X[lines].astype(np.float64)
    gram = np.exp(-0.2 * ((Xl ** 2).sum(1)[:, None] + (X.astype(np.float64) ** 2).sum(1)[None, :]
                          - 2 * Xl @ X.T.astype(np.float64))).astype(np.float32)
    y = np.where(rng.random(n) < 0.5, 1.0, -1.0).astype(np.float32)
    a = rng.uniform(0, C, n).astype(np.float32)
    a[rng.random(n) < 0.5] = 0.0
    a[rng.random(n) < 0.1] = np.float32(C)
    f = rng.normal(size=n).astype(np.float32)
    coef = rng.normal(scale=0.2, size=150).astype(np.float32)
    got = K.ws_select(gram, f, a, y, np.zeros(n, np.float32), np.arange(150), coef, [150], C)
    G, rpt = got["G"], got["rpt"]
    assert rpt == 2
    want_f = f + gram.astype(np.float64).T @ coef.astype(np.float64)
    np.testing.assert_allclose(got["f"], want_f, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(got["alpha"], a)
    cand = np.asarray(got["cand"], dtype=np.uint64).reshape(G, 2, KC)[:, :, :KC1]  # one block: KC1 per side
    np.testing.assert_array_equal(cand, candidates_model(got["f"], a, y, C, G, rpt, nc=KC1))


@pytest.mark.parametrize("clip", ["independent", "box"])
def test_ws_solve_second_order_matches_model(K, clip):
    """WSS2 (ws_wss = 2): hi by the reference's first-order rule, lo by the
    largest (f_lo - b_hi)^2 / eta(hi, lo); the first steps match the numpy
    model exactly, and the full solve ends on the same first-order stop test."""
    rng = np.random.default_rng(91 + (clip == "box"))
    C, q, q_max = 2.0, 120, 192
    Kq, f, a, y = sub_problem(rng, q, C, gamma=0.05)  # coupled rows: the choice differs from first order
    bh, bl = extremes(f, a, y, C)
    eps_floor = np.float32(3e-4)
    eps_in = max(eps_floor, np.float32(np.float32(0.3 * np.float32(0.5)) * np.float32(bl - bh)))
    Kp, fp, ap, yp = padded_block(Kq, f, a, y, q_max)
    box = clip == "box"
    for cap in (1, 3, 8):
        got = K.ws_solve(Kp, fp, ap, yp, [q], q_max, C, clip=clip, eps_floor=eps_floor, b_hi=bh, b_lo=bl,
                         inner_max=cap, wss=2)
        ref_a, ref_steps, _ = solve_model(Kq, f, a, y, C, box, eps_in, 1e-12, cap, w2=True)
        assert got["steps"] == [ref_steps]
        np.testing.assert_allclose(got["alpha"][:q], ref_a, rtol=2e-6, atol=2e-6 * C)
    first = solve_model(Kq, f, a, y, C, box, eps_in, 1e-12, 1, w2=False)[0]
    second = solve_model(Kq, f, a, y, C, box, eps_in, 1e-12, 1, w2=True)[0]
    assert not np.array_equal(first, second)  # the case really exercises a different choice
    got = K.ws_solve(Kp, fp, ap, yp, [q], q_max, C, clip=clip, eps_floor=eps_floor, b_hi=bh, b_lo=bl,
                     inner_max=4 * q_max, wss=2)
    an = got["alpha"][:q]
    fn = f + Kq.astype(np.float64) @ ((an.astype(np.float64) - a) * y)
    if got["steps"][0] < 4 * q_max:
        bh2, bl2 = extremes(fn, an, y, C)
        assert bl2 <= bh2 + 2 * eps_in + 1e-4


@pytest.mark.parametrize("ks", [1, 3])
def test_ws_select_wide_pass1_matches_model(K, ks):
    """The wide pass 1 (ws_pass1_v4_kernel: 1024-column groups, four columns per
    thread, 16-B row loads, ks list slices): d_f, the d'Qd / g'd partials and f
    after pass 2 match the float64 model and the selection-geometry kernel;
    n not a multiple of 1024 (the last group is partial)."""
    rng = np.random.default_rng(70 + ks)
    n, C, q_max, P = 3000, 2.0, 96, 4
    gram, f, a_new, y, dal, ch = select_state(rng, n, C, 160)
    c = dal.astype(np.float64) * y
    d_f = gram.astype(np.float64).T @ c
    q = float(np.sum(c[ch] * d_f[ch]))
    g = -float(np.sum(c[ch] * f.astype(np.float64)[ch]))
    nab = [40] * P
    got = K.ws_select(gram, f, a_new, y, dal, ch, c[ch].astype(np.float32), nab, C, q_max=q_max, ks=ks, wide=True)
    ref = K.ws_select(gram, f, a_new, y, dal, ch, c[ch].astype(np.float32), nab, C, q_max=q_max, ks=ks)
    assert got["p1G"] == (n + 1023) // 1024
    part = np.asarray(got["part"]).reshape(got["p1G"] * ks, 2)
    assert part[:, 0].sum() == pytest.approx(q, rel=1e-4)
    assert part[:, 1].sum() == pytest.approx(g, rel=1e-6, abs=1e-9)
    if ks == 1:
        np.testing.assert_allclose(got["dfs"], d_f, rtol=1e-4, atol=2e-5)
    assert got["t"] == pytest.approx(float(line_search_rule(part[:, 0].sum(), part[:, 1].sum(), P)), rel=1e-6)
    assert got["t"] == pytest.approx(ref["t"], rel=1e-5)
    np.testing.assert_allclose(got["f"], f + np.float32(got["t"]) * d_f, rtol=1e-4, atol=3e-5)
    np.testing.assert_allclose(got["f"], ref["f"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(got["alpha"], ref["alpha"], rtol=1e-5, atol=1e-6 * C)
    G, rpt = got["G"], got["rpt"]
    cand = np.asarray(got["cand"], dtype=np.uint64).reshape(G, 2, KC)
    np.testing.assert_array_equal(cand, candidates_model(got["f"], got["alpha"], y, C, G, rpt))
