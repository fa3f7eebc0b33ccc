"""Plain numpy model of the reference algorithm (svmTrainMain.cpp:235-310 +
svmTrain.cu:41-137) used as an independent oracle in the CPU tests.

float64 throughout; ties go to the lowest index (the native solvers' rule).
"""
import numpy as np


def rbf_gram(X, gamma):
    X = X.astype(np.float64)
    sq = (X * X).sum(1)
    d2 = np.maximum(sq[:, None] + sq[None, :] - 2.0 * X @ X.T, 0.0)
    return np.exp(-gamma * d2)


def smo_reference(X, y, C, gamma, eps=1e-3, max_iter=150000, clip="independent"):
    y = np.where(np.asarray(y) > 0, 1.0, -1.0)
    n = len(y)
    K = rbf_gram(X, gamma)
    a = np.zeros(n)
    f = -y.copy()
    it = 0
    while True:
        up = ((a == 0) & (y == 1)) | ((a == C) & (y != 1)) | ((a > 0) & (a < C))
        lo = ((a == 0) & (y != 1)) | ((a == C) & (y == 1)) | ((a > 0) & (a < C))
        fu = np.where(up, f, np.inf)
        fl = np.where(lo, -f, np.inf)
        ih, il = int(np.argmin(fu)), int(np.argmin(fl))  # argmin: first (lowest) index on ties
        bh, bl = f[ih], f[il]
        eta = max(2.0 - 2.0 * K[ih, il], 1e-12)
        s = y[il] * y[ih]
        aln = a[il] + y[il] * (bh - bl) / eta
        if clip == "box" and ih != il:
            # joint box; when alpha_lo lands on a bound that comes from alpha_hi's
            # own bound, alpha_hi takes that bound exactly (in exact arithmetic it
            # would): otherwise round-off leaves it a hair inside [0, C] and the
            # same pair is selected forever with a zero-length step (LIBSVM snaps
            # the same way)
            if y[ih] != y[il]:
                dl = a[il] - a[ih]
                L, hL = (dl, 0.0) if dl > 0 else (0.0, None)
                H, hH = (C + dl, C) if dl < 0 else (C, None)
            else:
                sm = a[il] + a[ih]
                L, hL = (sm - C, C) if sm > C else (0.0, None)
                H, hH = (sm, 0.0) if sm < C else (C, None)
            snap = None
            if aln <= L:
                aln, snap = L, hL
            elif aln >= H:
                aln, snap = H, hH
            ahn = snap if snap is not None else min(max(a[ih] + s * (a[il] - aln), 0.0), C)
        else:
            ahn = a[ih] + s * (a[il] - aln)
            aln, ahn = min(max(aln, 0.0), C), min(max(ahn, 0.0), C)
        dh, dl = ahn - a[ih], aln - a[il]
        a[il] = aln
        a[ih] = ahn
        f += dh * y[ih] * K[ih] + dl * y[il] * K[il]
        it += 1
        if not (bl > bh + 2 * eps) or it >= max_iter:
            break
    return a, (bl + bh) / 2.0, it


def decision(Xtr, ytr, alpha, b, gamma, Xte):
    Xtr = Xtr.astype(np.float64)
    Xte = Xte.astype(np.float64)
    d2 = np.maximum((Xte * Xte).sum(1)[:, None] + (Xtr * Xtr).sum(1)[None, :] - 2 * Xte @ Xtr.T, 0)
    return np.exp(-gamma * d2) @ (alpha * np.where(ytr > 0, 1.0, -1.0)) - b
