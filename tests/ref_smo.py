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
            if y[ih] != y[il]:
                L, H = max(0.0, a[il] - a[ih]), min(C, C + a[il] - a[ih])
            else:
                L, H = max(0.0, a[il] + a[ih] - C), min(C, a[il] + a[ih])
            aln = min(max(aln, L), H)
            ahn = min(max(a[ih] + s * (a[il] - aln), 0.0), C)
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
