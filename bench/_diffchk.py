import sys, os, torch, numpy as np
sys.path.insert(0, os.getcwd())
from dpsvm_amd._native import load
from dpsvm_amd.utils.datasets import synthetic
C = load()
for n in (5000, 60000):
    X, _ = synthetic("mnist", n=n, seed=1)
    d = X.shape[1]; dp = (d + 15) // 16 * 16
    rows = (n + 255) // 256 * 256 + 512
    x = torch.zeros(rows, dp, device="cuda"); x[:n, :d] = torch.from_numpy(X).cuda()
    s = torch.cuda.current_stream().cuda_stream
    xsq = torch.zeros(rows, device="cuda"); C.k_row_sqnorm(x.data_ptr(), rows, dp, dp, xsq.data_ptr(), s)
    for sym, nb in ((True, n), (False, (n + 7) // 8)):
        ld = (nb + 127) // 128 * 128
        outs = {}
        for v in (8, 11):
            o = torch.full((n, ld), -7.0, device="cuda")
            C.k_set_split_gemm_variant(v)
            C.k_rbf_gram_split(x.data_ptr(), xsq.data_ptr(), n, x.data_ptr(), xsq.data_ptr(), nb, dp, 0.25, o.data_ptr(), ld, sym, s)
            torch.cuda.synchronize(); outs[v] = o
        C.k_set_split_gemm_variant(0)
        a, b = outs[8], outs[11]
        dif = (a != b)
        nd = int(dif.sum())
        print(n, sym, "ndiff", nd, flush=True)
        if nd:
            idx = dif.nonzero()[:10].cpu().numpy()
            torch.set_printoptions(precision=3, linewidth=200, sci_mode=True)
            print("v8\n", a[:6, :6].cpu()); print("v11\n", b[:6, :6].cpu())
            print("v8 rows 64-66\n", a[64:67, :6].cpu()); print("v11 rows 64-66\n", b[64:67, :6].cpu())
            rr = dif.nonzero()
            print("  rows", int(rr[:, 0].min()), int(rr[:, 0].max()), "cols", int(rr[:, 1].min()), int(rr[:, 1].max()),
                  "maxabs", float((a - b).abs().max()), "valid-region diffs", int(dif[:, :nb].sum()))
        del outs, a, b; torch.cuda.empty_cache()
