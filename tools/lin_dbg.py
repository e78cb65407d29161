"""Quick check of bnn_linear_nsmall_fwd against float64 at a few shapes (prints the max error).

    python tools/lin_dbg.py
"""
import sys, os
sys.path.insert(0, "distributed-mnist-bnns_amd")
import torch
from bnn_amd import _lib as L
for M, K, N in [(16, 256, 10), (32, 1568, 10), (4096, 1568, 10)]:
    x = torch.randn(M, K, device="cuda"); w = torch.randn(N, K, device="cuda") * 0.05; b = torch.randn(N, device="cuda")
    y = torch.full((M, N), 7.0, device="cuda")
    rc = L.lib().bnn_linear_nsmall_fwd(L.ptr(x), M, K, L.ptr(w), L.ptr(b), N, L.ptr(y), L.stream())
    torch.cuda.synchronize()
    ref = x.double() @ w.double().T + b.double()
    print(M, K, N, "rc", rc, "maxerr", (y.double() - ref).abs().max().item(), "y00", y[0, :3].tolist(), "ref", ref[0, :3].tolist(), flush=True)
