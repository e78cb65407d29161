"""Concurrency probe (wide step shapes, random data): does an HBM/latency-bound BatchNorm backward
chain (bnn_bn_bwd_q6 on z16, the bn2 pass of the wide step) overlap an MFMA-bound FP6 weight-gradient
GEMM (dW: 8192 x 8192 x 65536) when the two run on separate streams?  Times each alone, both
serialised on one stream, and both on two streams (HIP events, medians of 5).

    python tools/overlap_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))


def main():
    from bnn_amd import functional as F
    dev = torch.device("cuda")
    M, C = 65536, 8192
    g = torch.Generator(device=dev).manual_seed(3)
    # dW = dz^T . X_b: A = column digits of dz [C, M], B = FP4 X_b^T panels
    dz = torch.randn(M, C, generator=g, device=dev)
    A, _ = F.quant6_cols_t(dz)
    xb = torch.randint(-1, 2, (C, M), generator=g, device=dev).float()
    B4, _ = F.sign_pack_fp4(xb)
    P = F.fp4_panels(B4, C, M)
    del xb, B4
    # the bn2 chain input: z16 + bias, dy fp32
    z16 = torch.randint(-400, 400, (M, C), generator=g, device=dev).to(torch.int16)
    bias = torch.randn(C, generator=g, device=dev)
    dy = torch.randn(M, C, generator=g, device=dev)
    gw, gb = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    z = z16.float() + bias
    mean, invstd, mlo = z.mean(0), (z.var(0, unbiased=False) + 1e-5).rsqrt(), torch.zeros(C, device=dev)
    del z
    dw = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)

    def gemm():
        F.gemm_fp6(A, None, C, k_true=M, panels=P, panel_ks=M // 64)

    def chain():
        F._bn_bwd_q6(None, dy, M, C, gw, gb, mean, invstd, mlo, True, 0.0, 0, dw, db, F._bn_ws(M, C, dev),
                     "bn_bwd_q6", z16=(z16, bias))

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        ts = []
        for _ in range(6):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts[1:])[2]

    def both_serial():
        gemm()
        chain()

    def both_conc():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            gemm()
        with torch.cuda.stream(s2):
            chain()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    for name, fn in (("gemm alone", gemm), ("chain alone", chain), ("serial", both_serial), ("two streams", both_conc)):
        print(f"{name:12s} {timed(fn):8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
