"""Time the first layer's pixel GEMMs (bnn_gemm_i8_affine) per kernel variant.

    python tools/px_sweep.py [--reps 5]
fc1 forward: (1,1) M=65536 N=8192 over K = 832 / 896 (pixel rows padded to 64 / 128), with and
without the col_off term; dW1: (3,1) M=8192 N=784 K=65536 with row_off."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    M, N = 65536, 8192
    for K in (832, 896):
        A = torch.randint(-128, 128, (M, K), generator=g, device="cuda", dtype=torch.int8)
        B = torch.randint(-1, 2, (N, K), generator=g, device="cuda", dtype=torch.int8)
        co = torch.randint(-784, 785, (N,), generator=g, device="cuda", dtype=torch.int64)
        bs = torch.full((N,), 1 / 255, device="cuda")
        for v in list(range(10)) + [-1]:
            L.call("bnn_gemm_set_variant", v)
            name = BF.gemm_kernel_name(1, 1, M, N, K)
            t0 = timeit(lambda: BF.gemm_i8(A, 1, B, 1, M, N), args.reps)
            t1 = timeit(lambda: BF.gemm_i8_affine(A, 1, B, 1, M, N, b_scale=bs, col_off=co, off_mul=128.0), args.reps)
            print(f"fc1 K={K} v{v} {name}: plain {t0:.3f} ms, affine {t1:.3f} ms", flush=True)
    M, N, K = 8192, 784, 65536
    A = torch.randint(-128, 128, (3, M, K), generator=g, device="cuda", dtype=torch.int8)
    B = torch.randint(-128, 128, (896, K), generator=g, device="cuda", dtype=torch.int8)[:N]
    ro = torch.randint(-2 ** 30, 2 ** 30, (M,), generator=g, device="cuda", dtype=torch.int64)
    sc = torch.full((M,), 2.0 ** -30, device="cuda")
    for v in list(range(10)) + [-1]:
        L.call("bnn_gemm_set_variant", v)
        name = BF.gemm_kernel_name(3, 1, M, N, K)
        t1 = timeit(lambda: BF.gemm_i8_affine(A, 3, B, 1, M, N, a_scale=sc, row_off=ro, off_mul=128.0), args.reps)
        print(f"dW1 v{v} {name}: {t1:.3f} ms", flush=True)
    L.call("bnn_gemm_set_variant", -1)


if __name__ == "__main__":
    main()
