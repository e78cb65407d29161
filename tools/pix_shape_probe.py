"""Probe what bounds the (1,1) int8 GEMM at the pixel layer's short K: time M x N x K for K = 832,
1664, 3328 and N = 8192 / 4096 (default variant, fp32 output), and a plain fill of the same C.

    python tools/pix_shape_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402


def timeit(fn, reps=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M = 65536
    for N in (8192, 4096):
        C = torch.empty(M, N, device="cuda")
        print(f"fill {M}x{N} fp32: {timeit(lambda: C.fill_(1.0)):.0f} us", flush=True)
        for K in (832, 1664, 3328):
            A = torch.randint(-128, 128, (M, K), device="cuda", dtype=torch.int8)
            B = torch.randint(-1, 2, (N, K), device="cuda", dtype=torch.int8)
            name = L.lib().bnn_gemm_i8_kernel(1, 1, M, N, K).decode()
            t = timeit(lambda: L.call("bnn_gemm_i8_affine", L.ptr(A), K, 0, 1, L.ptr(B), K, 0, 1, None, None, None,
                                      None, None, 0.0, L.ptr(C), N, M, N, K, L.stream()))
            print(f"gemm {M}x{N}x{K} {name}: {t:.0f} us  ({2 * M * N * K / t / 1e6:.0f} TOPS)", flush=True)
            del A, B


if __name__ == "__main__":
    main()
