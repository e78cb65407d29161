"""Does the (1,1) int8 GEMM at the pixel layer's shape (65536 x 8192 x 832) lose time to its fp32
output's power-of-two row stride?  Times ldc = 8192 (contiguous) against padded row strides.

    python tools/pix_ldc_probe.py
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
    M, N, K = 65536, 8192, 832
    A = torch.randint(-128, 128, (M, K), device="cuda", dtype=torch.int8)
    B = torch.randint(-1, 2, (N, K), device="cuda", dtype=torch.int8)
    for rnd in range(2):
        for pad in (0, 32, 64, 128, 256):
            ldc = N + pad
            C = torch.empty(M, ldc, device="cuda")
            t = timeit(lambda: L.call("bnn_gemm_i8_affine", L.ptr(A), K, 0, 1, L.ptr(B), K, 0, 1, None, None, None,
                                      None, None, 0.0, L.ptr(C), ldc, M, N, K, L.stream()))
            print(f"round {rnd} ldc {ldc}: {t:.0f} us", flush=True)
            del C


if __name__ == "__main__":
    main()
