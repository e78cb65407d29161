"""Is the pixel-layer GEMM (65536 x 8192 x 832, int8 (1,1), fp32 out) faster as column slices
(2 x 4096 or 4 x 2048 columns into the same C, ldc = 8192) than as one launch?

    python tools/pix_split_probe.py
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
    C = torch.empty(M, N, device="cuda")
    ref = None
    for rnd in range(2):
      for raster in (0, 1):
        L.call("bnn_gemm_set_raster", raster)
        for parts in (1, 2):
            ns = N // parts  # noqa: E111

            def run():
                for j in range(parts):
                    L.call("bnn_gemm_i8_affine", L.ptr(A), K, 0, 1, L.ptr(B[j * ns:]), K, 0, 1, None, None, None,
                           None, None, 0.0, L.ptr(C[:, j * ns:]), N, M, ns, K, L.stream())
            t = timeit(run)
            if ref is None:
                ref = C.clone()
            print(f"round {rnd} raster {raster} {parts} slice(s) of {ns} columns: {t:.0f} us equal={torch.equal(C, ref)}",
                  flush=True)


if __name__ == "__main__":
    main()
