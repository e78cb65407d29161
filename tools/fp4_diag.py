"""Time the wide step's fc3 forward GEMM (bnn_gemm_fp4_i16: ternary x ternary FP4, int16 output) at
M x N x K with the library BNN_LIB points at -- for timing-only builds (GEMM_DIAG_NOMAIN /
GEMM_DIAG_NOSTORE) against the real one.

    BNN_LIB=ab/<tag>/libbnn.so python tools/fp4_diag.py [M N K]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import functional as BF  # noqa: E402


def main():
    M, N, K = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (65536, 8192, 8192)
    torch.manual_seed(0)
    a4, _ = BF.sign_pack_fp4(torch.randn(M, K, device="cuda"))
    b4, _ = BF.sign_pack_fp4(torch.randn(N, K, device="cuda"))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        BF.gemm_fp4_i16(a4, b4, M, N)
    torch.cuda.synchronize()
    s.record()
    for _ in range(10):
        BF.gemm_fp4_i16(a4, b4, M, N)
    e.record()
    torch.cuda.synchronize()
    print(f"{os.environ.get('BNN_LIB', 'tree')}: {s.elapsed_time(e) / 10 * 1e3:.0f} us per launch", flush=True)


if __name__ == "__main__":
    main()
