"""Time the benched fc1 pixel GEMM (bnn_gemm_i8_affine_bnstats: u8 pixels x ternary W1, K = 832, fp32
z1 + bn1's forward statistics) at the wide step's shape with the library BNN_LIB points at -- for
timing-only builds (GEMM_DIAG_NOMAIN / GEMM_DIAG_NOSTORE) against the real one.

    BNN_LIB=ab/<tag>/libbnn.so python tools/pix_diag.py [M N]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    torch.manual_seed(0)
    u = torch.randint(0, 256, (M, 784), device="cuda").to(torch.uint8)
    w = torch.randn(N, 784, device="cuda")
    b = torch.randn(N, device="cuda")
    q, _ = BF.pixels_pack(u, want_q=True, want_qt=False)
    wq, _ = BF.packed_weight(w, "i8", True, False, False)
    R = BF.row_sums(wq, 784)
    bs = BF._const_vec(1 / 255.0, N, "cuda")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        BF._pixels_fwd_with_stats(q, wq, M, N, 784, bs, b, R, 128.0)
    torch.cuda.synchronize()
    s.record()
    for _ in range(10):
        BF._pixels_fwd_with_stats(q, wq, M, N, 784, bs, b, R, 128.0)
    e.record()
    torch.cuda.synchronize()
    print(f"{os.environ.get('BNN_LIB', 'tree')}: {s.elapsed_time(e) / 10 * 1e3:.0f} us per launch", flush=True)


if __name__ == "__main__":
    main()
