"""Run one GEMM shape with one kernel variant REPS times (a target for rocprofv3 PMC passes).

    python tools/gemm_one.py fp6|i8 VARIANT M N K [REPS]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402


def main():
    kind, v, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda")
    w = torch.randint(-1, 2, (N, K), device="cuda").float()
    if kind == "fp6":
        L.call("bnn_gemm_fp6_set_variant", v)
        op = BF.quant6_rows(x)
        w4, _ = BF.sign_pack_fp4(w)
        C = BF.gemm_fp6(op, w4, N)
        run = lambda: BF.gemm_fp6(op, w4, N, out=C)  # noqa: E731
    else:
        L.call("bnn_gemm_set_variant", v)
        d, sc = BF.quant_rows(x)
        wq, _ = BF.sign_pack(w, True, False)
        C = BF.gemm_i8(d, 3, wq, 1, M, N, a_scale=sc)
        run = lambda: BF.gemm_i8(d, 3, wq, 1, M, N, a_scale=sc, out=C)  # noqa: E731
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        run()
    e.record()
    torch.cuda.synchronize()
    print(f"{kind} v{v} {M}x{N}x{K}: {s.elapsed_time(e) / reps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
