"""Interleaved timing of bnn_gemm_fp6 variants on one shape (MI355X_MICROARCH rule: A/B in one
process, rounds interleaved, the clock settled first).  Timing-only diagnostic variants (9x) give
wrong results; the others are checked equal to the first.

    python tools/fp6_diag.py M N K ROUNDS REPS VARIANT...
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402


def main():
    M, N, K, rounds, reps = (int(a) for a in sys.argv[1:6])
    variants = [int(a) for a in sys.argv[6:]]
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda")
    w = torch.randint(-1, 2, (N, K), device="cuda").float()
    op = BF.quant6_rows(x)
    w4, _ = BF.sign_pack_fp4(w)
    del x, w
    C = torch.empty((M, N), device="cuda")
    ops = 2.0 * M * N * K
    ref = None
    for v in variants:
        if v >= 90:
            continue
        L.call("bnn_gemm_fp6_set_variant", v)
        BF.gemm_fp6(op, w4, N, out=C)
        if ref is None:
            ref = C.clone()
        else:
            print(f"v{v} equal to v{variants[0]}: {torch.equal(C, ref)}", flush=True)
    # settle the clock under load (~2 s)
    L.call("bnn_gemm_fp6_set_variant", variants[0])
    for _ in range(max(1, int(2000 / max(1.0, ops / 4.7e12 * 1e3)))):
        BF.gemm_fp6(op, w4, N, out=C)
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for v in variants:
            L.call("bnn_gemm_fp6_set_variant", v)
            BF.gemm_fp6(op, w4, N, out=C)
            s.record()
            for _ in range(reps):
                BF.gemm_fp6(op, w4, N, out=C)
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / reps)
    L.call("bnn_gemm_fp6_set_variant", -1)
    for v in variants:
        med = statistics.median(times[v])
        name = L.lib().bnn_gemm_fp6_kernel(M, N).decode() if False else ""
        print(f"v{v:3d} {M}x{N}x{K}: median {med:8.3f} ms  min {min(times[v]):8.3f}  "
              f"{ops / med / 1e12:7.1f} TOPS alg  {4 * ops / med / 1e12 / 10066.3 * 1e3:.3f} of the 4-pass peak",
              flush=True)


if __name__ == "__main__":
    main()
