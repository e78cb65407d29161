"""Interleaved A/B of the FP4 ternary GEMM's tile forms on the wide-MLP forward shape (65536 x 8192
x 8192, random ternary operands, fp32 output, one process): the default 256 x 256 tile (one
workgroup per CU) against two-workgroups-per-CU forms (gemm_fp4_h_k, bnn_gemm.hip variants 37-39).
Every form's C is checked bit-identical to the default's (exact integer sums).

    python tools/fp4_half_ab.py "6 7 8 9" [rounds] [reps]      (bnn_gemm_set_variant: FP4 id = 30 + v)
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402


def main():
    vs = [int(v) for v in sys.argv[1].split()]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    M, N, K = 65536, 8192, 8192
    g = torch.Generator(device="cuda").manual_seed(0)
    x4, _ = BF.sign_pack_fp4(torch.randint(-1, 2, (M, K), device="cuda", generator=g).float())
    w4, _ = BF.sign_pack_fp4(torch.randint(-1, 2, (N, K), device="cuda", generator=g).float())
    C = torch.empty(M, N, device="cuda")
    ops = 2.0 * M * N * K

    def run(v):
        L.call("bnn_gemm_set_variant", v)
        L.call("bnn_gemm_fp4", L.ptr(x4), x4.shape[1], L.ptr(w4), w4.shape[1], None, L.ptr(C), N, M, N, K // 2,
               L.stream())

    ref = None
    for v in vs:
        run(v)
        torch.cuda.synchronize()
        if ref is None:
            ref = C.clone()
        else:
            assert torch.equal(C, ref), v
    times = {v: [] for v in vs}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for v in vs:
            run(v)
            s.record()
            for _ in range(reps):
                run(v)
            e.record()
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / reps)
    for v in vs:
        med = statistics.median(times[v])
        print(f"FP4 variant {30 + v}: median {med:7.3f} ms  min {min(times[v]):7.3f}  "
              f"{ops / med / 1e9:7.1f} TOPS ({ops / med / 1e12 / 10066.3 * 1e3:.3f} of peak)", flush=True)
    L.call("bnn_gemm_set_variant", -1)


if __name__ == "__main__":
    main()
