"""Interleaved A/B timing of bnn_gemm_fp6 variants on the wide-MLP backward shapes, random data,
one process (cdna_hip_programming.md §5.4 rule 24): ROUNDS rounds x every variant, median and min.

    python tools/fp6_variants.py "7 10 12" [rounds] [reps]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1].split()]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    torch.manual_seed(0)
    shapes = [("dX", 65536, 8192, 8192), ("dW", 8192, 8192, 65536)]
    for tag, M, N, K in shapes:
        x = torch.randn(M, K, device="cuda")
        w = torch.randint(-1, 2, (N, K), device="cuda").float()
        op = BF.quant6_rows(x)
        w4, _ = BF.sign_pack_fp4(w)
        del x, w
        ops = 2.0 * M * N * K
        C = torch.empty(M, N, device="cuda")
        ref = None
        times = {v: [] for v in variants}
        names = {}
        for v in variants:
            L.call("bnn_gemm_fp6_set_variant", v)
            names[v] = L.lib().bnn_gemm_fp6_kernel(M, N).decode()
            BF.gemm_fp6(op, w4, N, out=C)
            torch.cuda.synchronize()
            if ref is None:
                ref = C.clone()
            elif v < 90:
                assert torch.equal(C, ref), (tag, v)
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
        for v in variants:
            med, mn = statistics.median(times[v]), min(times[v])
            print(f"{tag} v{v:<3d} {names[v]:44s} median {med:7.3f} ms  min {mn:7.3f}  "
                  f"{ops / med / 1e9:7.1f} TOPS alg  passes {4 * ops / med / 1e12:5.2f} POPS", flush=True)
        L.call("bnn_gemm_fp6_set_variant", -1)
        del op, w4, C, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
