"""Time every bnn_gemm_fp6 variant on the wide-MLP backward shapes (dX: 65536 x 8192 x 8192;
dW: 8192 x 8192 x 65536) and the first layer's forward (65536 x 8192 x 784), against the int8
3-digit kernel the default table picks for the same GEMM."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    torch.manual_seed(0)
    shapes = [("dX", 65536, 8192, 8192), ("dW", 8192, 8192, 65536), ("fc1 fwd", 65536, 8192, 784)]
    for tag, M, N, K in shapes:
        x = torch.randn(M, K, device="cuda")
        w = torch.randint(-1, 2, (N, K), device="cuda").float()
        op = BF.quant6_rows(x)
        w4, _ = BF.sign_pack_fp4(w)
        ops = 2.0 * M * N * K
        tq = timeit(lambda: BF.quant6_rows(x), reps)
        print(f"{tag}: quant6_rows {tq:.3f} ms ({(4 * M * K + 3 * M * K) / tq / 1e6:.0f} GB/s)", flush=True)
        ref = None
        last = None
        for v in range(8):
            L.call("bnn_gemm_fp6_set_variant", v)
            name = L.lib().bnn_gemm_fp6_kernel(M, N).decode()
            if name == last:
                continue
            last = name
            C = BF.gemm_fp6(op, w4, N)
            if ref is None:
                ref = C.clone()
            same = torch.equal(C, ref)
            ms = timeit(lambda: BF.gemm_fp6(op, w4, N, out=C), reps)
            print(f"  {name:34s} {ms:8.3f} ms  {ops / ms / 1e9:8.1f} TOPS alg  frac(int8 peak) {ops / ms / 1e9 / 5033.2:.3f}"
                  f"  frac(fp6 4-pass) {4 * ops / ms / 1e9 / 10066.3:.3f}  same={same}", flush=True)
        L.call("bnn_gemm_fp6_set_variant", -1)
        d, sc = BF.quant_rows(x)
        wq, _ = BF.sign_pack(w, True, False)
        ms = timeit(lambda: BF.gemm_i8(d, 3, wq, 1, M, N, a_scale=sc), reps)
        print(f"  int8 3-digit {BF.gemm_kernel_name(3, 1, M, N, d.shape[-1]):40s} {ms:8.3f} ms  {ops / ms / 1e9:8.1f} TOPS alg",
              flush=True)
        del x, w, op, w4, d, sc, wq, C, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
