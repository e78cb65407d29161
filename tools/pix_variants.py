"""Time the u8-pixel fc1 GEMM (bnn_gemm_i8_affine, digits (1,1), K = 832) of the wide step with each
int8 kernel variant, interleaved rounds in one process.

    python tools/pix_variants.py [M N]
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
    C = torch.empty(M, N, device="cuda")
    Kp = q.shape[1]
    ref = None
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for rnd in range(3):
        for v in (1, 2, 4, 5, 0):
            L.call("bnn_gemm_set_variant", v)
            run = lambda: L.call("bnn_gemm_i8_affine", L.ptr(q), Kp, 0, 1, L.ptr(wq), Kp, 0, 1, None, L.ptr(bs),  # noqa: E731
                                 L.ptr(b), None, L.ptr(R), 128.0, L.ptr(C), N, M, N, Kp, L.stream())
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = C.clone()
            ok = torch.equal(C, ref)
            s.record()
            for _ in range(5):
                run()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(v, []).append(s.elapsed_time(e) / 5)
            name = L.lib().bnn_gemm_i8_kernel(1, 1, M, N, Kp).decode()
            print(f"round {rnd} v{v} {name}: {s.elapsed_time(e) / 5 * 1e3:.0f} us equal={ok}", flush=True)
    L.call("bnn_gemm_set_variant", -1)
    for v, t in res.items():
        print(f"v{v}: min {min(t) * 1e3:.0f} us")


if __name__ == "__main__":
    main()
