"""Interleaved A/B of the FP6 backward GEMM's tile forms on the wide-MLP shapes (random data, one
process): the default 128 x 512 tile (one workgroup per CU) against the half-tile form (64 x 512
tiles, two workgroups per CU, bnn_gemm_fp6_set_half) at several first-round staggers.  dX carries
the residual plane (as the wide step's dX launches), dW the four planes.  Every form's C is checked
bit-identical to the default's.

    python tools/fp6_half_ab.py "0:0 1:0 1:65 1:130" [rounds] [reps]     (mode:stagger_us[:group]; dW uses mode 2)
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-mnist-bnns_amd"))
import torch  # noqa: E402

from bnn_amd import _lib as L  # noqa: E402
from bnn_amd import functional as BF  # noqa: E402


def main():
    cfgs = [(int(t[0]), float(t[1]), int(t[2]) if len(t) > 2 else 0) for t in (c.split(":") for c in sys.argv[1].split())]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    torch.manual_seed(0)
    for tag, M, N, K, res in (("dX+res", 65536, 8192, 8192, True), ("dW", 8192, 8192, 65536, False)):
        BF.FP6_RES = res
        x = torch.randn(M, K, device="cuda")
        op = BF.quant6_rows(x)
        del x
        w = torch.randint(-1, 2, (N, K), device="cuda").float()
        w4, _ = BF.sign_pack_fp4(w)
        del w
        panels = BF.fp4_panels(w4, N, K)
        C = torch.empty(M, N, device="cuda")
        ops = 2.0 * M * N * K
        ref = None
        times = {c: [] for c in cfgs}

        def run(c):
            mode, st, grp = c
            L.call("bnn_gemm_fp6_set_half", (mode if res or mode == 0 else 2), st)
            L.call("bnn_gemm_fp6_set_half_group", grp)
            BF.gemm_fp6(op, None, N, out=C, panels=panels, panel_ks=K // 64)

        for c in cfgs:
            run(c)
            torch.cuda.synchronize()
            if ref is None:
                ref = C.clone()
            else:
                assert torch.equal(C, ref), (tag, c, float((C - ref).abs().max()))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(rounds):
            for c in cfgs:
                run(c)
                s.record()
                for _ in range(reps):
                    run(c)
                e.record()
                torch.cuda.synchronize()
                times[c].append(s.elapsed_time(e) / reps)
        for c in cfgs:
            med, mn = statistics.median(times[c]), min(times[c])
            print(f"{tag:7s} mode {c[0]} stagger {c[1]:6.1f} us group {c[2]}: median {med:7.3f} ms  min {mn:7.3f}  "
                  f"{ops / med / 1e9:7.1f} TOPS alg", flush=True)
        L.call("bnn_gemm_fp6_set_half", 1, 0.0)
        L.call("bnn_gemm_fp6_set_half_group", 0)
        del op, w4, panels, C, ref
        torch.cuda.empty_cache()
    BF.FP6_RES = True


if __name__ == "__main__":
    main()
